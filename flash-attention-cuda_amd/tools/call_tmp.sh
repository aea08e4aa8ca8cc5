#!/bin/bash
# the new seeded random-shape W4 parity tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 600 python -u -m pytest tests/test_w4_gpu.py -k random -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_random.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_random.log; exit $rc
