#!/bin/bash
# un-instrumented workgroup cycles (FA_STAMPS build: start/end records only) -> cycles per tile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}/flash-attention-cuda_amd"
timeout -k 10 120 python tools/clock_check.py --batch 1 --seq 8192 2>&1 | grep -v amdgpu.ids &&
timeout -k 10 120 python tools/clock_check.py --batch 1 --seq 8192 --causal 2>&1 | grep -v amdgpu.ids &&
timeout -k 10 120 python tools/clock_check.py --batch 64 --seq 4096 --causal 2>&1 | grep -v amdgpu.ids
