set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_w4p_gpu.py tests/test_capi.py -m gpu -x -v -k "dispatched_long_heads" --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_w4p_d64_long.log 2>&1; rc=$?; tail -8 gpurun_out/r05_pytest_w4p_d64_long.log; exit $rc
