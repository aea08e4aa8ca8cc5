set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dispatch_sweep_gpu.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_dispatch_sweep.log 2>&1; rc=$?
tail -4 gpurun_out/r05_pytest_dispatch_sweep.log
exit $rc
