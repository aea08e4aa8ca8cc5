set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r05_final_pytest_gpu_all.log 2>&1; rc=$?
tail -3 gpurun_out/r05_final_pytest_gpu_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_final_smoke2.log 2>&1; rc=$?
tail -3 gpurun_out/r05_final_smoke2.log
exit $rc
