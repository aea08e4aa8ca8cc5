set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_w4_gpu.py -k second_item_chunk -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_chunk.log 2>&1 || { tail -30 gpurun_out/pytest_chunk.log; exit 1; }
tail -6 gpurun_out/pytest_chunk.log
VAR=dma bash flash-attention-cuda_amd/tools/run_var_ab.sh
