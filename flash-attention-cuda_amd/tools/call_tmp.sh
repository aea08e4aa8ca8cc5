set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_w4_gpu.py tests/test_d64_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_d64dma.log 2>&1 || { tail -30 gpurun_out/r05_pytest_d64dma.log; exit 1; }
tail -2 gpurun_out/r05_pytest_d64dma.log
AB="timeout -k 10 300 python flash-attention-cuda_amd/tools/ab.py --configs auto --libs ,prev --head-dim 64"
O=gpurun_out/r05_ab_d64dma.jsonl
$AB --seq 4096 --batch 64 --causal --rounds 9 --iters 10 > $O &&
$AB --seq 8192 --causal --rounds 9 --iters 20 >> $O &&
$AB --seq 8192 --rounds 9 --iters 20 >> $O &&
$AB --seq 16384 --causal --rounds 5 --iters 10 >> $O &&
$AB --seq 4096 --batch 64 --causal --rounds 7 --iters 10 --dtype bf16 >> $O || exit 1
cat $O
