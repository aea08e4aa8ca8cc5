set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_w4_pool_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_pool.log 2>&1 || { tail -40 gpurun_out/r05_pytest_pool.log; exit 1; }
tail -3 gpurun_out/r05_pytest_pool.log
AB="timeout -k 10 300 python flash-attention-cuda_amd/tools/ab.py --configs auto,static"
O=gpurun_out/r05_ab_pool.jsonl
$AB --seq 4096 --batch 64 --causal --rounds 9 --iters 10 > $O &&
$AB --seq 4096 --batch 32 --causal --rounds 9 --iters 10 >> $O &&
$AB --seq 8192 --batch 16 --rounds 7 --iters 10 >> $O &&
$AB --seq 4096 --batch 64 --causal --rounds 7 --iters 10 --head-dim 64 >> $O || exit 1
cat $O
cd flash-attention-cuda_amd
timeout -k 10 300 python tools/w4_tail.py --seq 4096 --batch 64 --causal > ../gpurun_out/r05_w4_tail_pool.jsonl && cat ../gpurun_out/r05_w4_tail_pool.jsonl | cut -c1-600
