set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_w4_gpu.py tests/test_w4p_gpu.py tests/test_split_gpu.py tests/test_persistent_gpu.py tests/test_fullsize_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_mix.log 2>&1 || { tail -30 gpurun_out/r05_pytest_mix.log; exit 1; }
tail -2 gpurun_out/r05_pytest_mix.log
AB="timeout -k 10 300 python flash-attention-cuda_amd/tools/ab.py --configs auto --libs ,nomix"
O=gpurun_out/r05_ab_mix.jsonl
$AB --seq 4096 --batch 64 --causal --rounds 9 --iters 10 > $O &&
$AB --seq 8192 --causal --rounds 9 --iters 20 >> $O &&
$AB --seq 8192 --rounds 9 --iters 20 >> $O &&
$AB --seq 1024 --causal --rounds 9 --iters 40 >> $O &&
$AB --seq 2048 --causal --rounds 9 --iters 40 >> $O &&
$AB --seq 4096 --batch 64 --causal --rounds 7 --iters 10 --dtype bf16 >> $O || exit 1
cat $O
