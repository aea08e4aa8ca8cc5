set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_w4_gpu.py -m gpu -x -q -k "d64_bf16" --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_d64_bf16.log 2>&1 || { tail -30 gpurun_out/r05_pytest_d64_bf16.log; exit 1; }
tail -2 gpurun_out/r05_pytest_d64_bf16.log
AB="timeout -k 10 400 python flash-attention-cuda_amd/tools/ab.py --configs static --libs ,eplines"
O=gpurun_out/r05_ab_seam_probes4.jsonl
$AB --seq 4096 --batch 64 --causal --rounds 7 --iters 10 > $O &&
$AB --seq 8192 --causal --rounds 9 --iters 20 >> $O || exit 1
cat $O
AB2="timeout -k 10 400 python flash-attention-cuda_amd/tools/ab.py --dtype bf16 --head-dim 64"
O2=gpurun_out/r05_ab_w4_d64_bf16.jsonl
$AB2 --configs 47,19 --seq 4096 --batch 64 --causal --rounds 7 --iters 10 > $O2 &&
$AB2 --configs 47,19 --seq 8192 --causal --rounds 9 --iters 20 >> $O2 &&
$AB2 --configs 46,18 --seq 8192 --rounds 9 --iters 20 >> $O2 || exit 1
cat $O2
