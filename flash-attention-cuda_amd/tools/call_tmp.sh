set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
AB="timeout -k 10 300 python flash-attention-cuda_amd/tools/ab.py --configs auto --libs ,prev --rounds 15 --iters 40"
O=gpurun_out/r05_ab_w4p_prologue2.jsonl
$AB --seq 4096 --heads 8 --causal > $O &&
$AB --seq 2048 --causal >> $O &&
$AB --seq 1024 --causal >> $O &&
$AB --seq 4096 --heads 8 --causal >> $O &&
$AB --seq 2048 --causal >> $O || exit 1
cat $O
