set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
AB="timeout -k 10 400 python flash-attention-cuda_amd/tools/ab.py --configs static --libs ,ew16"
O=gpurun_out/r05_ab_seam_probes3.jsonl
$AB --seq 4096 --batch 64 --causal --rounds 7 --iters 10 > $O &&
$AB --seq 4096 --batch 64 --causal --rounds 7 --iters 10 --data small >> $O &&
$AB --seq 8192 --causal --rounds 9 --iters 20 >> $O || exit 1
cat $O
