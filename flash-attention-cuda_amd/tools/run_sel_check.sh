# every fp16 d128 tier vs the default dispatch (auto) on short / mid shapes, one process per shape
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out/sel_check.jsonl; : > $O
AB="timeout -k 10 120 python flash-attention-cuda_amd/tools/ab.py --rounds 5 --iters 20"
for s in 512 1024 2048 4096; do
  $AB --configs auto,1,3,7,23,31,39,43 --seq $s --causal >> $O || exit 1
  $AB --configs auto,0,2,6,22,30,38,42 --seq $s >> $O || exit 1
done
$AB --configs auto,7,23,31,39 --seq 2048 --batch 4 --causal >> $O &&
$AB --configs auto,6,22,30,38 --seq 1024 --batch 8 >> $O
