set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
AB="timeout -k 10 400 python flash-attention-cuda_amd/tools/ab.py --configs auto --libs ,grp16,pg1,grp16pg1"
O=gpurun_out/r05_ab_pool_order2.jsonl
$AB --seq 4096 --batch 64 --causal --rounds 9 --iters 10 > $O &&
$AB --seq 4096 --batch 32 --causal --rounds 9 --iters 10 >> $O &&
$AB --seq 4096 --batch 64 --causal --rounds 7 --iters 10 --dtype bf16 >> $O &&
$AB --seq 8192 --batch 16 --rounds 7 --iters 10 >> $O &&
$AB --seq 4096 --batch 64 --causal --rounds 7 --iters 10 --head-dim 64 >> $O || exit 1
python - <<'PY'
import json
for l in open("gpurun_out/r05_ab_pool_order2.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print(d["batch"], d["seq"], d["causal"], d["head_dim"], d.get("dtype", ""), d["lib"], d["median_tflops"], d["min_tflops"])
PY
