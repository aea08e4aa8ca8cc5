#!/bin/bash
# scratch GPU script: code-placement A/B (W4_XP=shiftN variants)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
VARS="sh4,sh8,sh32" OUT=placement bash flash-attention-cuda_amd/tools/ab_vars.sh > gpurun_out/placement.txt 2>&1 &&
AB="timeout -k 10 300 python flash-attention-cuda_amd/tools/ab.py --configs auto --libs prod,sh4,sh8,sh32 --head-dim 64"
O=gpurun_out/ab_placement_d64.jsonl
$AB --seq 8192 --causal --rounds 7 --iters 20 > $O &&
$AB --seq 4096 --batch 64 --causal --rounds 5 --iters 10 >> $O &&
python - $O <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(f'd64 {r["lib"]:>8} B={r["batch"]:<3} S={r["seq"]:<6} {"c " if r["causal"] else "nc"} {r["median_tflops"]:8.1f}')
PY
cat gpurun_out/placement.txt
