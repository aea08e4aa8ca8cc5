#!/bin/bash
# usage: VARS="a,b" [OUT=name] bash tools/ab_vars.sh -- same-process A/B of the
# product library against variants lib/libfa_mi355x_{a,b}.so on the four
# persistent-tier shapes (headline, S=8192 causal / non-causal, S=16384 causal)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=flash-attention-cuda_amd/lib
cp $L/libfa_mi355x.so $L/libfa_mi355x_prod.so
AB="timeout -k 10 300 python flash-attention-cuda_amd/tools/ab.py --configs auto --libs prod,$VARS"
O=gpurun_out/ab_${OUT:-vars}.jsonl
$AB --seq 4096 --batch 64 --causal --rounds 7 --iters 10 > $O &&
$AB --seq 8192 --causal --rounds 7 --iters 20 >> $O &&
$AB --seq 8192 --rounds 7 --iters 20 >> $O &&
$AB --seq 16384 --causal --rounds 5 --iters 10 >> $O || exit 1
python - "$O" <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
for r in rows:
    print(f'{r["lib"]:>8} B={r["batch"]:<3} S={r["seq"]:<6} {"c " if r["causal"] else "nc"} {r["median_tflops"]:8.1f}')
PY
