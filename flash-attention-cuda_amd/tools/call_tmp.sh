#!/bin/bash
# removal probes (timing only, wrong results): TF/s and in-kernel clock per variant
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
AB="timeout -k 10 300 python flash-attention-cuda_amd/tools/ab.py --configs auto --libs stamps,c_norowsum,c_noexp,c_nocvt,c_nomax"
O=gpurun_out/ab_removal.jsonl
$AB --seq 8192 --causal --rounds 5 --iters 20 > $O &&
$AB --seq 4096 --batch 64 --causal --rounds 5 --iters 10 >> $O || exit 1
python - $O <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(f'{r["lib"]:>12} B={r["batch"]:<3} S={r["seq"]:<6} {"c " if r["causal"] else "nc"} {r["median_tflops"]:8.1f}')
PY
cd flash-attention-cuda_amd
for v in stamps c_norowsum c_noexp c_nocvt c_nomax; do
  timeout -k 10 120 python tools/clock_check.py --batch 1 --seq 8192 --causal --lib $v 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" || exit 1
done
