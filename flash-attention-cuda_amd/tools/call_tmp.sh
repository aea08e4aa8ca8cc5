#!/bin/bash
# scratch GPU script: GPU tests with MFMA zeroing; A/B against the v_accvgpr_write zeroing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_mfz.log 2>&1 || { tail -30 gpurun_out/pytest_mfz.log; exit 1; }
tail -1 gpurun_out/pytest_mfz.log
VARS="nomfz" OUT=mfz bash flash-attention-cuda_amd/tools/ab_vars.sh > gpurun_out/mfz.txt 2>&1 || exit 1
AB="timeout -k 10 300 python flash-attention-cuda_amd/tools/ab.py --configs auto --libs prod,nomfz --head-dim 64"
O=gpurun_out/ab_mfz_d64.jsonl
$AB --seq 8192 --causal --rounds 5 --iters 20 > $O &&
$AB --seq 4096 --batch 64 --causal --rounds 5 --iters 10 >> $O || exit 1
grep -v amdgpu.ids gpurun_out/mfz.txt
python - $O <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(f'd64 {r["lib"]:>8} B={r["batch"]:<3} S={r["seq"]:<6} {"c " if r["causal"] else "nc"} {r["median_tflops"]:8.1f}')
PY
