#!/bin/bash
# one barrier per item seam (W4_XP=onebar): W4/d64/split tests on the variant, A/B, prologue stamps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=flash-attention-cuda_amd/lib
cp $L/libfa_mi355x.so /tmp/prod_keep.so && cp $L/libfa_mi355x_ob.so $L/libfa_mi355x.so &&
timeout -k 10 400 python -u -m pytest tests/test_w4_gpu.py tests/test_d64_gpu.py tests/test_split_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ob.log 2>&1
rc=$?; cp /tmp/prod_keep.so $L/libfa_mi355x.so; tail -3 gpurun_out/pytest_ob.log; [ $rc -eq 0 ] || exit $rc
VARS="ob" OUT=ob bash flash-attention-cuda_amd/tools/ab_vars.sh > gpurun_out/ob.txt 2>&1 || exit 1
AB="timeout -k 10 300 python flash-attention-cuda_amd/tools/ab.py --configs auto --libs prod,ob --head-dim 64"
O=gpurun_out/ab_ob_d64.jsonl
$AB --seq 8192 --causal --rounds 5 --iters 20 > $O &&
$AB --seq 4096 --batch 64 --causal --rounds 5 --iters 10 >> $O || exit 1
grep -v amdgpu.ids gpurun_out/ob.txt
python - $O <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(f'd64 {r["lib"]:>8} B={r["batch"]:<3} S={r["seq"]:<6} {"c " if r["causal"] else "nc"} {r["median_tflops"]:8.1f}')
PY
cd flash-attention-cuda_amd
timeout -k 10 120 python tools/w4_prostamps.py --config 39 --batch 64 --seq 4096 --causal --lib p_ob 2>&1 | grep -v amdgpu.ids
