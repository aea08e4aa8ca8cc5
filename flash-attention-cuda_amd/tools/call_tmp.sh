#!/bin/bash
# scratch GPU script: GPU tests on the wait-coalesced item program, then tile stamps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_wage.log 2>&1 || { tail -30 gpurun_out/pytest_wage.log; exit 1; }
tail -3 gpurun_out/pytest_wage.log
cd flash-attention-cuda_amd
timeout -k 10 60 python tools/w4_stamps.py --config 38 --seq 8192 --lib s_wa8 > ../gpurun_out/stamps_wa8.txt 2>&1 &&
timeout -k 10 60 python tools/w4_stamps.py --config 39 --seq 8192 --causal --lib s_wa8 >> ../gpurun_out/stamps_wa8.txt 2>&1 &&
timeout -k 10 60 python tools/w4_stamps.py --config 39 --batch 64 --seq 4096 --causal --lib s_wa8 >> ../gpurun_out/stamps_wa8.txt 2>&1
grep -v amdgpu.ids ../gpurun_out/stamps_wa8.txt
cd "${GRAFT_REPO_ROOT:-/root/repo}"
AB="timeout -k 10 300 python flash-attention-cuda_amd/tools/ab.py --configs auto --libs prod,va3,wa0 --head-dim 64"
O=gpurun_out/ab_d64_va.jsonl
cp flash-attention-cuda_amd/lib/libfa_mi355x.so flash-attention-cuda_amd/lib/libfa_mi355x_prod.so
$AB --seq 8192 --causal --rounds 5 --iters 20 > $O &&
$AB --seq 4096 --batch 64 --causal --rounds 5 --iters 10 >> $O &&
$AB --seq 8192 --rounds 5 --iters 10 >> $O || exit 1
python - $O <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(f'd64 {r["lib"]:>8} B={r["batch"]:<3} S={r["seq"]:<6} {"c " if r["causal"] else "nc"} {r["median_tflops"]:8.1f}')
PY
