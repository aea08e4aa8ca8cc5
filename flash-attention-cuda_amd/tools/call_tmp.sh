set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_w4_gpu.py tests/test_d64_gpu.py -x -v --timeout 120 --timeout-method thread -k "d64" > gpurun_out/pytest_w4_d64.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_w4_d64.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_w4_d64.log | head -20; exit $rc; }
AB="timeout -k 10 200 python flash-attention-cuda_amd/tools/ab.py --rounds 7 --iters 20 --head-dim 64"
O=gpurun_out/ab_w4_d64.jsonl
$AB --configs 14,44 --seq 8192 > $O &&
$AB --configs 15,45 --seq 8192 --causal >> $O &&
$AB --configs 15,45 --seq 4096 --batch 64 --causal --iters 5 >> $O &&
$AB --configs 14,44 --seq 4096 >> $O &&
$AB --configs 15,45 --seq 16384 --causal --iters 10 >> $O &&
$AB --configs 15,45 --seq 2048 --batch 8 --causal >> $O || exit 1
python - "$O" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(f'{r["config"][:50]:>50} B={r["batch"]:<3} S={r["seq"]:<6} {"c " if r["causal"] else "nc"} {r["median_tflops"]:8.1f}')
PY
VARS=v14 OUT=r04_v14 bash flash-attention-cuda_amd/tools/ab_vars.sh || exit 1
cd flash-attention-cuda_amd
for v in s_base s_v14; do
  echo "== $v"
  timeout -k 10 60 python tools/w4_stamps.py --config 38 --seq 8192 --lib $v || exit 1
  timeout -k 10 60 python tools/w4_stamps.py --config 39 --batch 64 --seq 4096 --causal --lib $v || exit 1
done 2>&1 | grep -v amdgpu.ids | tee ../gpurun_out/r04_stamps_v14.txt
cd ..
L=flash-attention-cuda_amd/lib
cp $L/libfa_mi355x.so $L/libfa_mi355x_prod.so && cp $L/libfa_mi355x_v14.so $L/libfa_mi355x.so
timeout -k 10 600 python -u -m pytest tests/test_w4_gpu.py tests/test_split_gpu.py -x -q --timeout 120 --timeout-method thread -k "not d64" > gpurun_out/pytest_v14.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_v14.log; exit $rc
