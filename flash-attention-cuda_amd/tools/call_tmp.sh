set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
AB="timeout -k 10 120 python flash-attention-cuda_amd/tools/ab.py --rounds 5 --iters 30 --libs ,knodma,knoload,knomem"
O=gpurun_out/ab_w4k_mem.jsonl
$AB --configs 44 --seq 512 > $O &&
$AB --configs 44 --seq 1024 >> $O &&
$AB --configs 45 --seq 1024 --causal >> $O &&
$AB --configs 44 --seq 4096 --heads 2 >> $O || exit 1
python - "$O" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(f'{r["lib"]:>8} H={r["heads"]:<3} S={r["seq"]:<6} {"c " if r["causal"] else "nc"} {r["median_tflops"]:8.1f}')
PY
cd flash-attention-cuda_amd
for args in "--seq 512" "--seq 1024" "--seq 1024 --causal" "--seq 4096 --heads 2"; do
  timeout -k 10 60 python tools/w4k_stamps.py $args || exit 1
done 2>&1 | grep -v amdgpu.ids | tee ../gpurun_out/w4k_stamps.txt
