set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_w4p_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_w4p_d64.log 2>&1 || { tail -40 gpurun_out/r05_pytest_w4p_d64.log; exit 1; }
tail -2 gpurun_out/r05_pytest_w4p_d64.log
AB="timeout -k 10 300 python flash-attention-cuda_amd/tools/ab.py --head-dim 64 --rounds 7 --iters 40"
O=gpurun_out/r05_ab_w4p_d64.jsonl
: > $O
for sh in "1 32 1024" "1 32 2048" "1 32 512" "2 32 1024" "1 8 4096" "1 16 4096" "4 32 1024" "1 32 4096"; do
  set -- $sh
  $AB --configs 57,61,auto --batch $1 --heads $2 --seq $3 --causal >> $O || exit 1
done
for sh in "1 16 2048" "1 4 8192" "1 32 1024" "1 48 512" "1 32 2048"; do
  set -- $sh
  $AB --configs 56,60,auto --batch $1 --heads $2 --seq $3 >> $O || exit 1
done
# advice r04: d64 at the W4 tier's thresholds (W4 d64 / KV-pair d64 / 8-wave ping-pong d64 / auto)
for sh in "1 32 2048 --causal 45,27,15" "1 48 2048 --causal 45,27,15" "1 24 2048 --causal 45,27,15" "1 20 2048 44,26,14" "1 10 4096 44,26,14"; do
  set -- $sh
  if [ "$4" = "--causal" ]; then C=--causal; CF=$5; else C=; CF=$4; fi
  $AB --configs $CF,auto --batch $1 --heads $2 --seq $3 $C >> $O || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/r05_ab_w4p_d64.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print(d["batch"], d["heads"], d["seq"], d["causal"], d["config"][:40], d["median_tflops"])
PY
