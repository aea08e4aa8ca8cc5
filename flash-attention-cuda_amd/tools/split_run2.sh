set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 python -u -m pytest tests/test_w4_gpu.py tests/test_split_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/split2_test.log 2>&1 &&
cd flash-attention-cuda_amd &&
for spec in "1 8 4096" "1 4 8192" "1 2 16384" "1 16 2048" "1 4 4096" "2 8 2048" "1 8 2048"; do
  set -- $spec
  timeout -k 10 120 python tools/ab.py --configs auto,$(python -c "import sys; sys.path.insert(0,'.'); import fa_mi355x as f; print(f.select_config($1,$2,$3,True))") --batch $1 --heads $2 --seq $3 --causal --rounds 5 --iters 20 || exit 1
done > ../gpurun_out/split_ab2.jsonl 2>&1
