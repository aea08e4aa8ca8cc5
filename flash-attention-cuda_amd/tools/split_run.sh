set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_split_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/split_test.log 2>&1 &&
cd flash-attention-cuda_amd &&
for s in 512 768 1024 2048; do
  timeout -k 10 120 python tools/ab.py --configs auto,39,$(python -c "import sys; sys.path.insert(0,'.'); import fa_mi355x as f; print(f.select_config(1,32,$s,True))") --seq $s --causal --rounds 5 --iters 50 || exit 1
done > ../gpurun_out/split_ab.jsonl 2>&1
