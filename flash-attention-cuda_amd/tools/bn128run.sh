set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/bn128_test.log 2>&1 &&
cd flash-attention-cuda_amd &&
{ timeout -k 10 120 python tools/ab.py --configs 42,0,38 --seq 8192 --rounds 3 --iters 5 &&
  timeout -k 10 120 python tools/ab.py --configs 42,0,38 --seq 2048 --rounds 3 --iters 10 &&
  timeout -k 10 120 python tools/ab.py --configs 43,1,39 --seq 8192 --causal --rounds 3 --iters 5 ; } > ../gpurun_out/bn128_ab.jsonl 2>&1
