set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
cd flash-attention-cuda_amd
{ timeout -k 10 60 python tools/w4_debug.py --config 38 --base 2 --seq 512 &&
  timeout -k 10 60 python tools/w4_debug.py --config 39 --base 3 --seq 512 --causal ; } > ../gpurun_out/w4_debug.txt 2>&1
cd ..
timeout -k 10 400 python -u -m pytest tests/test_w4_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/w4_test.log 2>&1 &&
cd flash-attention-cuda_amd &&
{ timeout -k 10 120 python tools/ab.py --configs 7,39 --seq 8192 --causal --rounds 5 --iters 10 &&
  timeout -k 10 120 python tools/ab.py --configs 6,38 --seq 8192 --rounds 5 --iters 10 &&
  timeout -k 10 200 python tools/ab.py --configs 7,39 --batch 64 --seq 4096 --causal --rounds 3 --iters 3 ; } > ../gpurun_out/w4_ab.jsonl 2>&1
