set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_w4_gpu.py tests/test_bf16_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/w4_test.log 2>&1 &&
cd flash-attention-cuda_amd &&
{ timeout -k 10 60 python tools/w4_stamps.py --config 38 --seq 8192 --lib w4stamps &&
  timeout -k 10 60 python tools/w4_stamps.py --config 39 --batch 64 --seq 4096 --causal --lib w4stamps &&
  timeout -k 10 120 python tools/ab.py --configs 39 --seq 8192 --causal --rounds 5 --iters 10 --libs ,stagea,stageb &&
  timeout -k 10 120 python tools/ab.py --configs 38 --seq 8192 --rounds 5 --iters 10 --libs ,stagea,stageb &&
  timeout -k 10 200 python tools/ab.py --configs 7,39 --batch 64 --seq 4096 --causal --rounds 3 --iters 3 ; } > ../gpurun_out/w4_ab2.jsonl 2>&1 &&
cd .. &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_all.log 2>&1
