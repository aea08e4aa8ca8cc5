set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 python -u -m pytest tests/test_w4_gpu.py tests/test_split_gpu.py tests/test_parity_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/prol_test.log 2>&1 &&
cd flash-attention-cuda_amd &&
timeout -k 10 60 python tools/w4_pstamps.py --config 38 --batch 8 --seq 256 > ../gpurun_out/prol_ab.jsonl 2>&1 &&
timeout -k 10 60 python tools/w4_pstamps.py --config 39 --batch 64 --seq 4096 --causal >> ../gpurun_out/prol_ab.jsonl 2>&1 &&
timeout -k 10 200 python tools/ab.py --configs 39 --batch 64 --seq 4096 --causal --rounds 3 --iters 3 --libs ,dmablk,prev >> ../gpurun_out/prol_ab.jsonl 2>&1 &&
timeout -k 10 100 python tools/ab.py --configs 39 --seq 8192 --causal --rounds 5 --iters 10 --libs ,dmablk,prev >> ../gpurun_out/prol_ab.jsonl 2>&1 &&
timeout -k 10 100 python tools/ab.py --configs 38 --seq 8192 --rounds 5 --iters 10 --libs ,dmablk,prev >> ../gpurun_out/prol_ab.jsonl 2>&1 &&
timeout -k 10 100 python tools/ab.py --configs 38 --seq 2048 --rounds 5 --iters 20 --libs ,dmablk,prev >> ../gpurun_out/prol_ab.jsonl 2>&1 &&
timeout -k 10 100 python tools/ab.py --configs 38 --batch 8 --seq 256 --rounds 5 --iters 30 --libs ,dmablk,prev >> ../gpurun_out/prol_ab.jsonl 2>&1
