set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_w4_gpu.py tests/test_split_gpu.py tests/test_persistent_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_diag.log 2>&1 &&
timeout -k 10 300 python flash-attention-cuda_amd/tools/ab.py --configs auto --seq 4096 --batch 64 --causal --libs ,nodiag --rounds 7 --iters 10 > gpurun_out/ab_diag.jsonl &&
timeout -k 10 300 python flash-attention-cuda_amd/tools/ab.py --configs auto --seq 8192 --causal --libs ,nodiag --rounds 9 --iters 20 >> gpurun_out/ab_diag.jsonl &&
timeout -k 10 300 python flash-attention-cuda_amd/tools/ab.py --configs auto --seq 16384 --causal --libs ,nodiag --rounds 5 --iters 10 >> gpurun_out/ab_diag.jsonl
rc=$?; tail -3 gpurun_out/pytest_diag.log; cat gpurun_out/ab_diag.jsonl; exit $rc
