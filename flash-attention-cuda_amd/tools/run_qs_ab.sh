set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AB="timeout -k 10 300 python flash-attention-cuda_amd/tools/ab.py --configs auto --libs ,head"
timeout -k 10 600 python -u -m pytest tests/test_w4_gpu.py tests/test_split_gpu.py tests/test_persistent_gpu.py tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_qs.log 2>&1 &&
timeout -k 10 60 python flash-attention-cuda_amd/tools/w4_pstamps.py --config 39 --batch 64 --seq 4096 --causal > gpurun_out/ab_qs.jsonl &&
timeout -k 10 60 python flash-attention-cuda_amd/tools/w4_pstamps.py --config 38 --seq 8192 >> gpurun_out/ab_qs.jsonl &&
$AB --seq 4096 --batch 64 --causal --rounds 7 --iters 10 >> gpurun_out/ab_qs.jsonl &&
$AB --seq 8192 --causal --rounds 9 --iters 20 >> gpurun_out/ab_qs.jsonl &&
$AB --seq 256 --batch 64 --rounds 9 --iters 20 >> gpurun_out/ab_qs.jsonl
rc=$?; tail -3 gpurun_out/pytest_qs.log; cat gpurun_out/ab_qs.jsonl; exit $rc
