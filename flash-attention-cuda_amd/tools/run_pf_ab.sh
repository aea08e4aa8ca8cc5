set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AB="timeout -k 10 300 python flash-attention-cuda_amd/tools/ab.py --configs auto --libs ,head,pfbefore"
timeout -k 10 600 python -u -m pytest tests/test_w4_gpu.py tests/test_split_gpu.py tests/test_persistent_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pf.log 2>&1 &&
$AB --seq 4096 --batch 64 --causal --rounds 7 --iters 10 > gpurun_out/ab_pf.jsonl &&
$AB --seq 8192 --causal --rounds 9 --iters 20 >> gpurun_out/ab_pf.jsonl &&
$AB --seq 8192 --rounds 7 --iters 10 >> gpurun_out/ab_pf.jsonl &&
$AB --seq 2048 --batch 8 --rounds 9 --iters 20 >> gpurun_out/ab_pf.jsonl &&
$AB --seq 256 --batch 64 --rounds 9 --iters 20 >> gpurun_out/ab_pf.jsonl
rc=$?; tail -3 gpurun_out/pytest_pf.log; cat gpurun_out/ab_pf.jsonl; exit $rc
