set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_w4_gpu.py tests/test_split_gpu.py tests/test_persistent_gpu.py tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_xovl.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_xovl.log; [ $rc -eq 0 ] || exit $rc
AB="timeout -k 10 300 python flash-attention-cuda_amd/tools/ab.py --configs auto --libs ,prev"
O=gpurun_out/ab_xovl.jsonl
$AB --seq 4096 --batch 64 --causal --rounds 11 --iters 10 > $O &&
$AB --seq 8192 --causal --rounds 11 --iters 20 >> $O &&
$AB --seq 8192 --rounds 9 --iters 20 >> $O &&
$AB --seq 2048 --batch 8 --causal --rounds 11 --iters 20 >> $O &&
$AB --seq 256 --batch 64 --rounds 9 --iters 20 >> $O
rc=$?; cat $O; exit $rc
