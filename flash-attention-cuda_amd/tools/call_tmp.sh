set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=flash-attention-cuda_amd/lib
AB="timeout -k 10 300 python flash-attention-cuda_amd/tools/ab.py --configs auto --libs ,p1ahead --rounds 9 --iters 40"
O=gpurun_out/r05_ab_w4p_ahead.jsonl
$AB --seq 1024 --causal > $O &&
$AB --seq 4096 --heads 8 --causal >> $O &&
$AB --seq 512 --causal >> $O &&
$AB --seq 2048 --causal >> $O || exit 1
cat $O
cp $L/libfa_mi355x.so /tmp/prod.so
cp $L/libfa_mi355x_p1ahead.so $L/libfa_mi355x.so
timeout -k 10 600 python -u -m pytest tests/test_w4p_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_w4p_ahead.log 2>&1; rc=$?
tail -3 gpurun_out/r05_pytest_w4p_ahead.log
cp /tmp/prod.so $L/libfa_mi355x.so
exit $rc
