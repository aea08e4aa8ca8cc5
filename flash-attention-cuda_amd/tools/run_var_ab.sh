# usage: VAR=name bash tools/run_var_ab.sh -- A/B lib variant vs product, then the
# W4/split parity tests with the variant in the product's place (box copy only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=flash-attention-cuda_amd/lib
cp $L/libfa_mi355x.so $L/libfa_mi355x_prod.so
AB="timeout -k 10 300 python flash-attention-cuda_amd/tools/ab.py --configs auto --libs prod,$VAR"
O=gpurun_out/ab_$VAR.jsonl
$AB --seq 4096 --batch 64 --causal --rounds 9 --iters 10 > $O &&
$AB --seq 8192 --causal --rounds 9 --iters 20 >> $O &&
$AB --seq 8192 --rounds 9 --iters 20 >> $O &&
$AB --seq 16384 --causal --rounds 5 --iters 10 >> $O || exit 1
cat $O
cp $L/libfa_mi355x_$VAR.so $L/libfa_mi355x.so
timeout -k 10 600 python -u -m pytest tests/test_w4_gpu.py tests/test_split_gpu.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$VAR.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_$VAR.log; exit $rc
