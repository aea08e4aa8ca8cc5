set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python flash-attention-cuda_amd/tools/bf16_err_probe.py fp32w4 2>&1 | grep -v amdgpu.ids > gpurun_out/r05_bf16_peaked_err_fp32w4.jsonl || exit 1
cat gpurun_out/r05_bf16_peaked_err_fp32w4.jsonl
L=flash-attention-cuda_amd/lib
cp $L/libfa_mi355x.so /tmp/prod.so
cp $L/libfa_mi355x_fp32w4.so $L/libfa_mi355x.so
timeout -k 10 600 python -u -m pytest tests/test_w4_gpu.py tests/test_bf16_gpu.py tests/test_split_gpu.py tests/test_dispatch_sweep_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_w4_fp32w4.log 2>&1; rc=$?
tail -3 gpurun_out/r05_pytest_w4_fp32w4.log
cp /tmp/prod.so $L/libfa_mi355x.so
[ $rc -eq 0 ] || exit $rc
AB="timeout -k 10 300 python flash-attention-cuda_amd/tools/ab.py --configs auto --libs ,fp32w4 --rounds 7 --iters 20 --dtype bf16"
O=gpurun_out/r05_ab_w4_fp32w4.jsonl
$AB --batch 64 --seq 4096 --causal > $O &&
$AB --seq 8192 --causal >> $O &&
$AB --seq 8192 >> $O || exit 1
cat $O
