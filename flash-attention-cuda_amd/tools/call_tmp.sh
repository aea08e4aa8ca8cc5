set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python flash-attention-cuda_amd/tools/bf16_err_probe.py fp32pk 2>&1 | grep -v amdgpu.ids > gpurun_out/r05_bf16_peaked_err_fp32pk.jsonl || exit 1
cat gpurun_out/r05_bf16_peaked_err_fp32pk.jsonl
AB="timeout -k 10 300 python flash-attention-cuda_amd/tools/ab.py --configs auto --libs ,fp32scale,fp32pk --rounds 9 --iters 40 --dtype bf16"
O=gpurun_out/r05_ab_w4p_fp32pk.jsonl
$AB --seq 1024 --causal > $O &&
$AB --seq 2048 --causal >> $O &&
$AB --seq 1024 --causal --head-dim 64 >> $O &&
$AB --seq 1024 >> $O || exit 1
cat $O
L=flash-attention-cuda_amd/lib
cp $L/libfa_mi355x.so /tmp/prod.so
cp $L/libfa_mi355x_fp32pk.so $L/libfa_mi355x.so
timeout -k 10 600 python -u -m pytest tests/test_w4p_gpu.py tests/test_dispatch_sweep_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_w4p_fp32pk.log 2>&1; rc=$?
tail -3 gpurun_out/r05_pytest_w4p_fp32pk.log
cp /tmp/prod.so $L/libfa_mi355x.so
exit $rc
