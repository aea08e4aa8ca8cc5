set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}/flash-attention-cuda_amd"
for args in "--batch 64 --seq 4096 --causal" "--batch 1 --seq 8192" "--batch 1 --seq 8192 --causal"; do
  timeout -k 10 60 python tools/clock_check.py $args || exit 1
done 2>&1 | grep -v amdgpu.ids | tee ../gpurun_out/r04_clock_check.txt
