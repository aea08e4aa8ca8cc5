# Scratch GPU call script (gpurun -- 'bash flash-attention-cuda_amd/tools/call_tmp.sh').
# Left at the round's final-tree pass: parity + smoke + bench + rocprof +
# harness (tools/gpu_check.sh), then the SDPA head-to-heads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ROUND=r05 bash flash-attention-cuda_amd/tools/gpu_check.sh || exit 1
bash flash-attention-cuda_amd/tools/vs_sdpa_all.sh || exit 1
echo done
