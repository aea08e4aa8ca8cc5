set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python flash-attention-cuda_amd/tools/bf16_err_probe.py 2>&1 | grep -v amdgpu.ids > gpurun_out/r05_bf16_peaked_err.jsonl
