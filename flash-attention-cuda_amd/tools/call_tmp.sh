set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash flash-attention-cuda_amd/tools/vs_sdpa_all.sh || exit 1
cd flash-attention-cuda_amd
timeout -k 10 300 python tools/w4_tail.py --seq 4096 --batch 64 --causal > ../gpurun_out/w4_tail.jsonl || exit 1
echo done
