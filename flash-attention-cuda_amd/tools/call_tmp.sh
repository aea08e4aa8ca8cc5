#!/bin/bash
# SDPA head-to-head on the final tree, then the W4 prologue-phase stamps on it
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash flash-attention-cuda_amd/tools/vs_sdpa_all.sh || exit 1
cd flash-attention-cuda_amd
timeout -k 10 120 python tools/w4_prostamps.py --config 39 --batch 64 --seq 4096 --causal --lib prostamps > ../gpurun_out/prostamps_final.txt 2>&1 &&
timeout -k 10 120 python tools/w4_prostamps.py --config 39 --seq 8192 --causal --lib prostamps >> ../gpurun_out/prostamps_final.txt 2>&1
grep -v amdgpu.ids ../gpurun_out/prostamps_final.txt
