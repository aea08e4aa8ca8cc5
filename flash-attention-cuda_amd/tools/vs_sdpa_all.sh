#!/bin/bash
# PyTorch SDPA head-to-head for fp16 d128, bf16 d128, fp16 d64 (tools/vs_sdpa.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}/flash-attention-cuda_amd" || exit 1
mkdir -p ../gpurun_out
timeout -k 10 300 python tools/vs_sdpa.py > ../gpurun_out/vs_sdpa.jsonl 2>&1 &&
timeout -k 10 300 python tools/vs_sdpa.py --dtype bf16 --no-headline > ../gpurun_out/vs_sdpa_bf16.jsonl 2>&1 &&
timeout -k 10 300 python tools/vs_sdpa.py --head-dim 64 --no-headline > ../gpurun_out/vs_sdpa_d64.jsonl 2>&1
