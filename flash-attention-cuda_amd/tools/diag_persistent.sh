#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT}/flash-attention-cuda_amd" || exit 1
mkdir -p ../gpurun_out
{
for s in 4096 8192; do
  timeout -k 10 60 python tools/timeline.py --config 15 --seq $s --causal || exit 1
  timeout -k 10 60 python tools/stamps.py --config 15 --seq $s --causal || exit 1
done
timeout -k 10 60 python tools/timeline.py --config 15 --seq 4096 --batch 64 --causal || exit 1
} > ../gpurun_out/diag.txt 2>&1
