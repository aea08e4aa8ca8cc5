#!/bin/bash
# Short-launch diagnostics: KV-pair merge cost (diagnostic build without the merge) at B=1 H=32.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}/flash-attention-cuda_amd" || exit 1
mkdir -p ../gpurun_out
{
for s in 512 1024 2048; do
timeout -k 10 100 python tools/ab.py --configs 31,5 --libs ,nomerge --seq $s --causal --rounds 5 --iters 50 || exit 1
timeout -k 10 100 python tools/ab.py --configs 30,4 --libs ,nomerge --seq $s --rounds 5 --iters 50 || exit 1
done
} > ../gpurun_out/diag_short.txt 2>&1
