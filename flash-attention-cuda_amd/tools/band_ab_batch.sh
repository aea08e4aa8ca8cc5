#!/bin/bash
# Causal rank-band width on the config-5 shapes (B=64 and its N=8 shard B=8,
# H=32, S=4096): FA_CAUSAL_BAND override, one process per setting, two passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}/flash-attention-cuda_amd" || exit 1
mkdir -p ../gpurun_out
{
for pass in 1 2; do
  for b in 64 8; do
    for band in 2 4 8 16 32; do
      FA_CAUSAL_BAND=$band timeout -k 10 120 python tools/ab.py --configs 15 --batch $b --heads 32 --seq 4096 --causal --rounds 3 --iters 5 --env band$band || exit 1
    done
  done
done
} > ../gpurun_out/band_ab_batch.jsonl 2>&1
