#!/bin/bash
# Causal rank-band width A/B over batch (config 5 shapes, H=32, S=4096); variants
# as in band_ab.sh, all timed in one process, two passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}/flash-attention-cuda_amd" || exit 1
mkdir -p ../gpurun_out
out=../gpurun_out/${1:-band_ab_batch.jsonl}
{
for pass in 1 2; do
  for b in 8 64; do
    timeout -k 10 300 python tools/ab.py --configs 15 --batch $b --heads 32 --seq 4096 --causal \
      --rounds 3 --iters 5 --libs band2,band4,band8,band16 --env pass$pass || exit 1
  done
done
} > $out 2>&1
