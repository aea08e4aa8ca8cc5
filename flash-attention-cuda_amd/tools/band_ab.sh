#!/bin/bash
# Causal rank-band width A/B (FA_CAUSAL_BAND override, one process per setting).
# usage: band_ab.sh OUT.jsonl "H S" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}/flash-attention-cuda_amd" || exit 1
out=../gpurun_out/$1
shift
{
for hs in "$@"; do
  set -- $hs
  for band in 0 1 4 8 16; do
    FA_CAUSAL_BAND=$band timeout -k 10 120 python tools/ab.py --configs 15 --heads $1 --seq $2 --causal --rounds 3 --iters 10 --env band$band || exit 1
  done
done
} > $out 2>&1
