#!/bin/bash
# Causal rank-band width A/B: library variants built beforehand on the CPU
#   for b in 1 4 8 16; do make -C .. variant-band$b VFLAGS=-DFA_CAUSAL_BAND=$b; done
# all timed in ONE process (tools/ab.py --libs; '' = the product's automatic band).
# usage: band_ab.sh OUT.jsonl "H S" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}/flash-attention-cuda_amd" || exit 1
mkdir -p ../gpurun_out
out=../gpurun_out/$1
shift
{
for hs in "$@"; do
  set -- $hs
  timeout -k 10 300 python tools/ab.py --configs 15 --heads $1 --seq $2 --causal --rounds 3 --iters 10 \
    --libs ,band1,band4,band8,band16 || exit 1
done
} > $out 2>&1
