#!/bin/bash
# Tier study over head counts (B=1): 4-wave vs KV-pair vs persistent, both masks.
# usage: tier_study_heads.sh OUT.jsonl "H S" ["H S" ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}/flash-attention-cuda_amd" || exit 1
out=../gpurun_out/$1
shift
mkdir -p ../gpurun_out
{
for hs in "$@"; do
  set -- $hs
  timeout -k 10 120 python tools/ab.py --configs 4,30,14 --heads $1 --seq $2 --rounds 3 --iters 10 || exit 1
  timeout -k 10 120 python tools/ab.py --configs 5,31,15 --heads $1 --seq $2 --causal --rounds 3 --iters 10 || exit 1
done
} > $out 2>&1
