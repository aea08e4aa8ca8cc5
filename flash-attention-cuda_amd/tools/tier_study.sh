#!/bin/bash
# Dispatcher tier study: 4-wave loop vs KV-pair vs persistent ping-pong over
# batch x seq shapes (H=32), both masks.  One tools/ab.py process per shape.
# usage: tier_study.sh OUT.jsonl "B S" ["B S" ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}/flash-attention-cuda_amd" || exit 1
out=../gpurun_out/$1
shift
mkdir -p ../gpurun_out
{
for bs in "$@"; do
  set -- $bs
  timeout -k 10 120 python tools/ab.py --configs 4,30,14 --batch $1 --seq $2 --rounds 3 --iters 20 || exit 1
  timeout -k 10 120 python tools/ab.py --configs 5,31,15 --batch $1 --seq $2 --causal --rounds 3 --iters 20 || exit 1
done
} > $out 2>&1
