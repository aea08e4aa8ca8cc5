#!/bin/bash
# KV-quad vs KV-pair vs 4-wave loop vs persistent at short launches: parity first, then
# interleaved same-process timings (tools/ab.py).
# usage: quad_ab.sh OUT.jsonl "B H S" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
[ -n "$SKIP_TEST" ] || timeout -k 10 300 python -u -m pytest tests/test_kvpair_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_kvquad.log 2>&1 || exit 1
out=../gpurun_out/$1
shift
cd flash-attention-cuda_amd
{
for bhs in "$@"; do
  set -- $bhs
  timeout -k 10 120 python tools/ab.py --configs 4,30,38,14 --batch $1 --heads $2 --seq $3 --rounds 5 --iters 30 || exit 1
  timeout -k 10 120 python tools/ab.py --configs 5,31,39,15 --batch $1 --heads $2 --seq $3 --causal --rounds 5 --iters 30 || exit 1
done
} > $out 2>&1
