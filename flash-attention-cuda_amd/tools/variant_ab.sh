#!/bin/bash
# A variant library (make variant-X VFLAGS=...) against the product library:
# bit-identity on the dispatched tiers (tools/variant_check.py), then
# interleaved same-process A/B timings (tools/ab.py --libs) of the persistent
# tier on the config shapes.  usage: variant_ab.sh X[,Y...] [causal]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}/flash-attention-cuda_amd" || exit 1
mkdir -p ../gpurun_out
V=${1:?variant}
for v in ${V//,/ }; do
  timeout -k 10 300 python -u tools/variant_check.py $v > ../gpurun_out/variant_check_$v.log 2>&1 || exit 1
done
LIBS=",$V"
AB() { timeout -k 10 200 python tools/ab.py --libs "$LIBS" "$@" || exit 1; }
V=${V//,/_}
{
AB --configs 15 --batch 64 --heads 32 --seq 4096 --causal --rounds 5 --iters 5
AB --configs 15 --batch 1 --heads 32 --seq 8192 --causal --rounds 7 --iters 20
AB --configs 15 --batch 1 --heads 32 --seq 16384 --causal --rounds 5 --iters 10
AB --configs 15 --batch 8 --heads 32 --seq 4096 --causal --rounds 5 --iters 10
[ "$2" = causal ] && exit 0
AB --configs 14 --batch 1 --heads 32 --seq 8192 --rounds 7 --iters 20
AB --configs 14 --batch 1 --heads 32 --seq 4096 --rounds 7 --iters 20
AB --configs 14 --batch 8 --heads 32 --seq 2048 --rounds 7 --iters 20
} > ../gpurun_out/ab_$V.jsonl 2>&1
exit 0
