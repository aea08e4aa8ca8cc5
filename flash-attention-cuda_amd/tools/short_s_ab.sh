#!/bin/bash
# Short-sequence tier A/B on the box: 4-wave loop vs KV-pair vs persistent ping-pong,
# B=1 H=32, S in 512..2048, both masks (tools/ab.py, one process per shape).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}/flash-attention-cuda_amd" || exit 1
NC=${NC_CFGS:-4,30,14}
C=${C_CFGS:-5,31,15}
for s in ${SEQS:-512 768 1024 2048}; do
  timeout -k 10 120 python tools/ab.py --configs $NC --seq $s --rounds 5 --iters 50 || exit $?
  timeout -k 10 120 python tools/ab.py --configs $C --seq $s --causal --rounds 5 --iters 50 || exit $?
done
