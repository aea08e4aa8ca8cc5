#!/bin/bash
# One A/B pass on the box: KV-pair tests, then interleaved timings of configs
# (tools/ab.py).  Edit the AB lines per experiment.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kvpair_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_kvpair.log 2>&1 || exit 1
cd flash-attention-cuda_amd
AB() { timeout -k 10 200 python tools/ab.py "$@" || exit 1; }
{
for bhs in "1 32 512" "1 32 1024" "1 32 2048" "2 32 1024" "1 16 2048" "1 8 4096" "1 32 4096"; do
  set -- $bhs
  AB --configs 31,39,47,49,15 --batch $1 --heads $2 --seq $3 --causal --rounds 5 --iters 20
done
for bhs in "1 32 768" "1 32 1024" "1 16 2048"; do
  set -- $bhs
  AB --configs 30,38,46,48,14 --batch $1 --heads $2 --seq $3 --rounds 5 --iters 20
done
} > ../gpurun_out/ab.jsonl 2>&1
