#!/bin/bash
# Per-GPU throughput of the bench workload's batch shards (B=64/N for N=1,2,4,8;
# H=32, S=4096, causal): predicts bench.py's strong-scaling efficiency on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}/flash-attention-cuda_amd" || exit 1
mkdir -p ../gpurun_out
for b in 64 32 16 8; do
  timeout -k 10 200 python tools/ab.py --configs auto --seq 4096 --batch $b --causal --rounds 5 --iters $((320 / b)) || exit 1
done > ../gpurun_out/shard_rate.jsonl 2>&1
