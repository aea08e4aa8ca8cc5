#!/bin/bash
# One A/B pass on the box: interleaved timings of library variants
# (tools/ab.py --libs).  Edit the AB lines per experiment.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
cd flash-attention-cuda_amd
AB() { timeout -k 10 200 python tools/ab.py "$@" || exit 1; }
{
AB --configs 30 --libs ,voff --seq 1024 --rounds 5 --iters 30
AB --configs 31 --libs ,voff --seq 1024 --causal --rounds 5 --iters 30
AB --configs 31 --libs ,voff --seq 2048 --causal --rounds 5 --iters 20
AB --configs 15 --libs ,ppsoff --seq 4096 --batch 16 --causal --rounds 5 --iters 10
AB --configs 15 --libs ,ppsoff --seq 8192 --causal --rounds 5 --iters 10
AB --configs 14 --libs ,ppsoff --seq 8192 --rounds 5 --iters 10
} > ../gpurun_out/ab.jsonl 2>&1
