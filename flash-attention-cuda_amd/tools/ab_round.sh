#!/bin/bash
# One A/B pass on the box: parity of the product library, stamps, and
# interleaved timings of library variants (tools/ab.py --libs).
# Edit the AB lines per experiment.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_persistent_gpu.py tests/test_kvpair_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_parity.log 2>&1 || exit 1
cd flash-attention-cuda_amd
#timeout -k 10 60 python tools/stamps.py --config 31 --seq 1024 --causal > ../gpurun_out/stamps.txt 2>&1
timeout -k 10 60 python tools/stamps.py --config 15 --seq 4096 --batch 16 --causal > ../gpurun_out/stamps.txt 2>&1
AB() { timeout -k 10 200 python tools/ab.py "$@" || exit 1; }
{
AB --configs 14 --libs ,notail --heads 12 --seq 8192 --rounds 5 --iters 10
AB --configs 14 --libs ,notail --heads 48 --seq 2048 --rounds 5 --iters 20
AB --configs 14 --libs ,notail --heads 24 --seq 4096 --rounds 5 --iters 10
AB --configs 14 --libs ,notail --seq 8192 --rounds 5 --iters 10
AB --configs 15 --libs ,notail --seq 4096 --batch 16 --causal --rounds 5 --iters 10
} > ../gpurun_out/ab.jsonl 2>&1
