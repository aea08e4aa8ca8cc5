#!/bin/bash
# Per-tier MFMA utilisation / HBM traffic table (tools/tier_pmc.py): one
# un-profiled timing run, then three counter passes, each its own process
# under its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/tier_pmc
T=flash-attention-cuda_amd/tools/tier_pmc.py
mkdir -p $OUT
timeout -k 10 300 python $T run --time > $OUT/timing.jsonl 2> $OUT/timing.err &&
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $OUT/mfma -o mfma --output-format csv -- python $T run > $OUT/mfma.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python $T run > $OUT/fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python $T run > $OUT/write.log 2>&1 &&
timeout -k 10 600 python $T clocks > $OUT/clocks.jsonl 2> $OUT/clocks.err &&
python $T summary $OUT/timing.jsonl $OUT/mfma $OUT/fetch $OUT/write $OUT/tier_pmc.jsonl $OUT/clocks.jsonl
