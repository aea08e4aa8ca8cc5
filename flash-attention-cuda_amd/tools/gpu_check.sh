#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel trace + PMC
# traffic passes, reference-style harness.  Every GPU step has its own time
# limit and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
BENCH_SHORT="bench.py --steps 20 --warmup 5 --no-sweep --no-cpu-baseline"
step() { echo "[$(date +%T)] $*" >&2; }

step pytest-gpu
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 &&
step smoke &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
step rocprof-pmc-fetch &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/prof_fetch -o fetch --output-format csv -- python bench.py --steps 3 --warmup 1 --no-sweep --no-cpu-baseline > $OUT/prof_fetch.log 2>&1 &&
step rocprof-pmc-write &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/prof_write -o write --output-format csv -- python bench.py --steps 3 --warmup 1 --no-sweep --no-cpu-baseline > $OUT/prof_write.log 2>&1 &&
python flash-attention-cuda_amd/tools/pmc_traffic.py $OUT/prof_fetch $OUT/prof_write $OUT/pmc_traffic.json &&
cp $OUT/pmc_traffic.json profiles/${ROUND:-r01}_pmc_traffic.json &&
step bench &&
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err &&
step rocprof-kernel-trace &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_kt -o kt --output-format csv -- python $BENCH_SHORT > $OUT/prof_kt.log 2>&1 &&
step harness &&
FA_COOLDOWN_S=2 timeout -k 10 600 tests/harness/build/flash_attention > $OUT/harness.log 2>&1
rc=$?
step "done rc=$rc"
exit $rc
