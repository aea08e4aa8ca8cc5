#!/bin/bash
# One GPU-box pass: parity tests, smoke, the bench line (with its live PMC
# traffic passes), a rocprofv3 kernel trace of the same bench command, the
# reference-style harness.  Every GPU step has its own time limit and the chain
# stops at the first failure.  ROUND=r02 GIT_HEAD=<sha> tools/gpu_check.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out
R=${ROUND:-r02}
mkdir -p $OUT
step() { echo "[$(date +%T)] $*" >&2; }

step pytest-gpu
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
step smoke &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
step bench &&
timeout -k 10 900 python bench.py > $OUT/bench.json 2> $OUT/bench.err &&
step rocprof-kernel-trace &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_kt -o kt --output-format csv -- python bench.py --no-sweep --no-cpu-baseline --no-pmc > $OUT/bench_under_kt.json 2> $OUT/prof_kt.log &&
python flash-attention-cuda_amd/tools/kt_timed_avg.py $OUT/prof_kt/kt_kernel_trace.csv $OUT/bench_under_kt.json > $OUT/kt_timed_avg.json &&
step harness &&
FA_COOLDOWN_S=2 timeout -k 10 600 tests/harness/build/flash_attention > $OUT/harness.log 2>&1
rc=$?
step "done rc=$rc"
exit $rc
