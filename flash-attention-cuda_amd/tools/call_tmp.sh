# Scratch GPU call script (round 6, call 3): full GPU suite on the product
# (dbl default, bf16 fp32 scores in every tier), A/B vs the one-tile form and
# the round-5 bf16 form, the reference-style harness.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06c3b
mkdir -p $O
T=flash-attention-cuda_amd/tools
step() { echo "[$(date +%T)] $*"; }
step pytest &&
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
step "pytest rc=$?"
step ab &&
for sh in "--seq 8192 --causal" "--seq 8192" "--seq 16384 --causal" "--batch 64 --seq 4096 --causal --iters 10"; do
  timeout -k 10 300 python $T/ab.py --configs auto --libs ,nodbl --rounds 9 $sh >> $O/ab_dbl.jsonl 2>> $O/ab.err || exit 1
done
for sh in "--batch 64 --seq 4096 --causal --iters 10" "--seq 8192 --causal" "--seq 1024 --causal" "--heads 4 --seq 8192 --causal" "--seq 512" "--batch 4 --seq 1024 --causal"; do
  timeout -k 10 300 python $T/ab.py --dtype bf16 --configs auto --libs ,bf16q $sh >> $O/ab_bf16.jsonl 2>> $O/ab.err || exit 1
done
step harness &&
FA_COOLDOWN_S=2 timeout -k 10 600 tests/harness/build/flash_attention > $O/harness.log 2>&1
rc=$?
step "done rc=$rc"
exit $rc
