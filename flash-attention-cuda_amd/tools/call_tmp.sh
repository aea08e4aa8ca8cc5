# Scratch GPU call script (round 6, call 5): W4P pairs on a two-block
# program: correctness, A/B against the four-block program, stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06c5
mkdir -p $O
T=flash-attention-cuda_amd/tools
step() { echo "[$(date +%T)] $*"; }
step pytest &&
timeout -k 10 600 python -u -m pytest tests/test_w4p_gpu.py tests/test_dispatch_sweep_gpu.py -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
step "pytest rc=$?"
step ab &&
for sh in "--seq 1024 --causal" "--seq 512 --causal" "--heads 8 --seq 4096 --causal" "--heads 16 --seq 2048" "--batch 2 --heads 8 --seq 2048 --causal" "--seq 768 --causal"; do
  timeout -k 10 300 python $T/ab.py --configs auto --libs ,pnb4 --rounds 11 $sh >> $O/ab.jsonl 2>> $O/ab.err || exit 1
done
for sh in "--seq 1024 --causal" "--heads 8 --seq 4096 --causal"; do
  timeout -k 10 300 python $T/ab.py --dtype bf16 --head-dim 64 --configs auto --libs ,pnb4 --rounds 9 $sh >> $O/ab.jsonl 2>> $O/ab.err || exit 1
done
step stamps &&
timeout -k 10 120 python $T/w4p_stamps.py --lib w4pst --seq 1024 --causal > $O/stamps.jsonl
rc=$?
step "done rc=$rc"
exit $rc
