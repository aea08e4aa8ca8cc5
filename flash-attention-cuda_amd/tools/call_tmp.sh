# Scratch GPU call script (round 6, call 9): W4P singles dispatched -- their
# tests, the dispatch sweep; singles at S <= 128 and at head_dim 64
# non-causal against the tiers there.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06c9
mkdir -p $O
T=flash-attention-cuda_amd/tools
step() { echo "[$(date +%T)] $*"; }
step pytest &&
timeout -k 10 900 python -u -m pytest tests/test_w4p_gpu.py tests/test_dispatch_sweep_gpu.py tests/test_cpp_entry_gpu.py tests/test_kvpair_gpu.py -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
step "pytest rc=$?"
step ab &&
for sh in "--seq 128 --causal --configs auto,65" "--seq 128 --configs auto,64" \
          "--batch 4 --seq 128 --causal --configs auto,65" "--batch 4 --seq 128 --configs auto,64" \
          "--seq 64 --configs auto,64" "--batch 8 --seq 64 --causal --configs auto,65" \
          "--head-dim 64 --seq 512 --configs auto,68,56" "--head-dim 64 --heads 16 --seq 1024 --configs auto,68,56" \
          "--head-dim 64 --heads 8 --seq 2048 --configs auto,68,56" "--head-dim 64 --heads 4 --seq 4096 --configs auto,68" \
          "--head-dim 64 --seq 512 --causal --configs auto,57" "--dtype bf16 --seq 512 --configs auto,66,32"; do
  timeout -k 10 300 python $T/ab.py --rounds 9 $sh >> $O/ab.jsonl 2>> $O/ab.err || exit 1
done
rc=$?
step "done rc=$rc"
exit $rc
