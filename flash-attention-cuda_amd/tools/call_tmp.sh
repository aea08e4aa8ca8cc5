# Scratch GPU call script (round 6, call 2): full GPU suite on the product
# (bf16 fp32 score scaling, v9 workspace tiers), the W4 two-tiles-per-barrier
# variant ("dbl"): bit-identity vs the product, stamps, same-process A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06c2
mkdir -p $O
T=flash-attention-cuda_amd/tools
step() { echo "[$(date +%T)] $*"; }
step pytest &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
step "pytest rc=$?"
step equal &&
timeout -k 10 300 python $T/variant_equal.py --lib dbl --config 39 --dtypes fp16,bf16 --shapes 1:8:1000:1,2:4:3000:1,1:4:8192:1,1:1:64:1,1:3:200:1,1:2:300:1,1:5:513:1,1:2:16384:1 > $O/equal_c.jsonl 2>&1 &&
timeout -k 10 300 python $T/variant_equal.py --lib dbl --config 38 --dtypes fp16,bf16 --shapes 1:8:777:0,1:3:4097:0,1:1:64:0,1:2:300:0,1:4:8192:0 > $O/equal_nc.jsonl 2>&1 &&
timeout -k 10 300 python $T/variant_equal.py --lib dbl --config 39 --scale 6 --shapes 1:8:1000:1,1:4:8192:1 > $O/equal_peaked.jsonl 2>&1 &&
timeout -k 10 300 python $T/variant_equal.py --lib dbl --shapes 16:32:4096:1,1:32:8192:1,4:16:8192:0,32:32:4096:1 > $O/equal_auto.jsonl 2>&1
step "equal rc=$?"
step stamps &&
timeout -k 10 120 python $T/w4_stamps.py --lib w4st --config 38 --seq 8192 > $O/stamps.jsonl &&
timeout -k 10 120 python $T/w4_stamps.py --lib dblst --config 38 --seq 8192 >> $O/stamps.jsonl &&
timeout -k 10 120 python $T/w4_stamps.py --lib w4st --config 39 --seq 8192 --causal >> $O/stamps.jsonl &&
timeout -k 10 120 python $T/w4_stamps.py --lib dblst --config 39 --seq 8192 --causal >> $O/stamps.jsonl
step "stamps rc=$?"
step ab &&
for sh in "--seq 8192 --causal" "--seq 8192" "--seq 16384 --causal" "--seq 4096 --causal" "--batch 64 --seq 4096 --causal --iters 10" "--batch 8 --seq 4096 --causal"; do
  timeout -k 10 300 python $T/ab.py --configs auto --libs ,dbl $sh >> $O/ab.jsonl 2>> $O/ab.err || exit 1
done
for sh in "--batch 64 --seq 4096 --causal --iters 10" "--seq 8192 --causal" "--seq 1024 --causal" "--seq 2048 --causal"; do
  timeout -k 10 300 python $T/ab.py --dtype bf16 --configs auto --libs ,bf16q $sh >> $O/ab_bf16.jsonl 2>> $O/ab.err || exit 1
done
rc=$?
step "done rc=$rc"
exit $rc
