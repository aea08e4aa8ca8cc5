# Scratch GPU call script (round 6, call 7): W4P prologue stagger by pair
# rank, one-block removal probes (no DMA / no exp2), read-ahead on the
# two-tiles-per-barrier program.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06c7
mkdir -p $O
T=flash-attention-cuda_amd/tools
step() { echo "[$(date +%T)] $*"; }
step equal &&
timeout -k 10 200 python $T/variant_equal.py --lib pkv --config 49 --dtypes fp16,bf16 --head-dims 128 --shapes 1:32:1024:1,1:8:4096:1,2:3:1000:1,1:5:513:1,1:2:128:1 > $O/equal.jsonl 2>&1 &&
timeout -k 10 200 python $T/variant_equal.py --lib stg4 --config 49 --shapes 1:32:1024:1,2:3:1000:1 >> $O/equal.jsonl 2>&1
step "equal rc=$?"
step ab &&
for sh in "--seq 1024 --causal" "--seq 512 --causal" "--heads 8 --seq 4096 --causal" "--batch 2 --heads 8 --seq 2048 --causal" "--heads 16 --seq 2048"; do
  timeout -k 10 300 python $T/ab.py --configs auto --libs ,stg2,stg4,stg8,nodma,noexp,pkv --rounds 11 $sh >> $O/ab.jsonl 2>> $O/ab.err || exit 1
done
rc=$?
step "done rc=$rc"
exit $rc
