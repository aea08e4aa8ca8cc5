# Scratch GPU call script (round 6, call 6): W4P pair program with two key
# tiles per barrier (product) vs one (nodblp), one-block read-ahead variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06c6
mkdir -p $O
T=flash-attention-cuda_amd/tools
step() { echo "[$(date +%T)] $*"; }
step equal &&
timeout -k 10 200 python $T/variant_equal.py --lib nodblp --config 49 --dtypes fp16,bf16 --head-dims 128,64 --shapes 1:32:1024:1,1:8:4096:1,2:3:1000:1,1:5:513:1,1:1:200:1,1:2:128:1 > $O/equal.jsonl 2>&1 &&
timeout -k 10 200 python $T/variant_equal.py --lib nodblp --config 49 --scale 6 --shapes 1:32:1024:1,1:8:4096:1 >> $O/equal.jsonl 2>&1 &&
timeout -k 10 200 python $T/variant_equal.py --lib nodblp --config 48 --dtypes fp16,bf16 --shapes 1:16:2048:0,1:4:8192:0,2:3:1000:0,1:2:100:0 >> $O/equal.jsonl 2>&1 &&
for v in pk2 pkv; do
  timeout -k 10 200 python $T/variant_equal.py --lib $v --config 49 --dtypes fp16,bf16 --shapes 1:32:1024:1,1:8:4096:1,2:3:1000:1 >> $O/equal.jsonl 2>&1 || exit 1
done
step "equal rc=$?"
step pytest &&
timeout -k 10 600 python -u -m pytest tests/test_w4p_gpu.py tests/test_dispatch_sweep_gpu.py -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
step "pytest rc=$?"
step ab &&
for sh in "--seq 1024 --causal" "--seq 512 --causal" "--heads 8 --seq 4096 --causal" "--heads 16 --seq 2048" "--seq 768 --causal" "--batch 2 --heads 8 --seq 2048 --causal"; do
  timeout -k 10 300 python $T/ab.py --configs auto --libs ,nodblp,pk2,pv8,pkv --rounds 11 $sh >> $O/ab.jsonl 2>> $O/ab.err || exit 1
done
step stamps &&
timeout -k 10 120 python $T/w4p_stamps.py --lib w4pst --seq 1024 --causal > $O/stamps.jsonl &&
timeout -k 10 120 python $T/w4p_stamps.py --lib pdst --seq 1024 --causal >> $O/stamps.jsonl
rc=$?
step "done rc=$rc"
exit $rc
