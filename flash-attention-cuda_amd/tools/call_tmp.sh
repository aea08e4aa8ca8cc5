# Scratch GPU call script (round 6, call 1): pool-order traffic / speed and the
# timing-method reconciliation.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06c1
mkdir -p $O
T=flash-attention-cuda_amd/tools
step() { echo "[$(date +%T)] $*"; }
step pool-tests &&
timeout -k 10 300 python -u -m pytest tests/test_w4_pool_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_pool.log 2>&1 &&
step traffic &&
timeout -k 10 400 python $T/traffic_ab.py --libs ,pg1,pg2,pg4 --config auto --shapes 64x32x4096 --causal > $O/pool_traffic.jsonl 2> $O/pool_traffic.err &&
step pool-speed &&
timeout -k 10 300 python $T/ab.py --configs auto --libs ,pg1,pg2,pg4 --batch 64 --seq 4096 --causal --rounds 9 --iters 10 > $O/pool_speed.jsonl 2> $O/pool_speed.err &&
step methods &&
timeout -k 10 600 python $T/method_ab.py --shapes 1:32:4096:1,1:32:2048:1,1:32:1024:1,2:32:1024:1,4:32:1024:1,1:8:4096:1,1:16:4096:1 --arms 39,53,49,23,31,auto > $O/methods.jsonl 2> $O/methods.err &&
timeout -k 10 400 python $T/method_ab.py --shapes 1:16:2048:0,1:24:2048:0,1:4:8192:0,1:32:8192:1 --arms 38,48,22,30,39,auto > $O/methods_b.jsonl 2> $O/methods_b.err &&
step clocks &&
timeout -k 10 300 python $T/method_ab.py --lib stamps --shapes 1:32:4096:1,1:32:2048:1 --arms 39,53 > $O/methods_clock.jsonl 2> $O/methods_clock.err
rc=$?
step "done rc=$rc"
exit $rc
