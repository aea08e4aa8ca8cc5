#!/bin/bash
# W4P (paired short-sequence tier): GPU tests, then same-process A/B against the
# tier the dispatcher picks.  Every step under its own time limit; stop at the
# first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-w4p}
timeout -k 10 900 python -u -m pytest tests/test_w4p_gpu.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -3 gpurun_out/${TAG}_pytest.log
[ -n "$NOAB" ] && exit 0
cd flash-attention-cuda_amd
out=../gpurun_out/${TAG}_ab.jsonl
: > $out
for spec in "1 32 1024 --causal" "1 32 2048 --causal" "1 32 512 --causal" "1 32 4096 --causal" \
            "1 16 2048 --causal" "4 32 1024 --causal" "1 8 2048 --causal" "2 32 1024 --causal" \
            "1 32 512" "1 32 1024" "1 32 2048" "1 16 1024" "1 64 1024"; do
  set -- $spec
  c=$([ "$4" == "--causal" ] && echo 49 || echo 48)
  timeout -k 10 120 python tools/ab.py --configs $c,auto --batch $1 --heads $2 --seq $3 $4 --rounds 5 --iters 20 \
    >> $out 2>&1 || { echo "ab failed: $spec"; tail -5 $out; exit 1; }
done
grep -v amdgpu.ids $out
