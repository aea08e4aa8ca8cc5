#!/bin/bash
# W4P (paired short-sequence tier): GPU tests, then same-process A/B against the
# tier the dispatcher picks.  Every step under its own time limit; stop at the
# first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-w4p}
[ -z "$NOTEST" ] && { timeout -k 10 900 python -u -m pytest tests/test_w4p_gpu.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -3 gpurun_out/${TAG}_pytest.log; }
[ -n "$NOAB" ] && exit 0
cd flash-attention-cuda_amd
out=../gpurun_out/${TAG}_ab.jsonl
: > $out
SHAPES=${SHAPES:-"1,32,1024,--causal 1,32,2048,--causal 1,32,512,--causal 1,32,4096,--causal 1,16,2048,--causal 4,32,1024,--causal 1,8,2048,--causal 2,32,1024,--causal 1,32,512 1,32,1024 1,32,2048 1,16,1024 1,64,1024"}
for spec in $SHAPES; do
  spec=${spec//,/ }
  set -- $spec
  # the paired tier, the KV-pair, the KV-quad and the default dispatch (auto)
  c=$(python -c "import sys; sys.path.insert(0, '.'); import fa_mi355x as fa; m = 'causal' if '$4' == '--causal' else 'noncausal'; print(','.join(str(next(c.id for c in fa.configs() if c.name == n + m)) for n in ${TIERS:-('bm128_bn64_w4x32_m16_asm_pair_', 'bm128_bn64_w8_m16_kvpair_', 'bm64_bn64_w8_m16_kvquad_')}))")
  timeout -k 10 120 python tools/ab.py --configs $c,auto --batch $1 --heads $2 --seq $3 $4 --rounds 5 --iters 20 \
    >> $out 2>&1 || { echo "ab failed: $spec"; tail -5 $out; exit 1; }
done
grep -v amdgpu.ids $out
