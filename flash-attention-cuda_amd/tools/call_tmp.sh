#!/bin/bash
# all fp16 conversions ahead of phase A's first MFMA: A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
VARS="cvt0" OUT=cvt0 bash flash-attention-cuda_amd/tools/ab_vars.sh > gpurun_out/cvt0.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/cvt0.txt
