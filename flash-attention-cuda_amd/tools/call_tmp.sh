#!/bin/bash
# scratch GPU script: row sums at phase-A start (timing only) A/B + stamps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
VARS="rsA" OUT=rsa bash flash-attention-cuda_amd/tools/ab_vars.sh > gpurun_out/rsa.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/rsa.txt
cd flash-attention-cuda_amd
for v in s_base s_rsA; do
timeout -k 10 60 python tools/w4_stamps.py --config 38 --seq 8192 --lib $v 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 60 python tools/w4_stamps.py --config 39 --batch 64 --seq 4096 --causal --lib $v 2>&1 | grep -v amdgpu.ids || exit 1
done
