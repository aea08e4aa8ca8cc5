#!/bin/bash
# conversions spread one per gap (cvtearly): A/B, d64 A/B, stamps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
VARS="ce" OUT=ce bash flash-attention-cuda_amd/tools/ab_vars.sh > gpurun_out/ce.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ce.txt
cd flash-attention-cuda_amd
for v in s_base s_ce; do
timeout -k 10 60 python tools/w4_stamps.py --config 38 --seq 8192 --lib $v 2>&1 | grep -v amdgpu.ids || exit 1
done
