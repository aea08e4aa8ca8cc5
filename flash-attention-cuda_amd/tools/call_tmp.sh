#!/bin/bash
# final-tree pass: gpu_check (tests, smoke, bench, rocprof kernel trace, harness), then the per-tier table
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROUND=r04 bash flash-attention-cuda_amd/tools/gpu_check.sh || exit 1
bash flash-attention-cuda_amd/tools/tier_pmc.sh > gpurun_out/tier_pmc_summary.txt 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/tier_pmc_summary.txt
exit $rc
