#!/bin/bash
# Second half of the round's one final-tree pass (tools/gpu_check.sh is the
# first): the per-tier PMC table, the SDPA head-to-heads, the W4P stamped
# timelines and the W4 launch tail.  Each GPU step under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash flash-attention-cuda_amd/tools/tier_pmc.sh > gpurun_out/tier_pmc_table.txt 2> gpurun_out/tier_pmc.err || { tail -20 gpurun_out/tier_pmc.err; exit 1; }
bash flash-attention-cuda_amd/tools/vs_sdpa_all.sh || exit 1
cd flash-attention-cuda_amd
for spec in "1 32 1024 --causal" "1 32 2048 --causal --quad"; do
  set -- $spec
  timeout -k 10 120 python tools/w4p_stamps.py --batch $1 --heads $2 --seq $3 $4 $5 || exit 1
done 2>&1 | grep -v amdgpu.ids > ../gpurun_out/w4p_stamps.jsonl || exit 1
timeout -k 10 300 python tools/w4_tail.py --seq 4096 --batch 64 --causal > ../gpurun_out/w4_tail.jsonl || exit 1
cd ..
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_torchrun_n1.json 2> gpurun_out/bench_torchrun_n1.err || exit 1
echo done
