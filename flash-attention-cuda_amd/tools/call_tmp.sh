set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
cd flash-attention-cuda_amd
for spec in "1 32 1024 --causal" "1 32 2048 --causal --quad"; do
  set -- $spec
  timeout -k 10 120 python tools/w4p_stamps.py --batch $1 --heads $2 --seq $3 $4 $5 || exit 1
done 2>&1 | grep -v amdgpu.ids > ../gpurun_out/w4p_stamps.jsonl || exit 1
echo done
