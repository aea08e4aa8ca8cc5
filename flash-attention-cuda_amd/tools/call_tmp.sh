set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}/flash-attention-cuda_amd"
mkdir -p ../gpurun_out
O=../gpurun_out/r05_w4p_split_stamps.jsonl
for lib in w4pst w4pstsp; do
  timeout -k 10 120 python tools/w4p_stamps.py --seq 1024 --causal --lib $lib || exit 1
  timeout -k 10 120 python tools/w4p_stamps.py --seq 512 --causal --lib $lib || exit 1
done 2>&1 | grep -v amdgpu.ids > $O || exit 1
cat $O
