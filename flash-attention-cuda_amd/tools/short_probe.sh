set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}/flash-attention-cuda_amd"
for s in 512 1024 2048; do
  timeout -k 10 120 python tools/ab.py --configs 39,23,31 --seq $s --causal --rounds 5 --iters 50 || exit 1
done
