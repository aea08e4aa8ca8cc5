set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}/flash-attention-cuda_amd"
for b in 8 16 32 64; do
  timeout -k 10 120 python tools/ab.py --configs 38,6,0 --batch $b --seq 256 --rounds 3 --iters 30 || exit 1
done
for b in 1 2 4 8; do
  timeout -k 10 120 python tools/ab.py --configs 38,6 --batch $b --seq 2048 --rounds 3 --iters 20 || exit 1
done
