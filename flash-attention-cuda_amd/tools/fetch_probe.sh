set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}/flash-attention-cuda_amd"
for v in s_base s_noadv; do
  timeout -k 10 60 python tools/w4_stamps.py --config 38 --seq 8192 --lib $v || exit 1
  timeout -k 10 60 python tools/w4_stamps.py --config 39 --batch 64 --seq 4096 --causal --lib $v || exit 1
done
timeout -k 10 120 python tools/ab.py --configs 38 --seq 8192 --rounds 5 --iters 10 --libs ,noadv || exit 1
timeout -k 10 200 python tools/ab.py --configs 39 --batch 64 --seq 4096 --causal --rounds 3 --iters 3 --libs ,noadv
