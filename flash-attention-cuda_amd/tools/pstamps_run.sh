set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}/flash-attention-cuda_amd"
timeout -k 10 60 python tools/w4_pstamps.py --config 38 --batch 8 --seq 256 &&
timeout -k 10 60 python tools/w4_pstamps.py --config 38 --batch 64 --seq 256 &&
timeout -k 10 60 python tools/w4_pstamps.py --config 38 --batch 1 --seq 2048 &&
timeout -k 10 60 python tools/w4_pstamps.py --config 38 --batch 1 --seq 8192 &&
timeout -k 10 60 python tools/w4_pstamps.py --config 39 --batch 64 --seq 4096 --causal &&
timeout -k 10 60 python tools/w4_pstamps.py --config 39 --batch 1 --seq 1024 --causal
