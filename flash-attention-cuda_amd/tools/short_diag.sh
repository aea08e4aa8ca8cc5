set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}/flash-attention-cuda_amd"
timeout -k 10 60 python tools/timeline.py --config 23 --seq 1024 --causal &&
timeout -k 10 60 python tools/timeline.py --config 31 --seq 512 --causal &&
timeout -k 10 60 python tools/timeline.py --config 22 --seq 1024 --heads 32 &&
timeout -k 10 60 python tools/stamps.py --config 23 --seq 1024 --causal
