set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_w4_gpu.py tests/test_d64_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_d64sp2.log 2>&1 || { tail -30 gpurun_out/r05_pytest_d64sp2.log; exit 1; }
tail -2 gpurun_out/r05_pytest_d64sp2.log
cd flash-attention-cuda_amd
O=../gpurun_out/r05_w4_tail_xcd.jsonl
timeout -k 10 300 python tools/w4_tail.py --seq 4096 --batch 64 --causal > $O &&
timeout -k 10 300 python tools/w4_tail.py --seq 8192 --batch 1 >> $O &&
timeout -k 10 300 python tools/w4_tail.py --seq 8192 --batch 1 --causal >> $O || exit 1
cat $O
