set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/r05_band_traffic.jsonl
timeout -k 10 600 python flash-attention-cuda_amd/tools/traffic_ab.py --libs ,band4,band16 --config 39 --shapes 1x32x8192,1x32x16384 --causal > $O || { cat $O; exit 1; }
cat $O
AB="timeout -k 10 400 python flash-attention-cuda_amd/tools/ab.py --configs 39 --libs ,band4,band16"
O2=gpurun_out/r05_ab_band.jsonl
$AB --seq 8192 --causal --rounds 9 --iters 20 > $O2 &&
$AB --seq 16384 --causal --rounds 7 --iters 10 >> $O2 || exit 1
cat $O2
