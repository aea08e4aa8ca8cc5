set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AB="timeout -k 10 300 python flash-attention-cuda_amd/tools/ab.py --configs auto --libs ,tmajor"
$AB --seq 8192 --rounds 7 --iters 10 > gpurun_out/ab_tm.jsonl &&
$AB --seq 4096 --batch 64 --causal --rounds 5 --iters 5 >> gpurun_out/ab_tm.jsonl
rc=$?; cat gpurun_out/ab_tm.jsonl; exit $rc
