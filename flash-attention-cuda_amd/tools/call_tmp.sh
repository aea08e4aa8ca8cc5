# Scratch GPU call script: the driver's torchrun launch mode at N=1 on the final tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 5 --no-sweep --no-cpu-baseline > gpurun_out/r05_bench_torchrun_n1.json 2> gpurun_out/r05_bench_torchrun_n1.err || { tail -20 gpurun_out/r05_bench_torchrun_n1.err; exit 1; }
cat gpurun_out/r05_bench_torchrun_n1.json
