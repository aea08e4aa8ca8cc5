#!/usr/bin/env python3
"""bench.py -- MI355X flash-attention forward throughput (driver contract).

Workload (BASELINE.json configs[4], the largest single-GPU config and the one
the 1/2/4/8-GPU curve is defined on): batch=64, heads=32, head_dim=128,
seq=4096, causal, fp16 in / fp32 accumulate.  A *step* is one forward pass
(one fa_fwd_f16 launch) over this rank's batch shard.  Total batch is fixed
and sharded across ranks by batch index with no collective on the data path
(SURVEY.md §8(e)), so scaling is "strong".

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Rank 0 prints ONE JSON line.  `value` = total TFLOPS of the whole job
(reference FLOP convention 4*B*H*S^2*D/2 for causal, flash_attention.cu:938-939)
over the max-over-ranks wall time of K steps.  `roofline` is measured live with
HIP events around every launch on the launch stream.  `cpu_baseline` times the
CPU oracle (a restatement of the reference's cpu_attention) on a bounded
sample on this host (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "flash-attention-cuda_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "fp16 fwd TFLOPS + % MFMA peak, seq=512..16384 causal/non-causal, head_dim=128"
HEAD_DIM = 128
WORKLOAD = dict(name="b64_h32_s4096_d128_causal", batch=64, heads=32, seq_len=4096, causal=True)
# extra single-GPU configs reported beside the headline (BASELINE.json configs[1..3]
# plus the north_star target seq=8192 causal); timed with the reference's loop
SWEEP = [
    ("cfg1_s1024_causal", 1, 32, 1024, True),
    ("cfg2_s8192_noncausal", 1, 32, 8192, False),
    ("target_s8192_causal", 1, 32, 8192, True),
    ("cfg3_s16384_causal", 1, 32, 16384, True),
]
MFMA_FLOP_PER_CLK_PER_CU = 4096  # fp16 dense, gfx950 (16x16x32: 16384 FLOP / 16 clk / SIMD x 4)
CLOCK_HZ = 2.4e9                 # MI355X max engine clock (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0


def shard_range(total: int, world: int, rank: int):
    """Contiguous batch shard [lo, hi) of rank `rank` (sizes differ by at most 1)."""
    base, rem = divmod(total, world)
    lo = rank * base + min(rank, rem)
    hi = lo + base + (1 if rank < rem else 0)
    return lo, hi


def attention_flops(batch, heads, seq, head_dim, causal):
    f = 4.0 * batch * heads * seq * seq * head_dim
    return f / 2 if causal else f


def algorithmic_bytes(batch, heads, seq, head_dim):
    """Q, K, V read once + O written once, fp16."""
    return 8.0 * batch * heads * seq * head_dim


def mfma_peak_tflops(num_cus: int) -> float:
    return num_cus * CLOCK_HZ * MFMA_FLOP_PER_CLK_PER_CU / 1e12


def _dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def _make_inputs(torch, shape, seed, device):
    """Synthetic inputs with the reference's distribution (uniform [-0.5, 0.5]
    -> fp16, flash_attention.cu:764-769), drawn on-device from a seeded Philox
    generator (seed 42 + shard id) because the host generator would take
    minutes at 2 GiB per tensor."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    out = []
    for _ in range(3):
        t = torch.empty(shape, dtype=torch.float16, device=device)
        t.uniform_(-0.5, 0.5, generator=g)
        out.append(t)
    return out


def _time_reference_loop(torch, fa, q, k, v, o, causal, iters=100, warm=20, runs=3):
    """The reference's bench loop (:941-960): 20 warm-up, 100 timed, 3 runs."""
    res = []
    for _ in range(runs):
        for _ in range(warm):
            fa.flash_attention_fwd(q, k, v, causal, out=o)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fa.flash_attention_fwd(q, k, v, causal, out=o)
        b.record()
        b.synchronize()
        res.append(a.elapsed_time(b) / iters)
    return res


def cpu_baseline_oracle(seconds_budget: float = 20.0):
    """Oracle ("port" of cpu_attention, 1 thread) on a bounded sample of the
    workload: whole heads of the S=4096 causal problem, as many as fit the
    budget (at least one)."""
    import numpy as np

    import oracle

    s, d = WORKLOAD["seq_len"], HEAD_DIM
    q, k, v = oracle.gen_inputs(1, 1, s, d, 42)
    heads = 0
    t0 = time.perf_counter()
    while True:
        oracle.attention(q, k, v, True, threads=1)
        heads += 1
        el = time.perf_counter() - t0
        if el + el / heads > seconds_budget or heads >= 8:
            break
    flops = attention_flops(1, heads, s, d, True)
    del np
    return {"value": flops / el / 1e12, "unit": "TFLOPS", "cores": 1, "kind": "port",
            "sample": f"{heads} head(s) of b64_h32_s4096_d128_causal (S=4096, D=128, causal), "
                      f"oracle/fa_oracle.c cpu_attention restatement, 1 thread, {el:.1f} s"}


def cpu_baseline_torch(seconds_budget: float = 10.0):
    """Naive PyTorch-CPU eager fp32 attention, softmax(QK^T/sqrt(d)+mask)V
    (BASELINE.md §3), on whole heads of the workload."""
    import torch

    s, d = WORKLOAD["seq_len"], HEAD_DIM
    g = torch.Generator()
    g.manual_seed(42)
    q, k, v = ((torch.rand(1, 1, s, d, generator=g) - 0.5).half().float() for _ in range(3))
    mask = torch.full((s, s), float("-inf")).triu(1)
    heads = 0
    t0 = time.perf_counter()
    while True:
        sc = q @ k.transpose(-1, -2) / (d ** 0.5) + mask
        _ = torch.softmax(sc, dim=-1) @ v
        heads += 1
        el = time.perf_counter() - t0
        if el + el / heads > seconds_budget or heads >= 64:
            break
    flops = attention_flops(1, heads, s, d, True)
    return {"value": flops / el / 1e12, "unit": "TFLOPS", "cores": torch.get_num_threads(),
            "kind": "torch_eager_fp32", "host_cpus": os.cpu_count(),
            "sample": f"{heads} head(s) of S=4096 causal, fp32 eager, {el:.1f} s"}


def load_pmc_traffic():
    """HBM bytes per launch of the headline kernel from the committed rocprofv3
    PMC summary (profiles/*_pmc_traffic.json, FETCH_SIZE x2 + WRITE_SIZE, the
    gfx950 correction of MI355X_MICROARCH.md §HBM), or None."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")))
    if not files:
        return None
    try:
        with open(files[-1]) as f:
            d = json.load(f)
        if d.get("workload") == WORKLOAD["name"]:
            return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None
    return None


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-sweep", action="store_true", help="skip the per-config sweep")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    args = ap.parse_args()

    import torch

    import fa_mi355x as fa

    world, rank, local = _dist_env()
    if world != args.gpus:
        if rank == 0:
            print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE",
                  file=sys.stderr)
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    B, H, S, causal = WORKLOAD["batch"], WORKLOAD["heads"], WORKLOAD["seq_len"], WORKLOAD["causal"]
    lo, hi = shard_range(B, world, rank)
    b_local = hi - lo
    q, k, v = _make_inputs(torch, (b_local, H, S, HEAD_DIM), 42 + rank, dev)
    o = torch.empty_like(q)
    cfg_id = fa.select_config(b_local, H, S, causal)
    cfg_name = fa.configs()[cfg_id].name
    stream = torch.cuda.current_stream()

    for _ in range(args.warmup):
        fa.flash_attention_fwd(q, k, v, causal, out=o, stream=stream)
    torch.cuda.synchronize()

    # per-launch events on the launch stream (roofline), plus whole-region wall
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a, b in evs:
        a.record(stream)
        fa.flash_attention_fwd(q, k, v, causal, out=o, stream=stream)
        b.record(stream)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - t0
    launch_ms = [a.elapsed_time(b) for a, b in evs]
    region_ms = evs[0][0].elapsed_time(evs[-1][1])

    elapsed = torch.tensor([wall], dtype=torch.float64, device=dev)
    if dist is not None:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    wall_max = float(elapsed.item())

    total_flops = attention_flops(B, H, S, HEAD_DIM, causal) * args.steps
    value = total_flops / wall_max / 1e12
    ms_per_step = wall_max * 1e3 / args.steps

    props = torch.cuda.get_device_properties(dev)
    peak = mfma_peak_tflops(props.multi_processor_count)
    avg_launch_ms = sum(launch_ms) / len(launch_ms)
    flops_per_launch = attention_flops(b_local, H, S, HEAD_DIM, causal)
    achieved = flops_per_launch / (avg_launch_ms / 1e3) / 1e12

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    sweep = {}
    if world == 1 and not args.no_sweep:
        del q, k, v, o
        torch.cuda.empty_cache()
        for name, b, h, s, c in SWEEP:
            qq, kk, vv = _make_inputs(torch, (b, h, s, HEAD_DIM), 42, dev)
            oo = torch.empty_like(qq)
            runs = _time_reference_loop(torch, fa, qq, kk, vv, oo, c)
            tf = [attention_flops(b, h, s, HEAD_DIM, c) / (ms / 1e3) / 1e12 for ms in runs]
            avg = sum(tf) / len(tf)
            sweep[name] = {"tflops": round(avg, 1), "pct_mfma_peak": round(100 * avg / peak, 1),
                           "ms": round(sum(runs) / len(runs), 4),
                           "config": fa.configs()[fa.select_config(b, h, s, c)].name}
            del qq, kk, vv, oo

    cpu = None
    cpu_torch = None
    if world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline_oracle(args.cpu_seconds)
        except Exception as e:  # oracle not built: report, never fall back
            cpu = {"value": None, "error": repr(e)}
        try:
            cpu_torch = cpu_baseline_torch(args.cpu_seconds / 2)
        except Exception as e:
            cpu_torch = {"value": None, "error": repr(e)}

    traffic = load_pmc_traffic()
    line = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "TFLOPS",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "fp16",
        "data": "synthetic (uniform[-0.5,0.5] fp16, on-device Philox, seed 42+rank)",
        "pct_mfma_peak": round(100 * value / (peak * world), 2),
        "config": {
            "workload": WORKLOAD["name"],
            "batch": B, "heads": H, "seq_len": S, "head_dim": HEAD_DIM, "causal": causal,
            "global_batch": B, "per_gpu_batch": b_local,
            "parallelism": f"batch-shard x{world} (no collective)",
            "tile_config": cfg_name,
        },
        "roofline": {
            "bound": "mfma",
            "achieved": round(achieved, 2),
            "peak": round(peak, 1),
            "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4),
            "traffic": traffic,
            "kernel": ("fa_fwd_f16_persistent_kernel" if "persistent" in cfg_name
                       else "fa_fwd_f16_kvpair_kernel" if ("kvpair" in cfg_name or "kvquad" in cfg_name)
                       else "fa_fwd_f16_kernel") + f" ({cfg_name})",
            "avg_launch_ms": round(avg_launch_ms, 4),
            "flops_per_launch": flops_per_launch,
            "algorithmic_bytes_per_launch": algorithmic_bytes(b_local, H, S, HEAD_DIM),
            "hbm_gbs_algorithmic": round(algorithmic_bytes(b_local, H, S, HEAD_DIM)
                                         / (avg_launch_ms / 1e3) / 1e9, 1),
            "event_region_ms": round(region_ms, 3),
            "peak_basis": f"{props.multi_processor_count} CU x 2.4 GHz x 4096 FLOP/clk/CU",
        },
        "cpu_baseline": cpu,
        "cpu_baseline_torch": cpu_torch,
        "sweep": sweep or None,
    }
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
