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
over the max-over-ranks wall time of K steps.  `roofline.achieved` comes from
HIP events around every launch on the launch stream; `roofline.traffic` from
two rocprofv3 --pmc passes this run starts itself (FETCH_SIZE, WRITE_SIZE).
`cpu_baseline` times the CPU oracle (a restatement of the reference's
cpu_attention) on config 0 (S=512) on this host (rank 0, N=1 only).
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
# BASELINE.json configs[0] / BASELINE.md §3: the CPU baselines' shape
CPU_CONFIG = dict(name="cfg0_b1_h32_s512_d128_noncausal", batch=1, heads=32, seq_len=512,
                  causal=False)
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


# --------------------------------------------------------------------------
# CPU baselines (reported, not the optimisation target)
# --------------------------------------------------------------------------
def _host_cpus():
    """What this process may run on: the machine's CPUs, the affinity set, and
    the pool's per-GPU thread share (OMP_NUM_THREADS is 16 on the GPU box)."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count()
    return {"host_cpus": os.cpu_count(), "affinity_cpus": affinity,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline_oracle():
    """The reference's single-threaded cpu_attention (flash_attention.cu:668-697),
    restated in oracle/fa_oracle.c ("port"), timed once over the whole of
    config 0: B=1, H=32, S=512, D=128, non-causal, srand(42) inputs, 1 thread
    (BASELINE.md §3)."""
    import oracle

    c, d = CPU_CONFIG, HEAD_DIM
    q, k, v = oracle.gen_inputs(c["batch"], c["heads"], c["seq_len"], d, 42)
    t0 = time.perf_counter()
    oracle.attention(q, k, v, c["causal"], threads=1)
    el = time.perf_counter() - t0
    flops = attention_flops(c["batch"], c["heads"], c["seq_len"], d, c["causal"])
    return {"value": flops / el / 1e12, "unit": "TFLOPS", "cores": 1, "kind": "port",
            "ms": round(el * 1e3, 1),
            "sample": f"all of {c['name']} once (32 heads), oracle/fa_oracle.c restatement of "
                      f"cpu_attention, 1 thread, {el:.2f} s", **_host_cpus()}


def cpu_baseline_torch(seconds_budget: float = 5.0):
    """Naive PyTorch-CPU eager fp32 attention softmax(QK^T/sqrt(d)) V over the
    whole of config 0, repeated for ~seconds_budget.  Threads
    = torch.get_num_threads(): on the GPU box that is the pool's 16-CPU share
    per GPU (OMP_NUM_THREADS=16), not the whole machine's CPUs."""
    import torch

    c, d = CPU_CONFIG, HEAD_DIM
    shape = (c["batch"], c["heads"], c["seq_len"], d)
    g = torch.Generator()
    g.manual_seed(42)
    q, k, v = ((torch.rand(shape, generator=g) - 0.5).half().float() for _ in range(3))

    def once():
        sc = q @ k.transpose(-1, -2) / (d ** 0.5)
        if c["causal"]:
            sc = sc + torch.full((c["seq_len"],) * 2, float("-inf")).triu(1)
        return torch.softmax(sc, dim=-1) @ v

    once()  # first-call allocation / thread-pool start-up
    reps = 0
    t0 = time.perf_counter()
    while True:
        once()
        reps += 1
        el = time.perf_counter() - t0
        if el > seconds_budget or reps >= 1000:
            break
    flops = attention_flops(c["batch"], c["heads"], c["seq_len"], d, c["causal"])
    return {"value": flops * reps / el / 1e12, "unit": "TFLOPS", "cores": torch.get_num_threads(),
            "kind": "torch_eager_fp32", "ms": round(el / reps * 1e3, 2),
            "sample": f"all of {c['name']}, fp32 eager, {reps} reps in {el:.1f} s", **_host_cpus()}


# --------------------------------------------------------------------------
# HBM traffic (roofline.traffic) and its provenance
# --------------------------------------------------------------------------
def _source_files():
    import glob

    out = []
    # every file the library is compiled from, generated includes and their
    # generators included
    for pat in ("csrc/*.hip", "csrc/*.hpp", "csrc/*.cpp", "csrc/*.h", "csrc/*.inc", "csrc/*.py",
                "asm/*.py", "Makefile"):
        out += [os.path.relpath(f, PKG) for f in glob.glob(os.path.join(PKG, pat))]
    return sorted(out)


def source_digest():
    """sha256 over the kernel library's sources: ties a committed profile to the
    code it measured (the GPU box has no .git)."""
    import hashlib

    h = hashlib.sha256()
    for rel in _source_files():
        with open(os.path.join(PKG, rel), "rb") as f:
            h.update(rel.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def kernel_symbol(cfg_name):
    """Kernel-name substring rocprofv3 reports for a tile config."""
    import fa_mi355x as fa

    return fa.kernel_symbol(cfg_name)


def _pmc_child():
    """--pmc-child: 3 launches of the headline kernel for one rocprofv3 --pmc pass."""
    import torch

    import fa_mi355x as fa

    torch.cuda.set_device(0)
    B, H, S, causal = WORKLOAD["batch"], WORKLOAD["heads"], WORKLOAD["seq_len"], WORKLOAD["causal"]
    q, k, v = _make_inputs(torch, (B, H, S, HEAD_DIM), 42, torch.device("cuda", 0))
    o = torch.empty_like(q)
    for _ in range(3):
        fa.flash_attention_fwd(q, k, v, causal, out=o)
    torch.cuda.synchronize()


def _mean_counter(root, name, kernel_substr):
    import csv
    import glob

    per = {}
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if kernel_substr in r["Kernel_Name"] and r["Counter_Name"] == name:
                    d = int(r["Dispatch_Id"])
                    per[d] = per.get(d, 0.0) + float(r["Counter_Value"])
    vals = [per[d] for d in sorted(per)][1:]  # drop the cold first dispatch
    return sum(vals) / len(vals) if vals else None


def measure_traffic_live(kernel_substr, timeout_s=150):
    """HBM bytes per headline launch, measured in THIS run: two rocprofv3 --pmc
    passes (FETCH_SIZE, then WRITE_SIZE: they do not fit one pass) over a child
    process running 3 launches; FETCH_SIZE KiB x1024 x2 (gfx950 counts half of
    wide streaming reads) + WRITE_SIZE KiB x1024 (MI355X_MICROARCH.md §HBM).
    Returns (bytes, provenance) or (None, reason)."""
    import shutil
    import subprocess
    import tempfile

    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None, "rocprofv3 not found"
    got = {}
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(td, ctr)
            cmd = ["timeout", "-s", "KILL", str(timeout_s), prof, "--pmc", ctr, "-d", d,
                   "--output-format", "csv", "--", sys.executable, os.path.abspath(__file__),
                   "--pmc-child"]
            r = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT)
            if r.returncode != 0:
                return None, f"rocprofv3 --pmc {ctr} rc={r.returncode}: {r.stderr[-300:]}"
            got[ctr] = _mean_counter(d, ctr, kernel_substr)
            if got[ctr] is None:
                return None, f"no {ctr} rows for {kernel_substr}"
    fetch_b = got["FETCH_SIZE"] * 1024 * 2
    write_b = got["WRITE_SIZE"] * 1024
    return int(fetch_b + write_b), {
        "source": "live: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE passes run by this bench "
                  "(3 launches each, first dropped)",
        "fetch_bytes": int(fetch_b), "write_bytes": int(write_b),
        "fetch_size_kib": got["FETCH_SIZE"], "write_size_kib": got["WRITE_SIZE"]}


def load_pmc_traffic():
    """Fallback when the live passes cannot run: the committed
    profiles/*_pmc_traffic.json, used only if its recorded source digest equals
    this tree's (otherwise it measured other code and is dropped)."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")))
    if not files:
        return None, "no committed profile"
    try:
        with open(files[-1]) as f:
            d = json.load(f)
    except (OSError, ValueError) as e:
        return None, repr(e)
    if d.get("workload") != WORKLOAD["name"]:
        return None, "committed profile is for another workload"
    if d.get("source_digest") != source_digest():
        return None, f"{os.path.basename(files[-1])} measured other sources (digest mismatch)"
    return d.get("hbm_bytes_per_launch"), {
        "source": f"committed {os.path.relpath(files[-1], ROOT)} (git {d.get('git_head')})",
        "source_digest": d.get("source_digest")}


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-sweep", action="store_true", help="skip the per-config sweep")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=5.0,
                    help="time budget of the torch-eager CPU baseline")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the live rocprofv3 HBM-traffic passes")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.pmc_child:
        _pmc_child()
        return

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
            cpu = cpu_baseline_oracle()
        except Exception as e:  # oracle not built: report, never fall back
            cpu = {"value": None, "error": repr(e)}
        try:
            cpu_torch = cpu_baseline_torch(args.cpu_seconds)
        except Exception as e:
            cpu_torch = {"value": None, "error": repr(e)}

    kernel_name = kernel_symbol(cfg_name)
    traffic, provenance = None, "not measured at world > 1 (per-rank shard launches)"
    if world == 1:
        live_err = "skipped (--no-pmc)"
        if not args.no_pmc:
            try:
                traffic, live_err = measure_traffic_live(kernel_name)
            except Exception as e:
                traffic, live_err = None, repr(e)
            provenance = live_err
        if traffic is None:
            traffic, provenance = load_pmc_traffic()
            if traffic is None:
                provenance = f"live: {live_err}; committed: {provenance}"

    alg_bytes = algorithmic_bytes(b_local, H, S, HEAD_DIM)
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
            "traffic_over_algorithmic": round(traffic / alg_bytes, 3) if traffic else None,
            "traffic_provenance": provenance,
            "kernel": f"{kernel_name} ({cfg_name})",
            "avg_launch_ms": round(avg_launch_ms, 4),
            "flops_per_launch": flops_per_launch,
            "algorithmic_bytes_per_launch": alg_bytes,
            "hbm_gbs_algorithmic": round(alg_bytes / (avg_launch_ms / 1e3) / 1e9, 1),
            "event_region_ms": round(region_ms, 3),
            "peak_basis": f"{props.multi_processor_count} CU x 2.4 GHz x 4096 FLOP/clk/CU",
            "source_digest": source_digest(),
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
