"""Per-tier MFMA utilisation and HBM traffic table (north_star: "rocprof reports
achieved MFMA utilisation and HBM GB/s against the chip's fp16 peak for each
(BM,BN,warps) tile config").

One process walks a fixed list of shapes, each on the tier the dispatcher
picks for it, ITERS launches per shape, in a fixed order -- so the n-th fa::
dispatch of a rocprofv3 pass maps back to its shape.

  python tools/tier_pmc.py run [--time]      # the workload (under rocprofv3, or --time: HIP events)
  python tools/tier_pmc.py summary T.jsonl MFMA_DIR FETCH_DIR WRITE_DIR OUT.jsonl

Counter passes (separate runs, MI355X_MICROARCH.md §rocprofv3 PMC slots):
  --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE
  --pmc FETCH_SIZE          (x1024 B, x2: gfx950 half-counts wide reads)
  --pmc WRITE_SIZE          (x1024 B)
Derived per launch (first launch of each shape dropped):
  mfma_busy   = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)
                -- fraction of SIMD-cycles the matrix pipe was busy, at whatever
                clock the chip held (the guide's DVFS note)
  eff_clock   = GRBM_GUI_ACTIVE / 8 / profiled kernel time
  tflops_prof = algorithmic FLOPs / profiled kernel time (the SAME dispatches
                the counters come from; profiled runs hold a lower clock, so
                this is below the un-profiled HIP-event TFLOP/s)
  ghz_in_kernel = s_memtime cycles / s_memrealtime time per workgroup, median,
                from the stamps build after >= 2 s of launches (tier_pmc.py
                clocks), W4 and W4P rows only (the other tiers' stamps builds stamp
                every loop phase); eff_clock is left out below 0.3 ms, where it
                reads high, and above 2.4 GHz
  frac_nominal = TFLOP/s (un-profiled, HIP events) / 2516.6
  hbm_gbs     = (FETCH + WRITE bytes) / un-profiled time
"""
import csv
import glob
import json
import os
import sys

SHAPES = [  # (label, batch, heads, seq, causal[, forced tier name | "auto"])
    ("cfg0_s512_noncausal", 1, 32, 512, False),
    ("s512_causal", 1, 32, 512, True),
    ("cfg1_s1024_causal", 1, 32, 1024, True),
    ("s1024_noncausal", 1, 32, 1024, False),
    ("s768_causal", 1, 32, 768, True),
    ("s1536_causal", 1, 32, 1536, True),
    ("s2048_causal", 1, 32, 2048, True),
    ("s4096_noncausal", 1, 32, 4096, False),
    ("cfg2_s8192_noncausal", 1, 32, 8192, False),
    ("target_s8192_causal", 1, 32, 8192, True),
    ("cfg3_s16384_causal", 1, 32, 16384, True),
    ("cfg4_b8_s4096_causal_shard", 8, 32, 4096, True),   # one GPU's shard of config 5 at N=8
    ("headline_b64_s4096_causal", 64, 32, 4096, True),
    ("s256_b16_noncausal", 16, 32, 256, False),
    # the causal split tier (workspace entry; the default Python path)
    ("h8_s4096_causal", 1, 8, 4096, True, "auto"),
    ("split_h4_s8192_causal", 1, 4, 8192, True, "auto"),
    # non-dispatched tile configs (BM, BN, waves) on the same shapes: the
    # 8-wave persistent ping-pong W4 replaced, BN=128 (the reference's long
    # non-causal tile), the per-item ping-pong (what the persistent order buys)
    ("pingpong_s8192_noncausal", 1, 32, 8192, False, "bm256_bn64_w8_m16_pingpong_persistent_noncausal"),
    ("pingpong_s8192_causal", 1, 32, 8192, True, "bm256_bn64_w8_m16_pingpong_persistent_causal"),
    ("pingpong_headline_b64_s4096_causal", 64, 32, 4096, True,
     "bm256_bn64_w8_m16_pingpong_persistent_causal"),
    ("bn128_s8192_noncausal", 1, 32, 8192, False, "bm128_bn128_w4_m16_noncausal"),
    ("bn128_s8192_causal", 1, 32, 8192, True, "bm128_bn128_w4_m16_causal"),
    ("pingpong_item_s8192_causal", 1, 32, 8192, True, "bm256_bn64_w8_m16_pingpong_causal"),
    # what the round-6 singles / mixed / planned groups replaced
    ("pair_s768_causal", 1, 32, 768, True, "bm128_bn64_w4x32_m16_asm_pair_causal"),
    ("quad_s1536_causal", 1, 32, 1536, True, "bm256_bn64_w4x64_m16_asm_quad_causal"),
    ("pair_s512_causal", 1, 32, 512, True, "bm128_bn64_w4x32_m16_asm_pair_causal"),
    ("kvquad_cfg0_s512_noncausal", 1, 32, 512, False, "bm64_bn64_w8_m16_kvquad_noncausal"),
    # the KV-pair the round-5 paired / quad tier replaced on short causal launches
    ("kvpair_cfg1_s1024_causal", 1, 32, 1024, True, "bm128_bn64_w8_m16_kvpair_causal"),
    ("kvpair_s2048_causal", 1, 32, 2048, True, "bm128_bn64_w8_m16_kvpair_causal"),
    # head_dim 64 (label prefix d64_: the dispatcher's d64 twin, W4 on these)
    ("d64_target_s8192_causal", 1, 32, 8192, True, "auto"),
    ("d64_headline_b64_s4096_causal", 64, 32, 4096, True, "auto"),
]


def hd_of(label):
    return 64 if label.startswith("d64_") else 128
ITERS = 6
PEAK = 2516.6  # TFLOP/s, 256 CU x 2.4 GHz x 4096 FLOP/clk/CU
SIMDS = 1024
XCDS = 8
KERNEL_TAG = "fa::"


def run(time_it):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import fa_mi355x as fa

    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    names = {c.name: c.id for c in fa.configs()}
    only = set(os.environ.get("FA_TIER_ONLY", "").split(",")) - {""}
    for label, b, h, s, causal, *forced in SHAPES:
        if only and label not in only:
            continue
        hd = hd_of(label)
        shape = (b, h, s, hd)
        q, k, v = (torch.empty(shape, dtype=torch.float16, device="cuda").uniform_(-0.5, 0.5, generator=g)
                   for _ in range(3))
        o = torch.empty_like(q)
        cfg = (None if forced[0] == "auto" else names[forced[0]]) if forced else fa.select_config(b, h, s, causal)
        fwd = lambda: fa.flash_attention_fwd(q, k, v, causal, out=o, config=cfg)
        flops = fa.attention_flops(b, h, s, hd, causal)
        torch.cuda.synchronize()
        if time_it:
            for _ in range(3):
                fwd()
            n = 50 if flops < 1e12 else 10
            best = []
            for _ in range(3):
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                for _ in range(n):
                    fwd()
                en.record()
                en.synchronize()
                best.append(st.elapsed_time(en) / n)
            ms = sorted(best)[1]
            print(json.dumps({"label": label, "batch": b, "heads": h, "seq": s, "causal": causal,
                              "config": (fa.configs()[cfg].name if cfg is not None else
                                         "auto_d64 (W4 d64 twin)" if hd == 64 else
                                         "split_T%d" % fa.load_library().fa_fwd_split_pieces(b, h, s, 128, int(causal))),
                              "ms": ms,
                              "tflops": flops / (ms / 1e3) / 1e12, "flops": flops,
                              "alg_bytes": 8.0 * b * h * s * hd}), flush=True)
        else:
            for _ in range(ITERS):
                fwd()
            torch.cuda.synchronize()
        del q, k, v, o


def clocks():
    """In-kernel clock per shape from the stamps build (lib/libfa_mi355x_stamps.so,
    `make stamps`: every workgroup records s_memtime cycles and s_memrealtime
    ticks over its lifetime): GHz = cycles / (ticks x 10 ns), median over the
    launch's workgroups, after >= 2 s of back-to-back launches of the shape
    (MI355X_MICROARCH.md DVFS note 6).  Valid on short dispatches too, where
    GRBM_GUI_ACTIVE / kernel time reads high.  Tiers without stamps (the
    split tier) print no clock."""
    import ctypes
    import time

    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, here)
    import torch
    import fa_mi355x as fa

    fa.LIB_PATH = os.path.join(here, "lib", "libfa_mi355x_stamps.so")
    lib = fa.load_library()
    lib.fa_debug_timeline.argtypes = [ctypes.c_void_p, ctypes.c_int]
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    names = {c.name: c.id for c in fa.configs()}
    n = 4096
    buf = (ctypes.c_ulonglong * (4 * n))()
    for label, b, h, s, causal, *forced in SHAPES:
        shape = (b, h, s, hd_of(label))
        q, k, v = (torch.empty(shape, dtype=torch.float16, device="cuda").uniform_(-0.5, 0.5, generator=g)
                   for _ in range(3))
        o = torch.empty_like(q)
        cfg = (None if forced[0] == "auto" else names[forced[0]]) if forced else fa.select_config(b, h, s, causal)
        ctypes.memset(buf, 0, ctypes.sizeof(buf))
        lib.fa_debug_timeline(buf, n)  # (clears nothing on the device: records are per launch)
        t0 = time.time()
        while time.time() - t0 < 2.0:
            for _ in range(5):
                fa.flash_attention_fwd(q, k, v, causal, out=o, config=cfg)
            torch.cuda.synchronize()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        fa.flash_attention_fwd(q, k, v, causal, out=o, config=cfg)
        en.record()
        en.synchronize()
        ctypes.memset(buf, 0, ctypes.sizeof(buf))
        lib.fa_debug_timeline(buf, n)
        # the records persist across launches: keep this launch's (ending within
        # its duration of the newest record; 100-MHz realtime ticks)
        recs = [(buf[4 * i], buf[4 * i + 1], buf[4 * i + 3]) for i in range(n)
                if buf[4 * i + 1] > buf[4 * i] and buf[4 * i + 3] > 0]
        last = max((r[1] for r in recs), default=0)
        win = st.elapsed_time(en) * 1e5 * 1.2 + 100
        ghz = sorted(c / (t1 - t0) * 0.1 for t0, t1, c in recs if t1 >= last - win and t0 >= last - win)
        rec = {"label": label, "workgroups_stamped": len(ghz)}
        if ghz and cfg is not None:
            rec.update({"ghz_in_kernel_median": round(ghz[len(ghz) // 2], 3),
                        "ghz_p10": round(ghz[len(ghz) // 10], 3), "ghz_p90": round(ghz[9 * len(ghz) // 10], 3)})
        print(json.dumps(rec), flush=True)
        del q, k, v, o


def per_dispatch(root, names):
    """{counter: [value per fa:: dispatch, in dispatch order]} and kernel ns per dispatch."""
    files = glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {root}")
    per, dur, kname = {}, {}, {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if KERNEL_TAG not in r["Kernel_Name"] or r["Counter_Name"] not in names:
                continue
            d = int(r["Dispatch_Id"])
            per.setdefault(r["Counter_Name"], {}).setdefault(d, 0.0)
            per[r["Counter_Name"]][d] += float(r["Counter_Value"])
            dur[d] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            kname[d] = r["Kernel_Name"]
    order = sorted(dur)
    return {n: [per[n][d] for d in order] for n in per}, [dur[d] for d in order], [kname[d] for d in order]


def summary(timing_jsonl, mfma_dir, fetch_dir, write_dir, out, clocks_jsonl=None):
    timing = {json.loads(l)["label"]: json.loads(l) for l in open(timing_jsonl) if l.startswith("{")}
    clk = {}
    if clocks_jsonl and os.path.exists(clocks_jsonl):
        clk = {json.loads(l)["label"]: json.loads(l) for l in open(clocks_jsonl) if l.startswith("{")}
    m, dur, kn = per_dispatch(mfma_dir, {"SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_MFMA", "GRBM_GUI_ACTIVE"})
    f, _, _ = per_dispatch(fetch_dir, {"FETCH_SIZE"})
    w, _, _ = per_dispatch(write_dir, {"WRITE_SIZE"})
    # a launch may be one kernel (all dispatched tiers are single-kernel)
    assert len(dur) == ITERS * len(SHAPES), (len(dur), ITERS * len(SHAPES))
    rows = []
    for i, (label, b, h, s, causal, *_) in enumerate(SHAPES):
        sl = slice(i * ITERS + 1, (i + 1) * ITERS)  # drop the first (cold) launch
        mean = lambda xs: sum(xs[sl]) / len(xs[sl])
        busy, grbm, nmf = mean(m["SQ_VALU_MFMA_BUSY_CYCLES"]), mean(m["GRBM_GUI_ACTIVE"]), mean(m["SQ_INSTS_MFMA"])
        hbm = mean(f["FETCH_SIZE"]) * 1024 * 2 + mean(w["WRITE_SIZE"]) * 1024
        t = timing[label]
        mfma_per_flop = nmf * 16384.0 / t["flops"]  # 16x16x32: 16384 FLOP per MFMA
        busy_frac = busy / (SIMDS * grbm / XCDS)
        ghz = grbm / XCDS / mean(dur)
        tf_prof = t["flops"] / (mean(dur) * 1e-9) / 1e12
        rows.append({
            "label": label, "config": t["config"], "kernel": kn[i * ITERS].split("(")[0],
            "batch": b, "heads": h, "seq": s, "causal": causal,
            "ms": round(t["ms"], 4), "tflops": round(t["tflops"], 1),
            "frac_nominal_peak": round(t["tflops"] / PEAK, 4),
            "mfma_busy": round(busy_frac, 4),
            "mfma_insts": nmf, "busy_cycles_per_mfma": round(busy / nmf, 2),
            "mfma_per_useful_flop": round(mfma_per_flop, 4),
            # GRBM_GUI_ACTIVE / time reads high below ~0.3 ms (guide DVFS note);
            # a quotient above the 2.4 GHz maximum is a counter artefact, not a clock
            "eff_clock_ghz_profiled": round(ghz, 3) if mean(dur) >= 3e5 and ghz <= 2.4 else None,
            # in-kernel clocks only where the stamps build adds no stamps inside
            # the loop (W4: one start / end record per workgroup); the other
            # tiers' diagnostic builds stamp every phase, which moves their clock
            "ghz_in_kernel": (clk.get(label, {}).get("ghz_in_kernel_median")
                              if any(x in t["config"] for x in ("asm_persistent", "asm_pair", "asm_quad"))
                              else None),
            "ms_profiled": round(mean(dur) / 1e6, 4), "tflops_profiled": round(tf_prof, 1),

            "hbm_bytes": int(hbm), "alg_bytes": int(t["alg_bytes"]),
            "traffic_over_alg": round(hbm / t["alg_bytes"], 3),
            "hbm_gbs": round(hbm / (t["ms"] / 1e3) / 1e9, 1),
            "hbm_frac_8tbs": round(hbm / (t["ms"] / 1e3) / 8e12, 4),
        })
    with open(out, "w") as fo:
        for r in rows:
            fo.write(json.dumps(r) + "\n")
    hdr = (f"{'shape':30s} {'tier':50s} {'TF/s':>7s} {'%peak':>6s} {'GHz in-k':>8s} | {'TF/s pr':>7s} "
           f"{'mfma':>6s} {'GHz pr':>6s} | {'GB/s':>7s} {'tr/alg':>6s}")
    print(hdr)
    f2 = lambda x: "     —" if x is None else f"{x:6.2f}"
    for r in rows:
        print(f"{r['label']:30s} {r['config']:50s} {r['tflops']:7.1f} {100*r['frac_nominal_peak']:6.1f} "
              f"{f2(r['ghz_in_kernel']):>8s} | {r['tflops_profiled']:7.1f} {100*r['mfma_busy']:6.1f} "
              f"{f2(r['eff_clock_ghz_profiled'])} | {r['hbm_gbs']:7.1f} {r['traffic_over_alg']:6.2f}")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run("--time" in sys.argv)
    elif sys.argv[1] == "clocks":
        clocks()
    else:
        summary(*sys.argv[2:8])
