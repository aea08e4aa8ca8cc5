"""Timing-method reconciliation (verdict r05 item 3): the same tier arms on the
same shapes, in ONE process, timed two ways --
  burst : tools/ab.py's method, every arm's 30-launch burst interleaved with
          the other arms', 7 rounds, median;
  ref   : the reference's loop (flash_attention.cu:941-960): per arm, 3 runs of
          20 warm-up + 100 timed launches, one arm at a time;
  refslp: the same with the reference's 1 s sleep before each run (:943);
  long  : 1000 back-to-back launches (steady state under the power cap).
With --lib stamps (an FA_STAMPS build) every method also reports the in-kernel
clock of its last launch (median workgroup s_memtime cycles / s_memrealtime
span, W4 / W4P / KV kernels record a per-workgroup timeline).

usage: python tools/method_ab.py --shapes 1:32:4096:1,1:32:2048:1 --arms 39,53,49,auto
       [--lib stamps] [--methods burst,ref,refslp,long]
One JSON line per (shape, arm, method)."""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import torch  # noqa: E402

import fa_mi355x as fa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shapes", required=True, help="B:H:S:causal[,...]")
ap.add_argument("--arms", required=True, help="config ids, auto (workspace path) or static (fa_fwd_f16)")
ap.add_argument("--methods", default="burst,ref,refslp,long")
ap.add_argument("--lib", default="", help="lib/libfa_mi355x_<lib>.so (stamps: in-kernel clocks)")
ap.add_argument("--head-dim", type=int, default=128)
a = ap.parse_args()
if a.lib:
    fa.LIB_PATH = os.path.join(HERE, "lib", f"libfa_mi355x_{a.lib}.so")
lib = fa.load_library()
clocks = hasattr(lib, "fa_debug_timeline")
if clocks:
    lib.fa_debug_timeline.argtypes = [ctypes.c_void_p, ctypes.c_int]
NT = 65536
tl = (ctypes.c_ulonglong * (4 * NT))()
names = {c.id: c.name for c in fa.configs()}


def clock_ghz():
    """median in-kernel clock of the last launch's workgroups (stamps build)"""
    if not clocks:
        return None
    torch.cuda.synchronize()
    lib.fa_debug_timeline(tl, NT)
    g = []
    for i in range(NT):
        t0, t1, cyc = tl[4 * i], tl[4 * i + 1], tl[4 * i + 3]
        if t1 > t0 > 0 and cyc > 0:
            g.append(cyc / (t1 - t0) * 0.1)
    return round(statistics.median(g), 3) if g else None


def run_shape(b, h, s, causal):
    gen = torch.Generator(device="cuda")
    gen.manual_seed(42)
    q, k, v = (torch.empty((b, h, s, a.head_dim), dtype=torch.float16, device="cuda").uniform_(-0.5, 0.5, generator=gen)
               for _ in range(3))
    o = torch.empty_like(q)
    flops = fa.attention_flops(b, h, s, a.head_dim, causal)
    arms = [x for x in a.arms.split(",")]

    def fwd(arm):
        if arm == "static":
            lib.fa_fwd_f16(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), b, h, s, a.head_dim,
                           int(causal), torch.cuda.current_stream().cuda_stream)
        else:
            fa.flash_attention_fwd(q, k, v, causal, out=o, config=None if arm == "auto" else int(arm))

    ok = []
    for arm in arms:
        try:
            fwd(arm)
            ok.append(arm)
        except fa.FlashAttentionError:
            pass
    torch.cuda.synchronize()

    def timed(arm, n):
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(n):
            fwd(arm)
        en.record()
        en.synchronize()
        return flops / (st.elapsed_time(en) / n / 1e3) / 1e12

    out = []
    label = lambda arm: names.get(int(arm), arm) if arm.isdigit() else arm  # noqa: E731
    sel = fa.select_config(b, h, s, causal)
    for m in a.methods.split(","):
        res = {arm: [] for arm in ok}
        ghz = {}
        if m == "burst":
            for arm in ok:
                for _ in range(5):
                    fwd(arm)
            torch.cuda.synchronize()
            for _ in range(7):
                for arm in ok:
                    res[arm].append(timed(arm, 30))
                    ghz[arm] = clock_ghz()
        else:
            for arm in ok:
                if m == "long":
                    for _ in range(20):
                        fwd(arm)
                    res[arm].append(timed(arm, 1000))
                    ghz[arm] = clock_ghz()
                    continue
                for _ in range(3):
                    if m == "refslp":
                        time.sleep(1.0)
                    for _ in range(20):
                        fwd(arm)
                    torch.cuda.synchronize()
                    res[arm].append(timed(arm, 100))
                    ghz[arm] = clock_ghz()
        for arm in ok:
            agg = statistics.median(res[arm]) if m == "burst" else sum(res[arm]) / len(res[arm])
            line = {"shape": f"{b}x{h}x{s}", "causal": causal, "head_dim": a.head_dim, "arm": label(arm),
                    "dispatched": names[sel], "method": m, "tflops": round(agg, 1),
                    "runs": [round(x, 1) for x in res[arm]], "lib": a.lib or "base"}
            if clocks:
                line["last_launch_ghz"] = ghz.get(arm)
            print(json.dumps(line), flush=True)
            out.append(line)
    del q, k, v, o
    torch.cuda.empty_cache()
    return out


for sh in a.shapes.split(","):
    b, h, s, c = (int(x) for x in sh.split(":"))
    run_shape(b, h, s, bool(c))
