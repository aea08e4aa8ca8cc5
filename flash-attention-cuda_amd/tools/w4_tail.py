"""End-of-launch tail of the persistent W4 kernel (stamps build, `make stamps`):
one record per workgroup (start, end), so the launch's span against the mean
workgroup end is the time the first-finished CUs sit idle.
usage: python tools/w4_tail.py --seq 4096 --batch 64 --causal"""
import argparse
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import fa_mi355x as fa  # noqa: E402

fa.LIB_PATH = os.path.join(HERE, "lib", "libfa_mi355x_stamps.so")
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--seq", type=int, default=4096)
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--heads", type=int, default=32)
ap.add_argument("--causal", action="store_true")
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
lib = fa.load_library()
lib.fa_debug_timeline.argtypes = [ctypes.c_void_p, ctypes.c_int]
shape = (a.batch, a.heads, a.seq, 128)
q, k, v = (torch.empty(shape, dtype=torch.float16, device="cuda").uniform_(-0.5, 0.5) for _ in range(3))
o = torch.empty_like(q)
res = []
for rep in range(a.reps + 1):
    fa.flash_attention_fwd(q, k, v, a.causal, out=o)
    torch.cuda.synchronize()
    if rep == 0:
        continue
    n = 256
    buf = (ctypes.c_ulonglong * (4 * n))()
    lib.fa_debug_timeline(buf, n)
    st = [buf[4 * i] for i in range(n)]
    en = [buf[4 * i + 1] for i in range(n)]
    t0 = min(st)
    ends = sorted((e - t0) / 100.0 for e in en)  # us
    starts = sorted((s - t0) / 100.0 for s in st)
    xcc = [(buf[4 * i + 2] >> 32) & 0xff for i in range(n)]
    by_x = {}
    for i in range(n):
        by_x.setdefault(xcc[i], []).append((en[i] - t0) / 100.0)
    span = ends[-1]
    mean_end = sum(ends) / n
    res.append({"span_us": round(span, 1), "mean_end_us": round(mean_end, 1),
                "p10_end_us": round(ends[n // 10], 1), "min_end_us": round(ends[0], 1),
                "idle_tail_frac": round((span - mean_end) / span, 4),
                "start_skew_us": round(starts[-1], 2),
                # per XCD: mean / max workgroup end (is the spread per die or per CU?)
                "xcd_end_us": {x: [round(sum(v) / len(v), 1), round(max(v), 1)] for x, v in sorted(by_x.items())}})
print(json.dumps({"seq": a.seq, "batch": a.batch, "heads": a.heads, "causal": a.causal, "reps": res}))
