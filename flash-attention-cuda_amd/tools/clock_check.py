"""Cross-check of the in-kernel clock (stamps build): per-workgroup
s_memtime cycles and s_memrealtime span against the launch's HIP-event time.
usage: python tools/clock_check.py [--batch 64 --seq 4096 --causal]"""
import argparse
import ctypes
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import torch  # noqa: E402

import fa_mi355x as fa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--heads", type=int, default=32)
ap.add_argument("--seq", type=int, default=4096)
ap.add_argument("--causal", action="store_true")
ap.add_argument("--lib", default="stamps", help="lib/libfa_mi355x_<lib>.so, an FA_STAMPS build")
a = ap.parse_args()
fa.LIB_PATH = os.path.join(HERE, "lib", f"libfa_mi355x_{a.lib}.so")
lib = fa.load_library()
lib.fa_debug_timeline.argtypes = [ctypes.c_void_p, ctypes.c_int]
shape = (a.batch, a.heads, a.seq, 128)
q, k, v = (torch.empty(shape, dtype=torch.float16, device="cuda").uniform_(-0.5, 0.5) for _ in range(3))
o = torch.empty_like(q)
t0 = time.time()
while time.time() - t0 < 2.0:
    fa.flash_attention_fwd(q, k, v, a.causal, out=o)
    torch.cuda.synchronize()
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
st.record()
fa.flash_attention_fwd(q, k, v, a.causal, out=o)
en.record()
en.synchronize()
ms = st.elapsed_time(en)
n = 4096
buf = (ctypes.c_ulonglong * (4 * n))()
lib.fa_debug_timeline(buf, n)
recs = [(buf[4 * i], buf[4 * i + 1], buf[4 * i + 3]) for i in range(n) if buf[4 * i + 1] > buf[4 * i] > 0]
span_ticks = max(r[1] for r in recs) - min(r[0] for r in recs)
wg_ticks = sorted(r[1] - r[0] for r in recs)
cyc = sorted(r[2] for r in recs)
print(json.dumps({"shape": list(shape), "causal": a.causal, "workgroups": len(recs), "hip_event_ms": round(ms, 4),
                  "realtime_span_ticks": span_ticks, "realtime_span_ms_at_100MHz": round(span_ticks / 1e5, 4),
                  "wg_realtime_ms_median": round(wg_ticks[len(wg_ticks) // 2] / 1e5, 4),
                  "wg_memtime_cycles_median": cyc[len(cyc) // 2],
                  "ghz_memtime_over_realtime": round(cyc[len(cyc) // 2] / wg_ticks[len(wg_ticks) // 2] * 0.1, 3),
                  "ghz_memtime_over_hip_event": round(cyc[len(cyc) // 2] / (ms * 1e6), 3)}))
