"""Per-path cycle attribution of the W4P tier (diagnostic library built with
W4P_DIAG=stamps: tools/w4_variant.sh w4pst "W4P_DIAG=stamps").  Each wave
stores, over O[row 64*X0 + 16*wave][0:32 halves], 16 dwords: cycles of
steady-2 / steady-1 / generic iterations, their counts, DMA wait + barrier,
prologue, epilogue.  Prints per-shape means per wave and the heaviest item.
usage: python tools/w4p_stamps.py [--seq S --heads H --batch B --causal]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import fa_mi355x as fa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--seq", type=int, default=1024)
ap.add_argument("--heads", type=int, default=32)
ap.add_argument("--batch", type=int, default=1)
ap.add_argument("--causal", action="store_true")
ap.add_argument("--lib", default="w4pst")
a = ap.parse_args()
fa.LIB_PATH = os.path.join(os.path.dirname(fa.LIB_PATH), f"libfa_mi355x_{a.lib}.so")
fa._lib = None
g = torch.Generator(device="cuda")
g.manual_seed(5)
q, k, v = (torch.empty((a.batch, a.heads, a.seq, 128), dtype=torch.float16, device="cuda")
           .uniform_(-0.5, 0.5, generator=g) for _ in range(3))
cid = next(c.id for c in fa.configs() if c.name == "bm128_bn64_w4x32_m16_asm_pair_" + ("causal" if a.causal else "noncausal"))
for _ in range(20):
    out = fa.flash_attention_fwd(q, k, v, a.causal, config=cid)
torch.cuda.synchronize()
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
st.record()
for _ in range(20):
    out = fa.flash_attention_fwd(q, k, v, a.causal, config=cid)
en.record()
en.synchronize()
us = st.elapsed_time(en) / 20 * 1e3
o = out.detach().cpu().contiguous().view(torch.int16).numpy().view(np.uint16)
nq = (a.seq + 63) // 64
npair = (nq + 1) // 2
names = ["s2", "s1", "gen", "n_s2", "n_s1", "n_gen", "wait_bar", "prologue", "epilogue"]
rows = []
for bh in range(a.batch * a.heads):
    b, h = divmod(bh, a.heads)
    for r in range(npair):
        x0 = (nq - 1 - r) if a.causal else 2 * r
        for w in range(4):
            row = 64 * x0 + 16 * w
            if row >= a.seq:
                continue
            words = o[b, h, row, 0:32].copy().view(np.uint32)
            rows.append((r, w, words[:9].astype(np.int64)))
arr = np.array([x[2] for x in rows])
mean = arr.mean(axis=0)
tot = [int(x[2][0] + x[2][1] + x[2][2] + x[2][6] + x[2][7] + x[2][8]) for x in rows]
heavy = rows[int(np.argmax(tot))]
res = {"shape": [a.batch, a.heads, a.seq], "causal": a.causal, "us_per_launch": round(us, 2),
       "mean": {n: round(float(m), 1) for n, m in zip(names, mean)},
       "per_s2": round(float(mean[0] / max(mean[3], 1)), 1), "per_s1": round(float(mean[1] / max(mean[4], 1)), 1),
       "per_gen": round(float(mean[2] / max(mean[5], 1)), 1), "per_wait": round(float(mean[6] / max(mean[3] + mean[4] + mean[5], 1)), 1),
       "heaviest": {"rank": heavy[0], "wave": heavy[1], **{n: int(x) for n, x in zip(names, heavy[2])}, "total": max(tot)}}
print(json.dumps(res))
