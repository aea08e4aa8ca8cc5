"""Per-path cycle attribution of the W4P tier (diagnostic library built with
W4P_DIAG=stamps: tools/w4_variant.sh w4pst "W4P_DIAG=stamps").  Each wave
stores, over O[row of its block 0][0:32 halves], 13 dwords: cycles of the
iterations with 4 / 3 / 2 / 1 blocks with a QK^T and of the drains, their
counts, DMA wait + barrier, prologue, epilogue.  Prints per-shape means per
wave and the heaviest item.
usage: python tools/w4p_stamps.py [--seq S --heads H --batch B --causal --quad]"""
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
ap.add_argument("--quad", action="store_true")
a = ap.parse_args()
fa.LIB_PATH = os.path.join(os.path.dirname(fa.LIB_PATH), f"libfa_mi355x_{a.lib}.so")
fa._lib = None
g = torch.Generator(device="cuda")
g.manual_seed(5)
q, k, v = (torch.empty((a.batch, a.heads, a.seq, 128), dtype=torch.float16, device="cuda")
           .uniform_(-0.5, 0.5, generator=g) for _ in range(3))
tier = "bm256_bn64_w4x64_m16_asm_quad_" if a.quad else "bm128_bn64_w4x32_m16_asm_pair_"
cid = next(c.id for c in fa.configs() if c.name == tier + ("causal" if a.causal else "noncausal"))
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
G = 2 if a.quad else 1
npair = (nq + 1) // 2
nitem = (npair + G - 1) // G
names = ["q4", "q3", "q2", "q1", "drain", "n_q4", "n_q3", "n_q2", "n_q1", "n_drain", "wait_bar",
         "prologue", "epilogue"]


def blocks(r):
    """the item's blocks sorted by key tiles (fa_w4p_kernel.hpp)"""
    xs = []
    for g in range(G):
        rr = G * r + g
        if a.causal:
            hv = nq - 1 - rr
            xs += [hv if rr < npair else -1, rr if rr < hv else -1]
        else:
            xs += [2 * rr if 2 * rr < nq else -1, 2 * rr + 1 if 2 * rr + 1 < nq else -1]
    kv = [0 if x < 0 else (min(64 * x + 64, a.seq) if a.causal else a.seq) for x in xs]
    return [x for _, x in sorted(zip(kv, xs), key=lambda t: -t[0])]


rows = []
for bh in range(a.batch * a.heads):
    b, h = divmod(bh, a.heads)
    for r in range(nitem):
        x0 = blocks(r)[0]
        for w in range(4):
            row = 64 * x0 + 16 * w
            if row >= a.seq:
                continue
            words = o[b, h, row, 0:26].copy().view(np.uint32)
            rows.append((r, w, words[:13].astype(np.int64)))
arr = np.array([x[2] for x in rows])
mean = arr.mean(axis=0)
tot = [int(x[2][:5].sum() + x[2][10:13].sum()) for x in rows]
heavy = rows[int(np.argmax(tot))]
res = {"shape": [a.batch, a.heads, a.seq], "causal": a.causal, "grouping": "quad" if a.quad else "pair",
       "us_per_launch": round(us, 2), "mean": {n: round(float(m), 1) for n, m in zip(names, mean)},
       "per_iter": {n: round(float(mean[i] / max(mean[i + 5], 1e-9)), 1) for i, n in enumerate(names[:5])},
       "heaviest": {"rank": heavy[0], "wave": heavy[1], **{n: int(x) for n, x in zip(names, heavy[2])},
                    "total": max(tot)},
       "by_rank": {int(r): {n: round(float(np.mean([x[2][i] for x in rows if x[0] == r])), 1)
                            for i, n in enumerate(names) if n in ("q2", "q1", "drain", "n_q2", "n_q1", "wait_bar",
                                                                   "prologue", "epilogue")}
                   for r in sorted({x[0] for x in rows})}}
print(json.dumps(res))
