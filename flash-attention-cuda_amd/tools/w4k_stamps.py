"""Per-segment cycle split of the short tier from its stamps diagnostic build
(tools/w4k_variant.sh kstamps "W4K_DIAG=stamps" -DFA_W4K_STAMPS: every
(wave, segment) writes s_memtime at its start, after its prologue, at its
drain and after its epilogue to O instead of merging).
usage: python tools/w4k_stamps.py --seq S [--heads H] [--batch B] [--causal] [--lib kstamps]"""
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
ap.add_argument("--lib", default="kstamps")
a = ap.parse_args()
fa.LIB_PATH = os.path.join(os.path.dirname(fa.LIB_PATH), f"libfa_mi355x_{a.lib}.so")
name = "bm64_bn64_w4x64_asm_keysplit_" + ("causal" if a.causal else "noncausal")
cid = [c.id for c in fa.configs() if c.name == name][0]
g = torch.Generator(device="cuda")
g.manual_seed(1)
shape = (a.batch, a.heads, a.seq, 128)
q, k, v = (torch.empty(shape, dtype=torch.float16, device="cuda").uniform_(-0.5, 0.5, generator=g)
           for _ in range(3))
o = torch.zeros_like(q)
for _ in range(5):
    o.zero_()
    fa.flash_attention_fwd(q, k, v, a.causal, out=o, config=cid)
torch.cuda.synchronize()
raw = o.view(torch.int32).view(-1, 64).cpu().numpy().view(np.uint32)  # one row = 64 dwords
seg = []
for row in raw:
    n, wg = int(row[8]), int(row[9])
    if n == 0 or n > 100000:
        continue
    t = [int(row[2 * i]) | (int(row[2 * i + 1]) << 32) for i in range(4)]
    if not (t[0] <= t[1] <= t[2] <= t[3]) or t[3] - t[0] > 10 ** 8:
        continue
    seg.append((wg, n, t))
wgs = {}
for wg, n, t in seg:
    wgs.setdefault(wg, []).append((n, t))
pro = [t[1] - t[0] for _, n, t in seg]
per_tile = [(t[2] - t[1]) / (n - 1) for _, n, t in seg if n > 1]
epi = [t[3] - t[2] for _, n, t in seg]
spans, skew_end = [], []
for wg, ss in wgs.items():
    t0 = min(t[0] for _, t in ss)
    spans.append(max(t[3] for _, t in ss) - t0)
    ends = [t[3] for _, t in ss]
    skew_end.append(max(ends) - min(ends))
res = {"shape": [a.batch, a.heads, a.seq], "causal": a.causal, "segments": len(seg), "workgroups": len(wgs),
       "prologue_cyc": round(float(np.mean(pro)), 1), "prologue_max": int(np.max(pro)),
       "tile_cyc": round(float(np.mean(per_tile)), 1) if per_tile else None,
       "tile_cyc_max": round(float(np.max(per_tile)), 1) if per_tile else None,
       "drain_epilogue_cyc": round(float(np.mean(epi)), 1),
       "wg_span_mean": round(float(np.mean(spans)), 1), "wg_span_max": int(np.max(spans)),
       "wg_end_skew_mean": round(float(np.mean(skew_end)), 1)}
print(json.dumps(res))
