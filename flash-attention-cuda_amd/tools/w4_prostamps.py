"""Per-item prologue phases of the W4 asm kernel (cross-item overlap on) from
its prostamps diagnostic build (W4_DIAG=prostamps, tools/w4_variant.sh): each
wave sums, over its items, the cycles of [Q/K(0) wait, K(0) write + Q scale,
S(0) + the previous item's deferred epilogue, first softmax + exp2, V(0)/K(1)
writes + barrier, key loop] and stores them once, in its last item's first O
row.  Prints the per-item means.
usage: python tools/w4_prostamps.py --config ID --seq S [--batch B] [--heads H] [--causal]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import fa_mi355x as fa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, required=True)
ap.add_argument("--seq", type=int, default=8192)
ap.add_argument("--heads", type=int, default=32)
ap.add_argument("--batch", type=int, default=1)
ap.add_argument("--causal", action="store_true")
ap.add_argument("--lib", default="prostamps")
a = ap.parse_args()
fa.LIB_PATH = os.path.join(os.path.dirname(fa.LIB_PATH), f"libfa_mi355x_{a.lib}.so")
g = torch.Generator(device="cuda")
g.manual_seed(1)
shape = (a.batch, a.heads, a.seq, 128)
q, k, v = (torch.empty(shape, dtype=torch.float16, device="cuda").uniform_(-0.5, 0.5, generator=g)
           for _ in range(3))
o = torch.empty_like(q)
for _ in range(3):
    o.fill_(float("nan"))
    fa.flash_attention_fwd(q, k, v, a.causal, out=o, config=a.config)
torch.cuda.synchronize()
rows = o.view(torch.int32).view(-1, 64)[::64, :8].cpu().numpy().view(np.uint32).astype(np.float64)
items = rows[:, 6]
ok = (items >= 1) & (items < 5000) & (rows[:, 5] > 0) & (rows[:, 5] < 2 ** 31)
r = rows[ok]
tot = r[:, :6].sum(0) / r[:, 6].sum()
names = ["q_wait", "k0_write_q_scale", "s0_deferred_epilogue", "first_softmax_exp", "v0k1_write_barrier", "loop"]
res = {"config": fa.configs()[a.config].name, "shape": list(shape[:3]), "causal": a.causal,
       "waves": int(ok.sum()), "items": int(r[:, 6].sum())}
res.update({n: round(float(x), 1) for n, x in zip(names, tot)})
res["prologue_total"] = round(float(tot[:5].sum()), 1)
print(json.dumps(res))
