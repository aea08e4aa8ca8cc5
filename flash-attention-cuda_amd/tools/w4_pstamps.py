"""Per-item cycle split of the W4 asm kernel from its pstamps diagnostic build
(W4_DIAG=pstamps, tools/w4_variant.sh): prologue (item start -> loop), loop,
epilogue store issue, store drain -- averaged over every wave of every item.
usage: python tools/w4_pstamps.py --config ID --seq S [--batch B] [--heads H] [--causal]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import fa_mi355x as fa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, required=True)
ap.add_argument("--seq", type=int, default=8192)
ap.add_argument("--heads", type=int, default=32)
ap.add_argument("--batch", type=int, default=1)
ap.add_argument("--causal", action="store_true")
ap.add_argument("--lib", default="pstamps")
a = ap.parse_args()
fa.LIB_PATH = os.path.join(os.path.dirname(fa.LIB_PATH), f"libfa_mi355x_{a.lib}.so")
g = torch.Generator(device="cuda")
g.manual_seed(1)
shape = (a.batch, a.heads, a.seq, 128)
q, k, v = (torch.empty(shape, dtype=torch.float16, device="cuda").uniform_(-0.5, 0.5, generator=g)
           for _ in range(3))
o = torch.empty_like(q)
for _ in range(3):
    fa.flash_attention_fwd(q, k, v, a.causal, out=o, config=a.config)
torch.cuda.synchronize()
rows = o.view(torch.int32).view(a.batch, a.heads, a.seq, 64)[:, :, ::64, :4].reshape(-1, 4).cpu()
rows = rows.to(torch.float64)
n = rows.shape[0]
m = rows.mean(0)
print(json.dumps({"config": fa.configs()[a.config].name, "seq": a.seq, "batch": a.batch,
                  "causal": a.causal, "wave_items": n,
                  "cyc_prologue": round(m[0].item(), 1), "cyc_loop": round(m[1].item(), 1),
                  "cyc_epi_issue": round(m[2].item(), 1), "cyc_store_drain": round(m[3].item(), 1),
                  "p90_prologue": round(rows[:, 0].quantile(0.9).item(), 1),
                  "p90_store_drain": round(rows[:, 3].quantile(0.9).item(), 1)}))
