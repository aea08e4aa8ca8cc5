"""Per-tile cycle split of the W4 asm kernel from its stamps diagnostic build
(W4_DIAG=stamps, lib/libfa_mi355x_w4stamps.so): phase A (QK^T + cvt + max +
staging), phase B (PV + exps, fast path), barrier (wait + skew), averaged
over the steady iterations of every wave.
usage: python tools/w4_stamps.py --config ID --seq S [--batch B] [--heads H] [--causal]"""
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
ap.add_argument("--lib", default="w4stamps")
a = ap.parse_args()
fa.LIB_PATH = os.path.join(os.path.dirname(fa.LIB_PATH), f"libfa_mi355x_{a.lib}.so")
g = torch.Generator(device="cuda")
g.manual_seed(1)
shape = (a.batch, a.heads, a.seq, 128)
q, k, v = (torch.empty(shape, dtype=torch.float16, device="cuda").uniform_(-0.5, 0.5, generator=g)
           for _ in range(3))
o = torch.empty_like(q)
for _ in range(3):  # warm clocks
    fa.flash_attention_fwd(q, k, v, a.causal, out=o, config=a.config)
torch.cuda.synchronize()
rows = o.view(torch.int32).view(a.batch, a.heads, a.seq, 64)[:, :, ::64, :4].reshape(-1, 4).cpu()
tot = rows.to(torch.float64).sum(0)
it = tot[3].item()
res = {"config": fa.configs()[a.config].name, "seq": a.seq, "batch": a.batch, "causal": a.causal,
       "steady_iters": it, "cyc_phase_a": tot[0].item() / max(it, 1), "cyc_phase_b": tot[1].item() / max(it, 1),
       "cyc_barrier": tot[2].item() / max(it, 1)}
res["cyc_tile"] = res["cyc_phase_a"] + res["cyc_phase_b"] + res["cyc_barrier"]
print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in res.items()}))
