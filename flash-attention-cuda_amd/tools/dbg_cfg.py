"""Debug one tile config against a torch fp32 reference: error map by
16-row block and 16-column block.
usage: python tools/dbg_cfg.py --config ID [--seq S] [--causal] [--lib VARIANT]"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import torch  # noqa: E402

import fa_mi355x as fa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, required=True)
ap.add_argument("--seq", type=int, default=512)
ap.add_argument("--heads", type=int, default=1)
ap.add_argument("--causal", action="store_true")
ap.add_argument("--lib", default="")
ap.add_argument("--data", default="uniform")
a = ap.parse_args()
if a.lib:
    fa.LIB_PATH = os.path.join(HERE, "lib", f"libfa_mi355x_{a.lib}.so")
g = torch.Generator(device="cuda")
g.manual_seed(5)
shape = (1, a.heads, a.seq, 128)
q, k, v = (torch.empty(shape, dtype=torch.float16, device="cuda").uniform_(-0.5, 0.5, generator=g)
           for _ in range(3))
if a.data == "vid":  # V = one-hot of the key index mod 128 (shows which keys land where)
    v.zero_()
    idx = torch.arange(a.seq, device="cuda")
    v[0, :, idx, idx % 128] = 1.0
o = fa.flash_attention_fwd(q, k, v, a.causal, config=a.config)
s = (q.float() @ k.float().transpose(-1, -2)) / (128 ** 0.5)
if a.causal:
    m = torch.ones(a.seq, a.seq, device="cuda", dtype=torch.bool).tril()
    s = s.masked_fill(~m, float("-inf"))
ref = torch.softmax(s, -1) @ v.float()
d = (o.float() - ref).abs()[0, 0]
print("max diff", d.max().item())
R, C = (a.seq + 15) // 16, 8
for r in range(R):
    row = d[16 * r:16 * r + 16]
    cells = [row[:, 16 * c:16 * c + 16].max().item() for c in range(C)]
    print(f"rows {16*r:5d}: " + " ".join("." if x < 1e-3 else ("x" if x > 0.05 else "o") for x in cells),
          f" {row.max().item():.3g}")
