"""Stage-isolating probes for a tile config against an fp32 torch reference.
usage: python tools/w4_debug.py --config ID [--seq S] [--heads H] [--causal]
Prints, per probe, the max error and an error map by 16-row block (rows) x
16-column block, so a wrong stage shows up by its pattern:
  ones_v   V = 1            -> O = 1 (normalisation / row sums only)
  zero_q   Q = 0            -> O = mean of visible V rows (PV, l; no max)
  rand     uniform inputs   (everything)
  vrow     V[k, :] = k/S    -> O = weighted mean key index (P per key)
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import fa_mi355x as fa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, required=True)
ap.add_argument("--base", type=int, default=-1, help="also diff against this config")
ap.add_argument("--seq", type=int, default=512)
ap.add_argument("--heads", type=int, default=1)
ap.add_argument("--causal", action="store_true")
ap.add_argument("--lib", default="", help="library variant X = lib/libfa_mi355x_X.so")
ap.add_argument("--raw", action="store_true", help="print raw outputs (diagnostic variants)")
a = ap.parse_args()
if a.lib:
    fa.LIB_PATH = os.path.join(os.path.dirname(fa.LIB_PATH), f"libfa_mi355x_{a.lib}.so")
torch.manual_seed(0)
S, H = a.seq, a.heads
shape = (1, H, S, 128)


def ref(q, k, v):
    sc = q.float() @ k.float().transpose(-1, -2) / 128 ** 0.5
    if a.causal:
        sc = sc + torch.full((S, S), float("-inf"), device="cuda").triu(1)
    return torch.softmax(sc, -1) @ v.float()


def report(name, q, k, v):
    o = fa.flash_attention_fwd(q, k, v, causal=a.causal, config=a.config).float()
    r = ref(q, k, v)
    err = (o - r).abs()[0, 0]
    nb = (S + 15) // 16
    rows = [err[16 * i:16 * i + 16].max().item() for i in range(nb)]
    cols = [err[:, 16 * j:16 * j + 16].max().item() for j in range(8)]
    print(f"== {name}: max err {err.max().item():.3e}  nan {torch.isnan(o).any().item()}")
    print("   by 16-row block:", " ".join(f"{x:.0e}" for x in rows))
    print("   by 16-col block:", " ".join(f"{x:.0e}" for x in cols))
    # first bad row, its first values
    bad = (err > 1e-2).any(-1).nonzero()
    if len(bad):
        i = bad[0].item()
        print(f"   first bad row {i}: got {o[0, 0, i, :6].tolist()}")
        print(f"   {'':16s} want {r[0, 0, i, :6].tolist()}")
    if a.base >= 0:
        b = fa.flash_attention_fwd(q, k, v, causal=a.causal, config=a.base).float()
        d = (o - b).abs()[0, 0]
        print("   vs base by 16-row block:", " ".join(f"{d[16 * i:16 * i + 16].max().item():.0e}" for i in range(nb)))


def rnd():
    return torch.empty(shape, dtype=torch.float16, device="cuda").uniform_(-0.5, 0.5)


q, k, v = rnd(), rnd(), rnd()
if a.raw:
    z = torch.zeros_like(q)
    for name, args in (("q0k0v1", (z, z, torch.ones_like(v))), ("rand_v1", (q, k, torch.ones_like(v)))):
        o = fa.flash_attention_fwd(*args, causal=a.causal, config=a.config).float()[0, 0]
        print(f"== {a.lib} {name}: col0 per 16-row block:",
              " ".join(f"{o[16 * i:16 * i + 16, 0].mean().item():.4g}" for i in range((S + 15) // 16)))
        print(f"   row 0 cols 0..7: {o[0, :8].tolist()}   row 17: {o[17, :8].tolist()}")
    sys.exit(0)
report("ones_v", q, k, torch.ones_like(v))
report("zero_q", torch.zeros_like(q), k, v)
report("zero_q_zero_k", torch.zeros_like(q), torch.zeros_like(k), v)
vrow = (torch.arange(S, device="cuda", dtype=torch.float32) / S)[None, None, :, None].expand(shape)
report("vrow_zero_q", torch.zeros_like(q), k, vrow.half().contiguous())
report("vrow", q, k, vrow.half().contiguous())
report("rand", q, k, v)
