"""Interleaved A/B timing of tile configs in ONE process (guide §5.4 rule 24).
usage: python tools/ab.py --configs 2,6 --seq 8192 [--causal] [--batch B] [--heads H]
       [--rounds 7] [--iters 30]
Prints per-config median / min TFLOPS over rounds (random uniform[-0.5,0.5] fp16)."""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import fa_mi355x as fa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--configs", required=True)
ap.add_argument("--seq", type=int, default=8192)
ap.add_argument("--heads", type=int, default=32)
ap.add_argument("--batch", type=int, default=1)
ap.add_argument("--causal", action="store_true")
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--iters", type=int, default=30)
ap.add_argument("--env", default="", help="label only")
ap.add_argument("--dtype", default="fp16", choices=["fp16", "bf16"])
ap.add_argument("--head-dim", type=int, default=128, choices=[64, 128])
ap.add_argument("--data", default="uniform", choices=["uniform", "zeros", "small"],
                help="uniform[-0.5,0.5] (default), all zeros, or uniform[-0.01,0.01]")
ap.add_argument("--libs", default="", help="comma list of library variants: '' = libfa_mi355x.so, "
                "X = libfa_mi355x_X.so; every config is timed against every variant")
a = ap.parse_args()
g = torch.Generator(device="cuda")
g.manual_seed(3)
shape = (a.batch, a.heads, a.seq, a.head_dim)
dt = torch.bfloat16 if a.dtype == "bf16" else torch.float16
q, k, v = (torch.empty(shape, dtype=dt, device="cuda").uniform_(-0.5, 0.5, generator=g)
           for _ in range(3))
if a.data == "zeros":
    for t in (q, k, v):
        t.zero_()
elif a.data == "small":
    for t in (q, k, v):
        t.mul_(0.02)
o = torch.empty_like(q)
HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
libs = {}
for var in a.libs.split(","):
    fa._lib = None
    fa.LIB_PATH = os.path.join(HERE, "lib", "libfa_mi355x%s.so" % ("_" + var if var else ""))
    libs[var] = fa.load_library()
# "auto": the default dispatch (flash_attention_fwd with config=None: the
# workspace split tier where it applies)
# "static": the workspace-free C entry (fa_fwd_f16 / fa_fwd_bf16: the W4 tier's
# static item order, no tail pool)
cids = [(var, None if x == "auto" else x if x == "static" else int(x)) for x in a.configs.split(",")
        for var in libs]


def fwd(c):
    if c[1] != "static":
        fa.flash_attention_fwd(q, k, v, a.causal, out=o, config=c[1])
        return
    fn = fa._lib.fa_fwd_bf16 if dt == torch.bfloat16 else fa._lib.fa_fwd_f16
    fn(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), a.batch, a.heads, a.seq, a.head_dim,
       int(a.causal), torch.cuda.current_stream().cuda_stream)
flops = fa.attention_flops(a.batch, a.heads, a.seq, a.head_dim, a.causal)
res = {c: [] for c in cids}
for c in cids:  # warm
    fa._lib = libs[c[0]]
    for _ in range(5):
        fwd(c)
torch.cuda.synchronize()
for _ in range(a.rounds):
    for c in cids:
        fa._lib = libs[c[0]]
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(a.iters):
            fwd(c)
        en.record()
        en.synchronize()
        res[c].append(flops / (st.elapsed_time(en) / a.iters / 1e3) / 1e12)
names = {c.id: c.name for c in fa.configs()}
names["static"] = "static (fa_fwd_f16, no workspace)"
names[None] = "auto(split=%d)" % fa.load_library().fa_fwd_split_pieces(a.batch, a.heads, a.seq, a.head_dim, int(a.causal))
for c in cids:
    print(json.dumps({"config": names[c[1]], "lib": c[0] or "base", "env": a.env, "seq": a.seq, "head_dim": a.head_dim, "batch": a.batch, "heads": a.heads, "data": a.data, "causal": a.causal,
                      "median_tflops": round(statistics.median(res[c]), 1),
                      "min_tflops": round(min(res[c]), 1), "max_tflops": round(max(res[c]), 1)}))
