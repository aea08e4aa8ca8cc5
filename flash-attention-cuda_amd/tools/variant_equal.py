"""Bit-identity of a library variant against the product on given shapes, in
ONE process (both libraries loaded): a schedule-only change (e.g. the W4
program's two-tiles-per-barrier form) must not change a single output bit.
usage: python tools/variant_equal.py --lib dbl --shapes 1:32:8192:1,2:8:1000:0 [--dtypes fp16,bf16]
       [--head-dims 128,64] [--config auto|ID]
One JSON line per case; exit status 1 on any mismatch."""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import torch  # noqa: E402

import fa_mi355x as fa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", required=True)
ap.add_argument("--shapes", required=True, help="B:H:S:causal[,...]")
ap.add_argument("--dtypes", default="fp16")
ap.add_argument("--head-dims", default="128")
ap.add_argument("--config", default="auto")
ap.add_argument("--scale", type=float, default=1.0, help="inputs uniform[-scale/2, scale/2] (peaked: 6)")
a = ap.parse_args()
libs = {}
for var in ("", a.lib):
    fa._lib = None
    fa.LIB_PATH = os.path.join(HERE, "lib", "libfa_mi355x%s.so" % ("_" + var if var else ""))
    libs[var] = fa.load_library()
bad = 0
for sh in a.shapes.split(","):
    b, h, s, c = (int(x) for x in sh.split(":"))
    for d in (int(x) for x in a.head_dims.split(",")):
        for dts in a.dtypes.split(","):
            dt = torch.bfloat16 if dts == "bf16" else torch.float16
            g = torch.Generator(device="cuda")
            g.manual_seed(b * 1000003 + h * 1009 + s + d)
            q, k, v = (torch.empty((b, h, s, d), dtype=torch.float32, device="cuda")
                       .uniform_(-a.scale / 2, a.scale / 2, generator=g).to(dt) for _ in range(3))
            outs = []
            for var in ("", a.lib):
                fa._lib = libs[var]
                cfg = None if a.config == "auto" else int(a.config)
                if cfg is not None and (dt == torch.bfloat16 or d != 128):
                    # the twin of a forced fp16 head_dim-128 config for this dtype / head_dim
                    cs = fa.configs()
                    base = cs[cfg].name
                    want = ("bf16_" if dt == torch.bfloat16 else "") + ("d64_" if d == 64 else "") + base
                    cfg = next(c.id for c in cs if c.name == want)
                o = torch.full_like(q, float("nan"))
                fa.flash_attention_fwd(q, k, v, bool(c), out=o, config=cfg)
                outs.append(o)
            torch.cuda.synchronize()
            same = torch.equal(outs[0], outs[1])
            nd = int((outs[0] != outs[1]).sum().item()) if not same else 0
            bad += 0 if same else 1
            print(json.dumps({"shape": sh, "head_dim": d, "dtype": dts, "lib": a.lib, "identical": same,
                              "differing_elements": nd, "nan_free": bool(torch.isfinite(outs[1]).all())}),
                  flush=True)
sys.exit(1 if bad else 0)
