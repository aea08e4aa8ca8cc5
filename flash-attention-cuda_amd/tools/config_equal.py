"""Bit-identity of two forced configs of one library on given shapes (e.g. the
W4P single-block grouping against the pairs: the same per-block arithmetic in
another workgroup grouping), plus each one's max-abs error against fp32 torch.
usage: python tools/config_equal.py --pairs 65:49,64:48 --shapes 1:32:512:1,2:3:1000:1 [--dtypes fp16,bf16]
       [--head-dims 128,64]
A pair's ids name the fp16 head_dim-128 configs; bf16 / head_dim-64 runs use
their twins.  One JSON line per case; exit status 1 on any mismatch."""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import torch  # noqa: E402

import fa_mi355x as fa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pairs", required=True, help="A:B[,...]")
ap.add_argument("--shapes", required=True, help="B:H:S:causal[,...]")
ap.add_argument("--dtypes", default="fp16")
ap.add_argument("--head-dims", default="128")
a = ap.parse_args()
cs = fa.configs()
by_name = {c.name: c.id for c in cs}


def twin(cid, bf16, d):
    return by_name[("bf16_" if bf16 else "") + ("d64_" if d == 64 else "") + cs[cid].name]


bad = 0
for pr in a.pairs.split(","):
    ca, cb = (int(x) for x in pr.split(":"))
    for sh in a.shapes.split(","):
        b, h, s, c = (int(x) for x in sh.split(":"))
        if bool(c) != cs[ca].causal:
            continue
        for d in (int(x) for x in a.head_dims.split(",")):
            for dts in a.dtypes.split(","):
                bf = dts == "bf16"
                dt = torch.bfloat16 if bf else torch.float16
                g = torch.Generator(device="cuda")
                g.manual_seed(b * 1000003 + h * 1009 + s + d)
                q, k, v = (torch.empty((b, h, s, d), dtype=torch.float32, device="cuda")
                           .uniform_(-0.5, 0.5, generator=g).to(dt) for _ in range(3))
                outs = []
                for cid in (ca, cb):
                    o = torch.full_like(q, float("nan"))
                    fa.flash_attention_fwd(q, k, v, bool(c), out=o, config=twin(cid, bf, d))
                    outs.append(o)
                ref = torch.nn.functional.scaled_dot_product_attention(
                    q.float(), k.float(), v.float(), is_causal=bool(c))
                torch.cuda.synchronize()
                same = torch.equal(outs[0], outs[1])
                bad += 0 if same else 1
                print(json.dumps({"pair": pr, "shape": sh, "head_dim": d, "dtype": dts, "identical": same,
                                  "differing_elements": 0 if same else int((outs[0] != outs[1]).sum().item()),
                                  "err_a": float((outs[0].float() - ref).abs().max()),
                                  "err_b": float((outs[1].float() - ref).abs().max())}), flush=True)
sys.exit(1 if bad else 0)
