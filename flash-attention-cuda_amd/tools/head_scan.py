"""Dispatcher anomaly scan: TFLOP/s of the dispatched kernel over head counts
(B=1) and sequence lengths, both masks -- a shape whose rate falls far below
its neighbours points at a mapping / tier problem.
usage: python tools/head_scan.py [--heads 1,2,3,...] [--seqs 2048,8192] [--iters 10]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import fa_mi355x as fa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--heads", default="1,2,3,4,6,8,12,16,24,32,48,64")
ap.add_argument("--seqs", default="2048,8192")
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()


def timed(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(a.iters):
        fn()
    en.record()
    en.synchronize()
    return st.elapsed_time(en) / a.iters


cfgs = fa.configs()
for s in [int(x) for x in a.seqs.split(",")]:
    for h in [int(x) for x in a.heads.split(",")]:
        q, k, v = (torch.empty((1, h, s, 128), dtype=torch.float16, device="cuda").uniform_(-0.5, 0.5)
                   for _ in range(3))
        o = torch.empty_like(q)
        for causal in (False, True):
            ms = timed(lambda: fa.flash_attention_fwd(q, k, v, causal, out=o))
            print(json.dumps({"heads": h, "seq": s, "causal": causal,
                              "config": cfgs[fa.select_config(1, h, s, causal)].name,
                              "tflops": round(fa.attention_flops(1, h, s, 128, causal) / ms / 1e9, 1)}),
                  flush=True)
        del q, k, v, o
