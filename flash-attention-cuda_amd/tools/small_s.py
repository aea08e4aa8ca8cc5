"""Short-sequence study: every non-split config vs split-KV (auto and forced
split counts) at B=1 H=32, S in {512, 1024, 2048}, both masks.
usage: python tools/small_s.py [--seqs 512,1024,2048] [--iters 50]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import fa_mi355x as fa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--seqs", default="512,1024,2048")
ap.add_argument("--heads", type=int, default=32)
ap.add_argument("--iters", type=int, default=50)
a = ap.parse_args()


def timed(fn):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(a.iters):
        fn()
    en.record()
    en.synchronize()
    return st.elapsed_time(en) / a.iters


for s in [int(x) for x in a.seqs.split(",")]:
    for causal in (False, True):
        shape = (1, a.heads, s, 128)
        q, k, v = (torch.empty(shape, dtype=torch.float16, device="cuda").uniform_(-0.5, 0.5)
                   for _ in range(3))
        o = torch.empty_like(q)
        flops = fa.attention_flops(1, a.heads, s, 128, causal)
        res = {}
        for c in fa.configs():
            if c.causal != causal or c.split_kv:
                continue
            ms = timed(lambda: fa.flash_attention_fwd(q, k, v, causal, out=o, config=c.id))
            res[c.name] = round(flops / ms / 1e9, 1)
        auto = fa.load_library().fa_splitkv_num_splits(1, a.heads, s, int(causal))
        for ns in sorted({auto, 2, 4, 8, 16}):
            po, pml = fa.splitkv_buffers(1, a.heads, s, ns)
            ms = timed(lambda: fa.flash_attention_fwd_splitkv(q, k, v, causal, ns, out=o,
                                                              part_o=po, part_ml=pml))
            res[f"splitkv{ns}{'(auto)' if ns == auto else ''}"] = round(flops / ms / 1e9, 1)
        sel = fa.configs()[fa.select_config(1, a.heads, s, causal)].name
        print(json.dumps({"seq": s, "causal": causal, "selected": sel, "tflops": res}), flush=True)
