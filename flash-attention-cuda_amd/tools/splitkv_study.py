"""Where split-KV (flash-decoding style key split + LSE merge, the reference's
dead split-K path :169-180/:559-598) pays: few heads, long sequences.
Times the dispatcher's pick against fa_fwd_f16_splitkv (auto and forced split
counts; buffers allocated once, outside the timed loop).
usage: python tools/splitkv_study.py [--iters 10]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import fa_mi355x as fa  # noqa: E402

ap = argparse.ArgumentParser()
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


for b, h, s in ((1, 1, 16384), (1, 4, 16384), (1, 8, 8192), (1, 2, 32768), (1, 32, 4096)):
    for causal in (False, True):
        shape = (b, h, s, 128)
        q, k, v = (torch.empty(shape, dtype=torch.float16, device="cuda").uniform_(-0.5, 0.5)
                   for _ in range(3))
        o = torch.empty_like(q)
        flops = fa.attention_flops(b, h, s, 128, causal)
        res = {"batch": b, "heads": h, "seq": s, "causal": causal,
               "dispatch": fa.configs()[fa.select_config(b, h, s, causal)].name}
        res["dispatch_tflops"] = round(
            flops / timed(lambda: fa.flash_attention_fwd(q, k, v, causal, out=o)) / 1e9, 1)
        auto = fa.load_library().fa_splitkv_num_splits(b, h, s, int(causal))
        for n in sorted({auto, 4, 8, 16}):
            po, pml = fa.splitkv_buffers(b, h, s, n)
            ms = timed(lambda: fa.flash_attention_fwd_splitkv(q, k, v, causal, num_splits=n, out=o,
                                                             part_o=po, part_ml=pml))
            res[f"splitkv{n}{'(auto)' if n == auto else ''}_tflops"] = round(flops / ms / 1e9, 1)
            del po, pml
        print(json.dumps(res), flush=True)
