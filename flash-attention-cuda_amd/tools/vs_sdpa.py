"""Head-to-head on one MI355X: torch.ops.fa_mi355x.fwd vs PyTorch
scaled_dot_product_attention (fp16, BHSD, D=128) over the reference's sweep
(flash_attention.cu:888-896 shapes, B=1 H=32) plus the B=64 S=4096 causal
headline.  Each line reports TFLOP/s by the reference formula for both, the
SDPA backend PyTorch used, and the max-abs difference between the outputs.
usage: python tools/vs_sdpa.py [--seqs 512,1024,...] [--iters 20]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import fa_mi355x as fa  # noqa: E402
import fa_mi355x.torch_op  # noqa: E402,F401  (registers torch.ops.fa_mi355x.fwd)

ap = argparse.ArgumentParser()
ap.add_argument("--seqs", default="512,1024,2048,4096,8192,16384")
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--no-headline", action="store_true")
ap.add_argument("--head-dim", type=int, default=128, choices=[64, 128])
ap.add_argument("--dtype", default="fp16", choices=["fp16", "bf16"])
a = ap.parse_args()


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    en.synchronize()
    return st.elapsed_time(en) / iters


def sdpa_backend_name():
    try:
        from torch.nn.attention import SDPBackend  # noqa: F401
        return "auto (flash/efficient/math as PyTorch selects)"
    except ImportError:
        return "auto"


def run(b, h, s, causal):
    g = torch.Generator(device="cuda")
    g.manual_seed(42)
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float16
    q, k, v = (torch.empty((b, h, s, a.head_dim), dtype=dt, device="cuda")
               .uniform_(-0.5, 0.5, generator=g) for _ in range(3))
    flops = fa.attention_flops(b, h, s, a.head_dim, causal)
    iters = max(3, min(a.iters, int(2e13 / flops)))
    ours = torch.ops.fa_mi355x.fwd(q, k, v, causal)
    row = {"batch": b, "heads": h, "seq": s, "head_dim": a.head_dim, "dtype": a.dtype,
           "causal": causal}
    ms = timed(lambda: torch.ops.fa_mi355x.fwd(q, k, v, causal), iters)
    row["fa_mi355x_tflops"] = round(flops / ms / 1e9, 1)
    try:
        ref = F.scaled_dot_product_attention(q, k, v, is_causal=causal)
        ms2 = timed(lambda: F.scaled_dot_product_attention(q, k, v, is_causal=causal), iters)
        row["sdpa_tflops"] = round(flops / ms2 / 1e9, 1)
        row["speedup_vs_sdpa"] = round(ms2 / ms, 3)
        row["max_abs_diff_vs_sdpa"] = float((ours.float() - ref.float()).abs().max())
    except Exception as e:  # SDPA unavailable / out of memory: report, keep going
        row["sdpa_error"] = repr(e)[:200]
    return row


print(json.dumps({"torch": torch.__version__, "hip": torch.version.hip,
                  "device": torch.cuda.get_device_name(0), "sdpa": sdpa_backend_name()}), flush=True)
for s in [int(x) for x in a.seqs.split(",")]:
    for causal in (False, True):
        print(json.dumps(run(1, 32, s, causal)), flush=True)
if not a.no_headline:
    print(json.dumps(run(64, 32, 4096, True)), flush=True)
