"""Host-side cost per call of each entry path, on a shape whose kernel is far
shorter than the call (B=1 H=1 S=128, D=128): what a short launch pays before
the GPU sees it.  Prints one JSON line per path (microseconds per call, wall
clock over N back-to-back calls, then one synchronize).

usage: python tools/host_overhead.py [--calls 3000]"""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import fa_mi355x as fa  # noqa: E402
import fa_mi355x.torch_op  # noqa: E402,F401

ap = argparse.ArgumentParser()
ap.add_argument("--calls", type=int, default=3000)
ap.add_argument("--seq", type=int, default=128)
a = ap.parse_args()

q, k, v = (torch.randn(1, 1, a.seq, 128, dtype=torch.float16, device="cuda") for _ in range(3))
o = torch.empty_like(q)
lib = fa.load_library()
raw = (ctypes.c_void_p(q.data_ptr()), ctypes.c_void_p(k.data_ptr()), ctypes.c_void_p(v.data_ptr()),
       ctypes.c_void_p(o.data_ptr()), 1, 1, a.seq, 128, 1,
       ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))

# the same op registered through torch.library.custom_op (the round-1
# registration), to price custom_op's own dispatch layers
@torch.library.custom_op("fa_mi355x_customop::fwd", mutates_args=())
def _customop(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = False) -> torch.Tensor:
    return fa.flash_attention_fwd(q, k, v, causal)


paths = {
    "c_abi_ctypes_raw": lambda: lib.fa_fwd_f16(*raw),
    "flash_attention_fwd(out=)": lambda: fa.flash_attention_fwd(q, k, v, True, out=o),
    "flash_attention_fwd": lambda: fa.flash_attention_fwd(q, k, v, True),
    "torch.ops.fa_mi355x.fwd": lambda: torch.ops.fa_mi355x.fwd(q, k, v, True),
    "torch.ops.fa_mi355x_customop.fwd (custom_op twin)": lambda: torch.ops.fa_mi355x_customop.fwd(q, k, v, True),
    "sdpa": lambda: F.scaled_dot_product_attention(q, k, v, is_causal=True),
}
for name, fn in paths.items():
    for _ in range(200):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.calls):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(json.dumps({"path": name, "seq": a.seq, "host_us_per_call": round((t1 - t0) / a.calls * 1e6, 2),
                      "wall_us_per_call": round((t2 - t0) / a.calls * 1e6, 2)}), flush=True)
