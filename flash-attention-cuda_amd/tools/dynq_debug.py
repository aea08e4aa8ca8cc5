"""Diagnostic for the dynamic-queue experiment build (lib/libfa_mi355x_dyndbg.so):
items processed per launch vs the item count, and workgroups whose hardware
XCC id differs from blockIdx & 7."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import fa_mi355x as fa  # noqa: E402

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
fa._lib = None
fa.LIB_PATH = os.path.join(HERE, "lib", "libfa_mi355x_dyndbg.so")
lib = fa.load_library()
lib.fa_debug_dynq.argtypes = [ctypes.POINTER(ctypes.c_uint)]
out = (ctypes.c_uint * 3)()
for b, h, s in ((64, 32, 4096), (1, 32, 8192), (8, 32, 4096)):
    q, k, v = (torch.randn(b, h, s, 128, dtype=torch.float16, device="cuda") * 0.3 for _ in range(3))
    o = torch.empty_like(q)
    lib.fa_debug_dynq(out)  # clear
    for it in range(3):
        fa.flash_attention_fwd(q, k, v, True, out=o)
        torch.cuda.synchronize()
        lib.fa_debug_dynq(out)
        items = b * h * ((s + 255) // 256)
        print(f"B={b} H={h} S={s} launch {it}: processed {out[0]} of {items} items, "
              f"workgroups {out[2]}, xcc != blockIdx&7: {out[1]}", flush=True)
