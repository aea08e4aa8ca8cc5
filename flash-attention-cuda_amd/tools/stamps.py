"""Phase-stamp diagnostic (loads lib/libfa_mi355x_stamps.so, NOT the product lib).
usage: python tools/stamps.py --config 6 --seq 8192 [--causal] [--batch B]
Prints per-wave mean cycles per loop iteration in: MFMA block, barrier-1, softmax block, barrier-2."""
import argparse
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import fa_mi355x as fa  # noqa: E402

fa.LIB_PATH = os.path.join(HERE, "lib", os.environ.get("FA_STAMPS_LIB", "libfa_mi355x_stamps.so"))
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, required=True)
ap.add_argument("--seq", type=int, default=8192)
ap.add_argument("--batch", type=int, default=1)
ap.add_argument("--heads", type=int, default=32)
ap.add_argument("--causal", action="store_true")
a = ap.parse_args()
lib = fa.load_library()
lib.fa_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * 96)()
shape = (a.batch, a.heads, a.seq, 128)
q, k, v = (torch.empty(shape, dtype=torch.float16, device="cuda").uniform_(-0.5, 0.5) for _ in range(3))
fa.flash_attention_fwd(q, k, v, a.causal, config=a.config)
torch.cuda.synchronize()
lib.fa_debug_stamps(buf, 1)
fa.flash_attention_fwd(q, k, v, a.causal, config=a.config)
torch.cuda.synchronize()
lib.fa_debug_stamps(buf, 1)
print("wave  mfma_blk  bar1  softmax  bar2  lds_write | issue_tile  (cycles per iteration, first 64 "
      "workgroups) | prologue  epilogue (cycles per item)")
for w in range(8):
    iters = max(1, buf[w * 12 + 6])
    items = max(1, buf[w * 12 + 9])
    vals = [buf[w * 12 + i] / iters for i in range(6)]
    print(w, " ".join(f"{x:9.0f}" for x in vals[:5]), f" total {sum(vals[:5]):.0f} |", f"{vals[5]:.0f}",
          f" iters {iters} | {buf[w * 12 + 7] / items:.0f} {buf[w * 12 + 8] / items:.0f}  items {items}"
          f" | load-wait in lds_write {buf[w * 12 + 10] / iters:.0f}"
          f" | epi-pre-wait {buf[w * 12 + 11] / items:.0f}")
