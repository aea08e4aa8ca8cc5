"""Run one causal shape N times on a chosen library variant (for a rocprofv3
--pmc FETCH_SIZE pass comparing variants).
usage: python tools/lib_fetch.py VARIANT|base B H S [iters]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import fa_mi355x as fa  # noqa: E402

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
var, b, h, s = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 4
fa._lib = None
fa.LIB_PATH = os.path.join(HERE, "lib", "libfa_mi355x%s.so" % ("" if var == "base" else "_" + var))
fa.load_library()
q, k, v = (torch.empty(b, h, s, 128, dtype=torch.float16, device="cuda").uniform_(-0.5, 0.5) for _ in range(3))
o = torch.empty_like(q)
for _ in range(iters):
    fa.flash_attention_fwd(q, k, v, True, out=o)
torch.cuda.synchronize()
print("done", var)
