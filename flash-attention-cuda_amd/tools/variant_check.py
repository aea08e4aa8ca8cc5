"""Bit-identity check of a library variant against the product library on the
dispatched tiers (same inputs, same config id): a variant that only changes
scheduling or data movement must reproduce the product's output bit for bit.
usage: python tools/variant_check.py VARIANT [HEAD_DIM]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import fa_mi355x as fa  # noqa: E402

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
var = sys.argv[1]
hd = int(sys.argv[2]) if len(sys.argv) > 2 else 128
libs = {}
for v in ("", var):
    fa._lib = None
    fa.LIB_PATH = os.path.join(HERE, "lib", "libfa_mi355x%s.so" % ("_" + v if v else ""))
    libs[v] = fa.load_library()
SHAPES = [(1, 32, 4096), (2, 3, 1000), (1, 12, 8192), (1, 48, 2048), (4, 8, 4096), (1, 2, 16384),
          (1, 32, 1024), (1, 16, 2048), (1, 24, 1536), (1, 32, 512), (1, 8, 2048),
          (8, 32, 1280), (3, 5, 3333)]
g = torch.Generator(device="cuda")
g.manual_seed(11)
bad = 0
for dt in (torch.float16, torch.bfloat16):
    for b, h, s in SHAPES:
        q, k, v = (torch.empty((b, h, s, hd), dtype=dt, device="cuda").uniform_(-0.5, 0.5, generator=g)
                   for _ in range(3))
        for causal in (False, True):
            outs = []
            for key in ("", var):
                fa._lib = libs[key]
                outs.append(fa.flash_attention_fwd(q, k, v, causal))
            torch.cuda.synchronize()
            same = torch.equal(outs[0].view(torch.int16), outs[1].view(torch.int16))
            cfg = fa.configs()[fa.select_config(b, h, s, causal) if dt == torch.float16 else 0].name
            print(f"{str(dt):15s} D={hd} B={b} H={h} S={s} causal={causal} {cfg}: "
                  f"{'bit-identical' if same else 'DIFFERENT max %.3g' % (outs[0].float() - outs[1].float()).abs().max().item()}",
                  flush=True)
            bad += not same
print("variant_check", var, "FAIL" if bad else "OK", bad)
sys.exit(1 if bad else 0)
