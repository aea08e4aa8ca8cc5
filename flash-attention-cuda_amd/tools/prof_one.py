"""Run one tile config N times (for rocprofv3 counter/trace passes).
usage: python tools/prof_one.py --config ID --seq S [--causal] [--heads H] [--batch B] [--iters N]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import fa_mi355x as fa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=None)
ap.add_argument("--seq", type=int, default=8192)
ap.add_argument("--heads", type=int, default=32)
ap.add_argument("--batch", type=int, default=1)
ap.add_argument("--causal", action="store_true")
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()
g = torch.Generator(device="cuda")
g.manual_seed(1)
shape = (a.batch, a.heads, a.seq, 128)
q, k, v = (torch.empty(shape, dtype=torch.float16, device="cuda").uniform_(-0.5, 0.5, generator=g)
           for _ in range(3))
o = torch.empty_like(q)
for _ in range(a.iters):
    fa.flash_attention_fwd(q, k, v, a.causal, out=o, config=a.config)
torch.cuda.synchronize()
print("done", fa.configs()[a.config if a.config is not None else
                          fa.select_config(a.batch, a.heads, a.seq, a.causal)].name)
