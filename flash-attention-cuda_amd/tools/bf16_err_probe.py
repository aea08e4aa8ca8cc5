"""bf16 error budget on peaked inputs (profiles/r05_bf16_peaked_err.jsonl).

For the bf16 boundary shapes of tests/test_dispatch_sweep_gpu.py at q, k
scales 1, 4 and 6, prints the max-abs error against the fp32 model of
  ours                the dispatched kernel (flash_attention_fwd)
  sdpa_bf16           PyTorch's bf16 scaled_dot_product_attention
  qc_rounding_alone   the fp32 model with Q * scale * log2(e) rounded to bf16
                      (the product every bf16 tier feeds its QK^T MFMA)
  ours_vs_qc_model    the kernel against that rounded model
usage: python tools/bf16_err_probe.py [VARIANT]   (on a GPU box)
"""
import json
import math
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "tests"))
sys.path.insert(0, os.path.join(HERE, ".."))
import torch  # noqa: E402

import test_dispatch_sweep_gpu as t  # noqa: E402

fa = t._fa()
if len(sys.argv) > 1:  # a variant library: tools/w4_variant.sh NAME ...
    fa.LIB_PATH = os.path.join(os.path.dirname(fa.LIB_PATH), f"libfa_mi355x_{sys.argv[1]}.so")
    fa._lib = None
for shape in [s for s in t.BOUNDARY if s[5]]:
    b, h, s, d, causal, _ = shape
    for scale in (1.0, 4.0, 6.0):
        q, k, v = t._inputs(b, h, s, d, torch.bfloat16, 37, scale)
        ref = t._ref(q, k, v, causal)
        model = t._ref(q, k, v, causal, qc_bf16=True)
        o = fa.flash_attention_fwd(q, k, v, causal)
        sd = torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=causal)
        err = lambda x, r: (x.float() - r).abs().max().item()  # noqa: E731
        print(json.dumps({"shape": shape, "scale": scale, "ours": err(o, ref), "sdpa_bf16": err(sd, ref),
                          "qc_rounding_alone": err(model, ref), "ours_vs_qc_model": err(o, model),
                          "head_dim_scale": 1 / math.sqrt(d)}))
