"""Max-abs error of every fp16 / bf16 tile config and of PyTorch SDPA against a
torch fp32 reference on the same 16-bit inputs (S=512/2048, both masks, Q,K x1 and x4).
usage: python tools/dtype_error.py   (output: profiles/r01_dtype_error.jsonl)"""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import fa_mi355x as fa
def ref(q, k, v, causal):
    q, k, v = q.float(), k.float(), v.float()
    s = (q @ k.transpose(-1, -2)) / 128 ** 0.5
    if causal:
        n = q.shape[-2]
        s = s.masked_fill(~torch.ones(n, n, device="cuda", dtype=torch.bool).tril(), float("-inf"))
    return torch.softmax(s, -1) @ v
for s in (512, 2048):
    for causal in (False, True):
        for sc in (1.0, 4.0):
            g = torch.Generator(device="cuda"); g.manual_seed(1)
            q, k, v = (torch.empty((1, 8, s, 128), device="cuda").uniform_(-0.5, 0.5, generator=g) for _ in range(3))
            q, k = q * sc, k * sc
            for dt in (torch.float16, torch.bfloat16):
                qq, kk, vv = q.to(dt), k.to(dt), v.to(dt)
                r = ref(qq, kk, vv, causal)
                errs = {}
                for c in fa.configs():
                    if c.causal != causal or c.split_kv or c.dtype != str(dt).split(".")[1]:
                        continue
                    o = fa.flash_attention_fwd(qq, kk, vv, causal, config=c.id)
                    errs[c.name] = float((o.float() - r).abs().max())
                sd = torch.nn.functional.scaled_dot_product_attention(qq, kk, vv, is_causal=causal)
                print(json.dumps({"seq": s, "causal": causal, "qk_scale": sc, "dtype": str(dt),
                                  "max_err_worst_config": max(errs.values()),
                                  "sdpa_max_err": float((sd.float() - r).abs().max())}))
