"""Per-config TFLOPS sweep (the reference's bench loop, flash_attention.cu:886-971:
20 warm-up + 100 timed launches x 3 runs, event-timed, TFLOPS = 4*B*H*S^2*D (/2 causal)).
Usage: python tools/sweep.py [--seqs 512,1024,...] [--heads 32] [--batch 1] [--configs all|auto]
Prints one JSON line per (mode, seq, config)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import fa_mi355x as fa  # noqa: E402

PEAK_TFLOPS = 256 * 2.4e9 * 4096 / 1e12  # 256 CU x 2.4 GHz x 4096 fp16 FLOP/clk/CU


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seqs", default="512,768,1024,2048,4096,8192,16384")
    ap.add_argument("--heads", type=int, default=32)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--configs", default="auto")
    ap.add_argument("--modes", default="noncausal,causal")
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--runs", type=int, default=3)
    a = ap.parse_args()
    g = torch.Generator(device="cuda")
    g.manual_seed(42)
    for mode in a.modes.split(","):
        causal = mode == "causal"
        for s in [int(x) for x in a.seqs.split(",")]:
            shape = (a.batch, a.heads, s, 128)
            q = (torch.rand(shape, generator=g, device="cuda") - 0.5).half()
            k = (torch.rand(shape, generator=g, device="cuda") - 0.5).half()
            v = (torch.rand(shape, generator=g, device="cuda") - 0.5).half()
            o = torch.empty_like(q)
            if a.configs == "auto":
                cids = [None]
            elif a.configs == "all":
                cids = [c.id for c in fa.configs() if c.causal == causal and not c.split_kv]
            else:
                cids = [int(x) for x in a.configs.split(",")]
            flops = fa.attention_flops(a.batch, a.heads, s, 128, causal)
            for cid in cids:
                runs = []
                for _ in range(a.runs):
                    for _ in range(20):
                        fa.flash_attention_fwd(q, k, v, causal, out=o, config=cid)
                    torch.cuda.synchronize()
                    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    st.record()
                    for _ in range(a.iters):
                        fa.flash_attention_fwd(q, k, v, causal, out=o, config=cid)
                    en.record()
                    en.synchronize()
                    ms = st.elapsed_time(en) / a.iters
                    runs.append(flops / (ms / 1e3) / 1e12)
                used = cid if cid is not None else fa.select_config(a.batch, a.heads, s, causal)
                avg = sum(runs) / len(runs)
                print(json.dumps({"mode": mode, "seq": s, "heads": a.heads, "batch": a.batch,
                                  "config": fa.configs()[used].name,
                                  "tflops": [round(x, 1) for x in runs], "avg_tflops": round(avg, 1),
                                  "pct_peak": round(100 * avg / PEAK_TFLOPS, 1)}), flush=True)
            del q, k, v, o


if __name__ == "__main__":
    main()
