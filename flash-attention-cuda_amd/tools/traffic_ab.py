#!/usr/bin/env python3
"""HBM traffic of library variants on given shapes (rocprofv3 --pmc, one pass
per counter as MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE x1024 x2 +
WRITE_SIZE x1024 per launch, first dispatch dropped).

usage: python tools/traffic_ab.py --libs ,snake --config 7 --shapes 1x32x8192,1x32x16384 --causal
Prints one JSON line per (lib, shape): bytes per launch and the ratio to the
algorithmic bytes 8*B*H*S*D (Q, K, V read once, O written once)."""
import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def child(a):
    import torch

    import fa_mi355x as fa

    fa._lib = None
    fa.LIB_PATH = os.path.join(HERE, "lib", "libfa_mi355x%s.so" % ("_" + a.lib if a.lib else ""))
    fa.load_library()
    b, h, s = (int(x) for x in a.shapes.split("x"))
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    q, k, v = (torch.empty((b, h, s, 128), dtype=torch.float16, device="cuda").uniform_(-0.5, 0.5, generator=g)
               for _ in range(3))
    o = torch.empty_like(q)
    for _ in range(a.iters):
        fa.flash_attention_fwd(q, k, v, a.causal, out=o, config=None if a.config == "auto" else int(a.config))
    torch.cuda.synchronize()


def counter(root, name):
    per = {}
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "fa_fwd" in r["Kernel_Name"] and r["Counter_Name"] == name:
                    d = int(r["Dispatch_Id"])
                    per[d] = per.get(d, 0.0) + float(r["Counter_Value"])
    vals = [per[d] for d in sorted(per)][1:]
    return sum(vals) / len(vals) if vals else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="")
    ap.add_argument("--config", required=True, help="tile config id, or auto (the default dispatch: "
                    "workspace path, tail pool)")
    ap.add_argument("--shapes", required=True, help="BxHxS[,BxHxS...]")
    ap.add_argument("--causal", action="store_true")
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--lib", default="")
    a = ap.parse_args()
    if a.child:
        child(a)
        return
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    for shape in a.shapes.split(","):
        b, h, s = (int(x) for x in shape.split("x"))
        alg = 8.0 * b * h * s * 128
        for lib in a.libs.split(","):
            got = {}
            for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
                with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
                    cmd = ["timeout", "-s", "KILL", "120", prof, "--pmc", ctr, "-d", td, "--output-format",
                           "csv", "--", sys.executable, os.path.abspath(__file__), "--child", "--lib", lib,
                           "--config", a.config, "--shapes", shape, "--iters", str(a.iters)]
                    if a.causal:
                        cmd.append("--causal")
                    r = subprocess.run(cmd, capture_output=True, text=True)
                    if r.returncode != 0:
                        print(json.dumps({"lib": lib, "shape": shape, "error": r.stderr[-400:]}), flush=True)
                        sys.exit(1)
                    got[ctr] = counter(td, ctr)
            tb = got["FETCH_SIZE"] * 2048 + got["WRITE_SIZE"] * 1024
            print(json.dumps({"lib": lib or "base", "config": a.config, "shape": shape, "causal": a.causal,
                              "fetch_bytes": int(got["FETCH_SIZE"] * 2048),
                              "write_bytes": int(got["WRITE_SIZE"] * 1024), "traffic_bytes": int(tb),
                              "algorithmic_bytes": int(alg), "traffic_over_algorithmic": round(tb / alg, 3)}),
                  flush=True)


if __name__ == "__main__":
    main()
