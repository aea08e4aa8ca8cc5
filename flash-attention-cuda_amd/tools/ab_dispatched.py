#!/usr/bin/env python3
"""Same-process A/B (tools/ab.py) of library variants on the config the
dispatcher picks for each shape.

usage: python tools/ab_dispatched.py --libs ,X  BxHxS[c] ...   (c = causal)"""
import argparse
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

import fa_mi355x as fa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--libs", required=True)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--iters", type=int, default=50)
ap.add_argument("shapes", nargs="+")
a = ap.parse_args()
for sh in a.shapes:
    causal = sh.endswith("c")
    b, h, s = (int(x) for x in sh.rstrip("c").split("x"))
    cid = fa.select_config(b, h, s, causal)
    cmd = ["timeout", "-k", "10", "150", sys.executable, os.path.join(HERE, "tools", "ab.py"),
           "--configs", str(cid), "--batch", str(b), "--heads", str(h), "--seq", str(s),
           "--libs", a.libs, "--rounds", str(a.rounds), "--iters", str(a.iters)]
    if causal:
        cmd.append("--causal")
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        print(r.stderr[-500:], file=sys.stderr)
        sys.exit(r.returncode)
    print(r.stdout.strip(), flush=True)
