"""Per-kernel averages of rocprofv3 --pmc counter_collection.csv files (first
dispatch of each kernel dropped) and the derived wave-time split.
usage: python tools/pmc_summary.py DIR [DIR ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict

for root in sys.argv[1:]:
    files = glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(lambda: defaultdict(dict))
    dur = defaultdict(dict)
    for f in files:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            d = int(r["Dispatch_Id"])
            per[k][r["Counter_Name"]][d] = per[k][r["Counter_Name"]].get(d, 0.0) + float(r["Counter_Value"])
            dur[k][d] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for k in per:
        ds = sorted(dur[k])[1:] or sorted(dur[k])
        avg = {c: sum(v[d] for d in ds) / len(ds) for c, v in per[k].items()}
        t = sum(dur[k][d] for d in ds) / len(ds)
        print(f"== {root}  {k[-60:]}  dispatches={len(ds)}  avg {t / 1e6:.4f} ms")
        for c in sorted(avg):
            print(f"   {c:28s} {avg[c]:.4g}")
        g = avg.get("GRBM_GUI_ACTIVE")
        if g:
            print(f"   clock GHz (GRBM/8/t)         {g / 8 / t:.3f}")
            if "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
                print(f"   MFMA busy                    {avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * g / 8):.3f}")
        w = avg.get("SQ_WAVE_CYCLES")
        if w:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
                if c in avg:
                    print(f"   {c:28s} / wave cycles  {avg[c] / w:.3f}")
