#!/usr/bin/env python3
"""Average kernel duration over the TIMED launches of a bench run under
`rocprofv3 --kernel-trace` (the last --steps dispatches of the headline
kernel; the warm-up dispatches, the first of them cold, are dropped), beside
the bench line's own ms_per_step from the same run.

    python tools/kt_timed_avg.py <kt_kernel_trace.csv> <bench_under_kt.json> [substr]
"""
import csv
import json
import sys


def main():
    trace, bench = sys.argv[1], sys.argv[2]
    with open(bench) as f:
        line = json.loads(f.read().strip().splitlines()[-1])
    substr = sys.argv[3] if len(sys.argv) > 3 else line["roofline"]["kernel"].split()[0]
    with open(trace) as f:
        rows = [r for r in csv.DictReader(f) if substr in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    k = line["steps"]
    timed = ms[-k:]
    out = {
        "kernel": substr,
        "dispatches": len(ms),
        "timed_dispatches": len(timed),
        "avg_ms_all": round(sum(ms) / len(ms), 4),
        "avg_ms_timed": round(sum(timed) / len(timed), 4),
        "bench_ms_per_step": line["ms_per_step"],
        "bench_avg_launch_ms_hip_events": line["roofline"]["avg_launch_ms"],
        "timed_avg_le_ms_per_step": sum(timed) / len(timed) <= line["ms_per_step"],
        "source_digest": line["roofline"].get("source_digest"),
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
