"""Turn the rocprofv3 FETCH_SIZE / WRITE_SIZE passes of bench.py into the
per-launch HBM traffic summary bench.py reports as roofline.traffic.

usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR OUT_JSON

Per MI355X_MICROARCH.md §HBM: counters come from separate --pmc passes,
FETCH_SIZE / WRITE_SIZE are in KiB, and gfx950 FETCH_SIZE reports half the
bytes of wide streaming reads (x2).  The first (cold) dispatch is dropped."""
import csv
import glob
import json
import os
import sys

KERNEL = "fa_fwd_f16"  # fa_fwd_f16_kernel or fa_fwd_f16_persistent_kernel
WORKLOAD = "b64_h32_s4096_d128_causal"


def mean_counter(root, name):
    files = glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {root}")
    per = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if KERNEL not in r["Kernel_Name"] or r["Counter_Name"] != name:
                continue
            d = int(r["Dispatch_Id"])
            per[d] = per.get(d, 0.0) + float(r["Counter_Value"])
    vals = [per[d] for d in sorted(per)]
    if len(vals) > 1:
        vals = vals[1:]
    return sum(vals) / len(vals), len(vals)


def main():
    fetch_dir, write_dir, out = sys.argv[1:4]
    fetch_kib, nf = mean_counter(fetch_dir, "FETCH_SIZE")
    write_kib, nw = mean_counter(write_dir, "WRITE_SIZE")
    fetch_b = fetch_kib * 1024 * 2
    write_b = write_kib * 1024
    d = {
        "workload": WORKLOAD,
        "kernel": KERNEL,
        "hbm_bytes_per_launch": int(fetch_b + write_b),
        "fetch_bytes_per_launch": int(fetch_b),
        "write_bytes_per_launch": int(write_b),
        "fetch_size_kib_raw": fetch_kib,
        "write_size_kib_raw": write_kib,
        "dispatches": [nf, nw],
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes of "
                  "bench.py --steps 3 --warmup 1 --no-sweep --no-cpu-baseline; mean over "
                  "dispatches 2..N; FETCH x1024 x2 (gfx950 half-count), WRITE x1024",
    }
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
    import bench

    d["source_digest"] = bench.source_digest()
    d["git_head"] = os.environ.get("GIT_HEAD")
    with open(out, "w") as f:
        json.dump(d, f, indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
