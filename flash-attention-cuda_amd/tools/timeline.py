"""Workgroup timeline diagnostic (stamps build): per-CU busy fraction, tail, order.
usage: python tools/timeline.py --config 7 --seq 8192 --causal [--batch B]"""
import argparse
import collections
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import fa_mi355x as fa  # noqa: E402

fa.LIB_PATH = os.path.join(HERE, "lib", "libfa_mi355x_stamps.so")
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, required=True)
ap.add_argument("--seq", type=int, default=8192)
ap.add_argument("--batch", type=int, default=1)
ap.add_argument("--heads", type=int, default=32)
ap.add_argument("--causal", action="store_true")
a = ap.parse_args()
lib = fa.load_library()
lib.fa_debug_timeline.argtypes = [ctypes.c_void_p, ctypes.c_int]
cfg = fa.configs()[a.config]
nblk = a.batch * a.heads * ((a.seq + cfg.block_m - 1) // cfg.block_m)  # records: one per item
shape = (a.batch, a.heads, a.seq, 128)
q, k, v = (torch.empty(shape, dtype=torch.float16, device="cuda").uniform_(-0.5, 0.5) for _ in range(3))
for _ in range(3):
    fa.flash_attention_fwd(q, k, v, a.causal, config=a.config)
torch.cuda.synchronize()
n = min(nblk, 65536)
buf = (ctypes.c_ulonglong * (4 * n))()
lib.fa_debug_timeline(buf, n)
rows = [(buf[4 * i], buf[4 * i + 1], buf[4 * i + 2]) for i in range(n)]
clk = [buf[4 * i + 3] / max(1, buf[4 * i + 1] - buf[4 * i]) * 0.1 for i in range(n)]  # GHz
clk.sort()
print(f"  in-kernel clock (memtime/realtime): med {clk[len(clk)//2]:.3f} GHz p10 {clk[len(clk)//10]:.3f} p90 {clk[9*len(clk)//10]:.3f}")
t0 = min(r[0] for r in rows)
t1 = max(r[1] for r in rows)
span = (t1 - t0) / 100.0  # us
cu = collections.defaultdict(float)
for s_, e_, hw in rows:
    h = hw & 0xFFFFFFFF
    key = ((hw >> 32) & 0xFF, (h >> 13) & 7, (h >> 12) & 1, (h >> 8) & 15)  # xcc, se, sh, cu
    cu[key] += (e_ - s_) / 100.0
busy = sorted(cu.values())
durs = sorted((e_ - s_) / 100.0 for s_, e_, _ in rows)
ends = sorted((e_ - t0) / 100.0 for _, e_, _ in rows)
print(f"{cfg.name} seq={a.seq} batch={a.batch}: {n} workgroups on {len(cu)} CUs, span {span:.1f} us")
print(f"  CU busy: mean {sum(busy)/len(busy):.1f} us ({100*sum(busy)/len(busy)/span:.1f}%), "
      f"min {busy[0]:.1f}, max {busy[-1]:.1f}")
print(f"  workgroup duration: min {durs[0]:.2f} med {durs[len(durs)//2]:.2f} max {durs[-1]:.2f} us")
print(f"  last 1% of workgroups end after {ends[int(0.99*len(ends))]:.1f} us; "
      f"first end {ends[0]:.1f} us")

# per-CU gaps between consecutive workgroups, and duration vs query block
percu = collections.defaultdict(list)
byqb = collections.defaultdict(list)
byh = collections.defaultdict(list)
for s_, e_, hw in rows:
    h = hw & 0xFFFFFFFF
    percu[((hw >> 32) & 0xFF, (h >> 13) & 7, (h >> 12) & 1, (h >> 8) & 15)].append((s_, e_))
    byqb[(hw >> 40) & 0xFFFF].append((e_ - s_) / 100.0)
    byh[(hw >> 56) & 0xFF].append((e_ - s_) / 100.0)
gaps = []
for lst in percu.values():
    lst.sort()
    gaps += [(b[0] - a_[1]) / 100.0 for a_, b in zip(lst, lst[1:])]
gaps.sort()
if gaps:
    print(f"  gap between consecutive WGs on a CU: mean {sum(gaps)/len(gaps):.2f} "
          f"med {gaps[len(gaps)//2]:.2f} p90 {gaps[int(0.9*len(gaps))]:.2f} us")
xs = sorted(byqb)
pts = [(qb + 1, sum(v) / len(v)) for qb, v in ((x, byqb[x]) for x in xs)]
if len(pts) > 2:
    n_ = len(pts)
    mx = sum(p_[0] for p_ in pts) / n_
    my = sum(p_[1] for p_ in pts) / n_
    sl = sum((p_[0] - mx) * (p_[1] - my) for p_ in pts) / sum((p_[0] - mx) ** 2 for p_ in pts)
    print(f"  duration ~ {my - sl * mx:.2f} us + {sl:.3f} us x (qb+1)   [causal: per 256-row key step]")
    print("  qb:dur " + " ".join(f"{x}:{sum(byqb[x])/len(byqb[x]):.1f}" for x in xs[:32]))
    bys = collections.defaultdict(list)
    for s_, e_, hw in rows:
        bys[(hw >> 40) & 0xFFFF].append((s_ - t0) / 100.0)
    print("  qb:start " + " ".join(f"{x}:{sum(bys[x])/len(bys[x]):.1f}/{max(bys[x]):.1f}" for x in xs[:32]))
    # per-XCD busy: are the heavy blocks on a few XCDs / sharing CUs?
    percu_n = collections.Counter(((hw >> 32) & 0xFF, ((hw & 0xFFFFFFFF) >> 13) & 7, ((hw & 0xFFFFFFFF) >> 12) & 1, ((hw & 0xFFFFFFFF) >> 8) & 15) for _, _, hw in rows)
    print("  WGs per CU histogram:", dict(collections.Counter(percu_n.values())))
    # shader engine / array of each query block's workgroups, and duration by SE
    se_qb = collections.defaultdict(collections.Counter)
    dur_se = collections.defaultdict(list)
    for s_, e_, hw in rows:
        h = hw & 0xFFFFFFFF
        se, sa = (h >> 13) & 7, (h >> 12) & 1
        se_qb[(hw >> 40) & 0xFFFF][(se, sa)] += 1
        dur_se[(se, sa)].append((e_ - s_) / 100.0)
    print("  qb -> (se,sa):count " + " | ".join(
        f"{x}:" + ",".join(f"{k[0]}{k[1]}:{v}" for k, v in sorted(se_qb[x].items())) for x in xs[:16]))
    dur_x = collections.defaultdict(list)
    dur_cu = collections.defaultdict(list)
    for s_, e_, hw in rows:
        h = hw & 0xFFFFFFFF
        dur_x[(hw >> 32) & 0xFF].append((e_ - s_) / 100.0)
        dur_cu[(h >> 8) & 15].append((e_ - s_) / 100.0)
    print("  dur by head: " + " ".join(f"{k}:{sum(v)/len(v):.0f}/{max(v):.0f}" for k, v in sorted(byh.items())[:64]))
    print("  dur by xcc: " + " ".join(f"{k}:{sum(v)/len(v):.1f}/{max(v):.1f}" for k, v in sorted(dur_x.items())))
    print("  dur by cu-in-sa: " + " ".join(f"{k}:{sum(v)/len(v):.1f}/{max(v):.1f}" for k, v in sorted(dur_cu.items())))
    print("  dur by (se,sa): " + " ".join(f"{k[0]}{k[1]}:{sum(v)/len(v):.1f}(n{len(v)})" for k, v in sorted(dur_se.items())))
