#!/usr/bin/env python3
"""Generate csrc/fa_w4_tile_asm.inc: the hand-scheduled common-case tile body of
the W4x64 loop (64 query rows per wave, one wave per SIMD, BN = 64, head_dim
128, fp16) as ONE inline-asm statement.

Why one statement: hipcc sees no MFMA latency inside asm, so with one MFMA per
statement it clusters the softmax VALU instead of spacing it between the
MFMAs.  Here the order is fixed by hand:

  QK^T   64 MFMAs t-major (S = K . Q^T + (-m_ref)), K fragments double-
         buffered in 8 slots, each ds_read_b128 has 16 MFMAs to land
  max    per-lane partial row maxima (v_max3), V reads of the first PV half
         in flight meanwhile; any row past RESCALE_LOG2 -> flag = 1, exit
         (the caller reruns the tile on the plain path: rescale is rare)
  exp    P = exp2(S) for keys 0-31 (exposed), then keys 32-63 one v_exp per
         PV MFMA; v_cvt_pk_f16_f32 packs P in place over S
  PV     O += V^T . P and l += ones . P, 72 MFMAs, the second half's V
         fragments read into slots as the first half frees them

Register contract (the statement clobbers v[144:255]; nothing asm-owned lives
across statements):
  negm[b]   v[144+4b : +3]   -m_ref broadcast (C of the first QK^T MFMA)
  S[b][cb]  v[160+16b+4cb : +3]; P[b][u] packed in place at S[b][2u]
  slot j    v[224+4j : +3]   K fragments (QK^T), V fragments (PV)
  O, l, Q   compiler-allocated AGPR tuples ("+a" / "a" operands)
Hazards (hipcc pads nothing inside asm): 2+ wait states between a VALU write
and an MFMA reading it (s_nop 1); 19 between the last QK^T MFMA and the first
VALU read of S; EXEC is all ones (ds_read_b64_tr_b16 requires it).

    python tools/gen_w4_tile_asm.py   (run by the Makefile)
"""
import os

import sys

QB, NTQ, NKB, NE, NU = 4, 4, 4, 8, 2
# diagnostic variants (timing only, wrong results): nosm = no max/exp/cvt,
# nolds = no LDS reads either (MFMAs on stale fragments)
VARIANT = sys.argv[1] if len(sys.argv) > 1 else ""
NOSM = VARIANT in ("nosm", "nolds")
NOLDS = VARIANT == "nolds"
RESCALE_LOG2 = "8.0"

# operand numbering (outputs first, "+" operands are outputs)
OPS = []


def op(name, cons, expr):
    OPS.append((name, cons, expr))
    return len(OPS) - 1


acc = [[op(f"acc{b}{e}", "+a", f"acc[{b}][{e}]") for e in range(NE)] for b in range(QB)]
lacc = [op(f"lacc{b}", "+a", f"lacc[{b}]") for b in range(QB)]
flag = op("flag", "=&s", "flag")
N_OUT = len(OPS)
qf = [[op(f"q{b}{t}", "a", f"qf[{b}][{t}]") for t in range(NTQ)] for b in range(QB)]
mref = [op(f"m{b}", "v", f"m_ref[{b}]") for b in range(QB)]
ka = [op(f"ka{t}", "v", f"ka[{t}]") for t in range(NTQ)]
va = [op(f"va{ep}", "v", f"va[{ep}]") for ep in range(2)]
ones = op("ones", "v", "ones")


def o(i):
    return f"%{i}"


def V(i):
    return f"v{i}"


def VR(i, n=4):
    return f"v[{i}:{i + n - 1}]"


NEGM = lambda b: 144 + 4 * b
S = lambda b, cb: 160 + 16 * b + 4 * cb
P = lambda b, u: S(b, 2 * u)
SLOT = lambda j: 224 + 4 * j

lines = []


def emit(l):
    if NOSM and l.split()[0] in ("v_max3_f32", "v_max_f32_e32", "v_cmp_lt_f32_e32", "s_cbranch_vccnz",
                                 "v_exp_f32_e32", "v_cvt_pk_f16_f32"):
        return
    if NOLDS and l.split()[0].startswith("ds_read"):
        return
    lines.append(l)

emit("s_waitcnt lgkmcnt(0)")  # older LDS / scalar loads of the compiler drained
# K fragments of t = 0 and t = 1 (slot 4*(t&1) + cb)
for t in (0, 1):
    for cb in range(NKB):
        emit(f"ds_read_b128 {VR(SLOT(4 * t + cb))}, {o(ka[t])} offset:{4096 * cb}")
# negm[b] = -m_ref[b] broadcast while the reads fly
for b in range(QB):
    for i in range(4):
        emit(f"v_mul_f32_e32 {V(NEGM(b) + i)}, -1.0, {o(mref[b])}")
emit("s_nop 1")
for t in range(NTQ):
    # fragments of t ready: the 4 reads of t+1 (if issued) may stay in flight
    emit(f"s_waitcnt lgkmcnt({4 if t + 1 < NTQ else 0})")
    for cb in range(NKB):
        for b in range(QB):
            c = VR(NEGM(b)) if t == 0 else VR(S(b, cb))
            emit(f"v_mfma_f32_16x16x32_f16 {VR(S(b, cb))}, {VR(SLOT(4 * (t & 1) + cb))}, {o(qf[b][t])}, {c}")
    if t + 2 < NTQ:  # refill this t's slots with t+2 (their last readers issued)
        for cb in range(NKB):
            emit(f"ds_read_b128 {VR(SLOT(4 * (t & 1) + cb))}, {o(ka[t + 2])} offset:{4096 * cb}")
# first PV half's V fragments (slot e) in flight during the max
def v_reads(u, e):
    base = 8192 * u + 512 * (e >> 1)
    emit(f"ds_read_b64_tr_b16 {VR(SLOT(e), 2)}, {o(va[e & 1])} offset:{base}")
    emit(f"ds_read_b64_tr_b16 {VR(SLOT(e) + 2, 2)}, {o(va[e & 1])} offset:{base + 4096}")


for e in range(NE):
    v_reads(0, e)
emit("s_nop 7")
emit("s_nop 7")
emit("s_nop 3")
# per-lane partial maxima of each row block
for b in range(QB):
    regs = [S(b, cb) + i for cb in range(NKB) for i in range(4)]
    m = NEGM(b)  # negm[b] is dead after QK^T: it holds the running max
    emit(f"v_max3_f32 {V(m)}, {V(regs[0])}, {V(regs[1])}, {V(regs[2])}")
    k = 3
    while k < 16:
        if k + 1 < 16:
            emit(f"v_max3_f32 {V(m)}, {V(m)}, {V(regs[k])}, {V(regs[k + 1])}")
            k += 2
        else:
            emit(f"v_max_f32_e32 {V(m)}, {V(m)}, {V(regs[k])}")
            k += 1
# any lane of any row block past the threshold -> rare path
for b in range(QB):
    emit(f"v_cmp_lt_f32_e32 vcc, {RESCALE_LOG2}, {V(NEGM(b))}")
    emit(f"s_cbranch_vccnz W4_RARE_%=")
emit(f"s_mov_b32 {o(flag)}, 0")
# exps of keys 0-31 (S blocks cb 0, 1) for every b, packed in place into P[b][0]
def exp_block(b, cb):
    for i in range(4):
        emit(f"v_exp_f32_e32 {V(S(b, cb) + i)}, {V(S(b, cb) + i)}")


def cvt_pair(b, u):
    s0, s1 = S(b, 2 * u), S(b, 2 * u + 1)
    emit(f"v_cvt_pk_f16_f32 {V(s0 + 0)}, {V(s0 + 0)}, {V(s0 + 1)}")
    emit(f"v_cvt_pk_f16_f32 {V(s0 + 1)}, {V(s0 + 2)}, {V(s0 + 3)}")
    emit(f"v_cvt_pk_f16_f32 {V(s0 + 2)}, {V(s1 + 0)}, {V(s1 + 1)}")
    emit(f"v_cvt_pk_f16_f32 {V(s0 + 3)}, {V(s1 + 2)}, {V(s1 + 3)}")


for b in range(QB):
    exp_block(b, 0)
    exp_block(b, 1)
    cvt_pair(b, 0)
emit("s_waitcnt lgkmcnt(0)")
emit("s_nop 1")
# VALU filler queue for the first PV half: exps of cb 2, 3 and their packing
fill = []
for b in range(QB):
    for cb in (2, 3):
        for i in range(4):
            fill.append(f"v_exp_f32_e32 {V(S(b, cb) + i)}, {V(S(b, cb) + i)}")
    s0, s1 = S(b, 2), S(b, 3)
    fill += [f"v_cvt_pk_f16_f32 {V(s0 + 0)}, {V(s0 + 0)}, {V(s0 + 1)}",
             f"v_cvt_pk_f16_f32 {V(s0 + 1)}, {V(s0 + 2)}, {V(s0 + 3)}",
             f"v_cvt_pk_f16_f32 {V(s0 + 2)}, {V(s1 + 0)}, {V(s1 + 1)}",
             f"v_cvt_pk_f16_f32 {V(s0 + 3)}, {V(s1 + 2)}, {V(s1 + 3)}"]
fill.reverse()
# PV, first half (u = 0): e-outer, b-inner; slot e refilled with u = 1 once its 4 MFMAs issued
for e in range(NE):
    for b in range(QB):
        emit(f"v_mfma_f32_16x16x32_f16 {o(acc[b][e])}, {VR(SLOT(e))}, {VR(P(b, 0))}, {o(acc[b][e])}")
        if fill:
            emit(fill.pop())
    v_reads(1, e)
for b in range(QB):
    emit(f"v_mfma_f32_16x16x32_f16 {o(lacc[b])}, {o(ones)}, {VR(P(b, 0))}, {o(lacc[b])}")
    if fill:
        emit(fill.pop())
while fill:
    emit(fill.pop())
emit("s_waitcnt lgkmcnt(0)")
emit("s_nop 1")
for e in range(NE):
    for b in range(QB):
        emit(f"v_mfma_f32_16x16x32_f16 {o(acc[b][e])}, {VR(SLOT(e))}, {VR(P(b, 1))}, {o(acc[b][e])}")
for b in range(QB):
    emit(f"v_mfma_f32_16x16x32_f16 {o(lacc[b])}, {o(ones)}, {VR(P(b, 1))}, {o(lacc[b])}")
emit("s_branch W4_END_%=")
emit("W4_RARE_%=:")
emit("s_waitcnt lgkmcnt(0)")  # the V reads issued before the test
emit(f"s_mov_b32 {o(flag)}, 1")
emit("W4_END_%=:")

asm_text = "\\n\\t".join(lines)
outs = ", ".join(f'"{c}"({e})' for _, c, e in OPS[:N_OUT])
ins = ", ".join(f'"{c}"({e})' for _, c, e in OPS[N_OUT:])
clob = ", ".join(f'"v{i}"' for i in range(144, 256))

body = f'''// GENERATED by tools/gen_w4_tile_asm.py -- do not edit.  See that script's
// docstring for the schedule, the register contract and the hazard padding.
// Common-case tile body of the W4x64 loop: returns 0 when the tile was
// computed (O, l updated), 1 when some row's max grew past RESCALE_LOG2
// (nothing written: the caller reruns the tile on the plain path).
__device__ __forceinline__ int w4_tile_asm(f32x4 (&acc)[4][8], f32x4 (&lacc)[4],
                                           const f16x8 (&qf)[4][4], const float (&m_ref)[4],
                                           const int (&ka)[4], const int (&va)[2], f16x8 ones) {{
  int flag;
  asm volatile(
      "{asm_text}"
      : {outs}
      : {ins}
      : {clob}, "vcc", "scc", "memory");
  return flag;
}}
'''
out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc",
                   "fa_w4_tile_asm%s.inc" % ("_" + VARIANT if VARIANT else ""))
with open(out, "w") as f:
    f.write(body)
print(f"wrote {out}: {len(lines)} instructions, {len(OPS)} operands")
