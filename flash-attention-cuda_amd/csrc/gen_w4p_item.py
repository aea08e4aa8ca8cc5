#!/usr/bin/env python3
"""Generator of the multi-block one-wave-per-SIMD item program (fa_w4p_item.inc).

The short-sequence tier W4P (fa_w4p_kernel.hpp): one workgroup = 4 waves, one
per SIMD, on up to FOUR 64-row query blocks X0..X3 of one head (sorted by key
tile count T0 >= T1 >= T2 >= T3; an absent block has T = 0).  Wave w holds 16
rows of each -- row block b = rows 64 X_b + 16 w + r16 -- and the four waves
walk ONE shared K/V stream (key tiles 0 .. T0-1, double-buffered LDS images
filled by LDS-DMA, exactly the W4 images).  Causal launches group the heavy
block nqb-1-r with the light block r of the same head (a pair), one or two
pairs per workgroup, so every workgroup walks the same number of 64x64 tile
products (the reference's heaviest-first order, flash_attention.cu:103-112,
taken to its balanced end).  A launch of B*H*S query rows then fills the chip
at 128 rows per workgroup (pairs: B=1 H=32 S=1024 is 256 workgroups, where
W4's 256-row items leave half of it idle) and keeps 4 blocks per wave for as
many tiles as possible at 256 (quads).

Per key tile j (after the prologue computed S(0)) a wave runs, with NP = the
blocks that have tile j (PV(j)) and NQ = those that have tile j+1 (QK^T(j+1)):
  phase A: QK^T(j+1), 16 NQ MFMAs in 4 NQ four-deep chains, beside the fp16
           conversion of P(j) of the NP blocks, the running maxima of S(j+1),
           the K fragment reads (each feeds NQ MFMAs) and the LDS-DMA of
           K(j+2) / V(j+1)
  mask:    the blocks whose tile j+1 is their last (T_b = j+2): the limit
           mask (causal diagonal / ragged end), then their maxima again
  phase B: PV(j) + row sums, 18 NP MFMAs, beside the rescale decision and
           exp2 of S(j+1) and the V^T transposed reads
  s_waitcnt vmcnt(0), one barrier.
A kind per (NP, NQ): steady (NQ = NP), one block's PV drain (NQ = NP - 1),
all blocks' drain (NQ = 0).

The arithmetic is M16's (fa_fwd_kernel.hpp) with the rescale decision per
16-row block, checked against the oracle (reference cpu_attention) at the
1e-3 gate.  Hazards and LDS waits: gen_w4_item.Stream.

usage: python3 gen_w4p_item.py [OUT.inc]      (the Makefile runs it)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_w4_item as w4  # noqa: E402
from gen_w4_item import DT, NINF, R, Stream, dsr, mfma, salu, set_dtype, valu, vmem  # noqa: E402

NB = 4                 # query blocks per workgroup (at most: the register map's)
# blocks of the generated function: 4 (quads, G = 2) or 2 (pairs, G = 1: no
# absent blocks' Q loads / scaling / O, l zeroing in the prologue, no
# 3- and 4-block kinds; round 6)
CURNB = {"nb": 4}


def nb():
    return CURNB["nb"]
# head_dim of the generated function (set_hd: 128, the reference's, or 64):
# k-steps of a QK^T chain, 16-column O blocks, bytes of a Q/K/V/O row (HBM
# and the packed LDS images), of a 64-key tile, 1-KiB LDS-DMA pieces per wave
# and tensor, row shift
NT, NE, ROWB, TILEB, NPIECE, ROWSH = 4, 8, 256, 16384, 4, 8
PASSL = 4096           # LDS stride of a 4-KiB staging pass (32 rows at 64, 16 at 128)


def set_hd(hd):
    global NT, NE, ROWB, TILEB, NPIECE, ROWSH
    NT, NE, ROWB = hd // 32, hd // 16, 2 * hd
    TILEB = 64 * ROWB
    NPIECE = TILEB // 4096
    ROWSH = 8 if hd == 128 else 7
    w4.set_hd(hd)
RESCALE = "0x41000000"  # 8.0: m_ref moves when a row max grew past it (log2 units)


def fp32scale():
    """bf16 scores in fp32, as gen_w4_item.fp32scale: Q unscaled into the
    MFMA, NEGM = -m_ref / c, every score times c after its chain"""
    return w4.BF16_FP32SCALE and DT.get("bf16", False)


def scale_ops(b, cb):
    """S(b, cb) *= c in fp32 (four scalar multiplies: packed fp32 VALU beside
    MFMAs costs more issue, MI355X_MICROARCH.md constants table)"""
    cl = w4.c_lits()[0]
    x = 16 * b + 4 * cb
    return [valu(f"v_mul_f32_e32 v{x + i}, {cl}, v{x + i}", r=[f"v{x + i}"], w=[f"v{x + i}"]) for i in range(4)]

# ---------------------------------------------------------------------------
# register map (VGPR v0-v213, AGPR a0-a239; the compiler keeps the rest)
# ---------------------------------------------------------------------------


def S(b, cb, i=None):      # S^T tile: block b, 16-key block cb (fp32, exp2'd in place)
    base = 16 * b + 4 * cb
    return R("v", base, 4) if i is None else R("v", base + i)


def P(b, u, r=None):       # P fp16, B operand of PV: block b, 32-key step u
    base = 64 + 8 * b + 4 * u
    return R("v", base, 4) if r is None else R("v", base + r)


def NEGM(b, i=None):       # -m_ref broadcast: C operand of the first MFMA of a chain
    return R("v", 96 + 4 * b, 4) if i is None else R("v", 96 + 4 * b + i)


def KF(slot):              # K fragments: 8 slots (two 16-key blocks)
    return R("v", 112 + 4 * slot, 4)


def VF(slot, half=None):   # V^T fragments: 8 slots
    base = 144 + 4 * slot
    return R("v", base, 4) if half is None else R("v", base + 2 * half, 2)


def KD(i):                 # per-pass LDS-DMA source offsets
    return R("v", 176 + i)


def VD(i):
    return R("v", 180 + i)


ONES = R("v", 184, 4)
MREF = [R("v", 188 + b) for b in range(NB)]
RMAX = [R("v", 192 + b) for b in range(NB)]   # running partial maxima per block
VNINF = R("v", 196)
T = [R("v", 197 + i) for i in range(11)]      # v197-v207 temporaries
KOFF = ["%[koff]"] + [R("v", 208 + i) for i in range(3)]
VOFF = ["%[voff]"] + [R("v", 211 + i) for i in range(3)]
EPI = [f"v{144 + i}" for i in range(8)]       # epilogue staging (the free V^T slots)
XY = ["v152", "v153", "v154", "v155"]         # one store: X = v152,153 ; Y = v154,155
NV = 217   # v214-v216: the V image bases + 64 KiB (dbl programs)


def O(b, e, i=None):       # O^T accumulator, block b, d-block e
    base = 32 * b + 4 * e
    return R("a", base, 4) if i is None else R("a", base + i)


def L(b, i=None):          # row sums l
    return R("a", 128 + 4 * b, 4) if i is None else R("a", 128 + 4 * b + i)


def Q(b, t):               # Q * c (fp16), B operand of QK^T
    return R("a", 144 + 16 * b + 4 * t, 4)


def KST1(i):               # prologue staging: K(1) / V(0)
    return R("a", 208 + 4 * i, 4)


def VST1(i):
    return R("a", 224 + 4 * i, 4)


NA = 240

# LDS images (W4's): K at 0 / 16384, V at 32768 / 49152
KBUF = [0, 16384]
VBUF = [32768, 49152]


# Two key tiles per barrier (the pair program at head_dim 128, as
# gen_w4_item.py's dbl): four K / V images (K at 0-48 KiB, V at 64-112 KiB),
# tiles DMA'd two ahead, a pair iteration of two steady tiles -- same
# kind, every live block steady for both: T[k-1] >= j + 4 -- with one DMA
# wait and one barrier, the second tile's key-block-0 fragments read in the
# first tile's PV tail.  W4_XP=nodblp: the one-tile loop.
def pdbl():
    return (nb() == 2 or "dblq" in w4.XP) and NT == 4 and "nodblp" not in w4.XP and "p1nolds" not in w4.XP


def nbuf():
    return 4 if pdbl() else 2


def look():
    return 2 if pdbl() else 1


def kbuf(i):  # ds offset of tile i's K image
    return 16384 * (i % nbuf())


def vbuf(i):  # ds offset of tile i's V image from vaddr()
    return 16384 * (i % 4) if pdbl() else VBUF[i % 2]


def vbuf_abs(i):  # LDS offset of tile i's V image (M0 of its DMA)
    return 65536 + 16384 * (i % 4) if pdbl() else VBUF[i % 2]


def vaddr(k):
    return ("v214", "v215")[k] if pdbl() else VADDR[k]


def vlds():
    return "v216" if pdbl() else "%[vlds]"
KADDR = [f"%[ka{t}]" for t in range(4)]
VADDR = ["%[va0]", "%[va1]"]

# SGPR scratch (clobbered s40-s71)
SK, SV = "s[40:43]", "s[44:47]"
SKREM, SVREM = "s48", "s49"
SJ, SJ1 = "s50", "s51"
ST0, ST1 = "s52", "s53"
KV0 = "s54"
SNP = "s55"
RQ, RO = "s[56:59]", "s[60:63]"
SM0 = "s64"
DIVS = "s[66:67]"
SJ2 = "s68"
STMP = "s69"
NS_LO, NS_HI = 40, 72

# block b's row base (64 X_b + 16 w), key bound, key tiles, of the C++ side
QR = [f"%[qr{b}]" for b in range(NB)]
KVH = [f"%[kvh{b}]" for b in range(NB)]
TB = [f"%[t{b}]" for b in range(NB)]

MAX_OFF, LEFT_OFF, DEC_GAP = 2, 3, 6
# prologue experiment (W4_XP=latev0k1): S(0) starts once Q and K(0) are in,
# V(0) / K(1) written after S(0) and the first softmax, before the
# prologue's second barrier.  Measured and not kept: the prologue stays at
# 7.0k cycles and the launches are level to slower (config 1 534.2 vs
# 537.7, B=2 S=1024 causal 677.2 vs 697.9, H=16 S=2048 957.5 vs 972.8;
# S=2048 causal 882.6 vs 870.8; profiles/r06_ab_w4p_prologue_nolds.jsonl)
LATE_V0K1 = "latev0k1" in w4.XP


def lag():  # chains between a chain and its maxima (a chain is NT MFMAs)
    return 2 if NT == 4 else 3

# diagnostic builds only (never the product library; tools/w4_variant.sh):
# W4P_DIAG=stamps accumulates per wave the shader cycles of the prologue, of
# the iterations with 4 / 3 / 2 / 1 blocks with a QK^T (steady or not), of
# the drains (no QK^T), their counts, the end-of-iteration DMA wait + barrier
# and the epilogue, and stores them over O[qr0][0:32] (every lane the same
# 64 bytes)
DIAG = os.environ.get("W4P_DIAG", "")
STAMPS = DIAG == "stamps"
# s72 start, s74 path, s76 stamp, s78-s82 cycles of paths 0-4, s83-s87
# counts, s88 wait+barrier, s89 prologue, s90 epilogue, s91 select tmp
NS_DIAG = 92
NPATH = 5


def stamp_now(st, dst):
    if STAMPS:
        st.raw(f"s_memtime s[{dst}:{dst + 1}]")
        st.raw("s_waitcnt lgkmcnt(0)")
        st.lgkm = []


def stamp_path(st, k):
    """at an iteration kind's label: its start stamp and id"""
    if STAMPS:
        stamp_now(st, 72)
        st.raw(f"s_mov_b32 s74, {k}")


def stamp_path_end(st):
    """at the iteration end (before the DMA wait): the path's cycles and count"""
    if not STAMPS:
        return
    stamp_now(st, 76)
    st.raw("s_sub_u32 s75, s76, s72")
    for k in range(NPATH):
        st.raw(f"s_cmp_eq_u32 s74, {k}")
        st.raw("s_cselect_b32 s77, s75, 0")
        st.raw("s_cselect_b32 s91, 1, 0")
        st.raw(f"s_add_u32 s{78 + k}, s{78 + k}, s77")
        st.raw(f"s_add_u32 s{83 + k}, s{83 + k}, s91")


# one-block iterations' LDS read-ahead: V^T fragments 8 MFMAs ahead instead
# of 6 (W4_XP=nop1v8: 6), K fragments two 16-key blocks ahead instead of one
# (the third set in block 1's free S registers; W4_XP=nop1k2: one).  Measured
# alone on the one-tile-per-barrier program: +0.8 / -0.4 %; together on the
# two-tiles-per-barrier program: config 1 +1.9 %, B=2 H=8 S=2048 causal
# +1.4 %, +0.4-0.5 % on S=512 causal / H=8 S=4096 causal / H=16 S=2048
# (bit-identical; profiles/r06_ab_w4p_probes.jsonl)
P1V8 = "nop1v8" not in w4.XP
P1K2 = "nop1k2" not in w4.XP


def vahead(np_):
    """V^T fragments read ahead of their PV MFMAs: >= 8 MFMAs of cover for the
    LDS latency (at head_dim 64 at most the tile's 8)"""
    if np_ == 1 and P1V8:
        return min(8, 2 * NE)
    return min({1: 6, 2: 4}.get(np_, 3), 2 * NE)


def kreg(cb, t, one=False):
    """K fragment register of (16-key block cb, k-step t); one (P1K2, one-block
    kinds): three sets, key block 2's in block 1's S registers v16-v31"""
    if one and cb == 2:
        return R("v", 16 + 4 * t, 4)
    if one and cb == 3:
        return KF(t)  # key block 0's set, consumed by then
    return KF(kslot(cb, t))


def kslot(cb, t):
    """K fragment slot: two 16-key blocks' fragments at head_dim 128 (read one
    block ahead), the whole tile's 8 at 64"""
    return 4 * (cb & 1) + t if NT == 4 else 2 * cb + t


def k_read(t, cb, kb, one=False):
    r = kreg(cb, t, one)
    return dsr(f"ds_read_b128 {r}, {KADDR[t]} offset:{kb + 16 * ROWB * cb}", r, KADDR[t])


def k_reads_tile(kb):
    """head_dim 64: every K fragment of the tile at once (the 8 slots hold it)"""
    return [k_read(t, cb, kb) for cb in range(4) for t in range(NT)]


def v_reads(f, vb):
    u, e = divmod(f, NE)
    slot = f % 8
    off = vb + 32 * ROWB * u + 512 * (e >> 1)
    a = vaddr(e & 1)
    return [dsr(f"ds_read_b64_tr_b16 {VF(slot, 0)}, {a} offset:{off}", VF(slot, 0), a),
            dsr(f"ds_read_b64_tr_b16 {VF(slot, 1)}, {a} offset:{off + 16 * ROWB}", VF(slot, 1), a)]


def qk_chain(b, cb, one=False):
    out = []
    for t in range(NT):
        c = NEGM(b) if t == 0 else S(b, cb)
        out.append(mfma(S(b, cb), kreg(cb, t, one), Q(b, t), c))
    return out


def cvt_block(b, cb):
    p = 64 + 8 * b + 4 * (cb >> 1) + 2 * (cb & 1)
    s = 16 * b + 4 * cb
    return [valu(f"{DT['cvt_pk']} v{p}, v{s}, v{s + 1}", r=[f"v{s}", f"v{s + 1}"], w=[f"v{p}"]),
            valu(f"{DT['cvt_pk']} v{p + 1}, v{s + 2}, v{s + 3}", r=[f"v{s + 2}", f"v{s + 3}"], w=[f"v{p + 1}"])]


def max_block(b, cb, first):
    s = 16 * b + 4 * cb
    m = RMAX[b]
    if first:
        return [valu(f"v_max3_f32 {m}, v{s}, v{s + 1}, v{s + 2}", r=[f"v{s}", f"v{s + 1}", f"v{s + 2}"], w=[m]),
                valu(f"v_max_f32 {m}, {m}, v{s + 3}", r=[m, f"v{s + 3}"], w=[m])]
    return [valu(f"v_max3_f32 {m}, {m}, v{s}, v{s + 1}", r=[m, f"v{s}", f"v{s + 1}"], w=[m]),
            valu(f"v_max3_f32 {m}, {m}, v{s + 2}, v{s + 3}", r=[m, f"v{s + 2}", f"v{s + 3}"], w=[m])]


def exp_ops(b):
    return [valu(f"v_exp_f32 v{x}, v{x}", r=[f"v{x}"], w=[f"v{x}"], kind="trans")
            for x in range(16 * b, 16 * b + 16)]


def pv_mfmas(np_):
    """PV + row sums of blocks 0..np-1: for u: for e: the blocks; then their row sums"""
    ms, frag_first = [], {}
    for u in range(2):
        for e in range(NE):
            frag_first[u * NE + e] = len(ms)
            for b in range(np_):
                ms.append(mfma(O(b, e), VF((u * NE + e) % 8), P(b, u), O(b, e)))
        ms += [mfma(L(b), ONES, P(b, u), L(b)) for b in range(np_)]
    return ms, frag_first


def dma_pieces(p):
    """LDS-DMA of K(j+1+look) -> its K image, V(j+look) -> its V image
    (one tile ahead: K(j+2) -> kbuf[p], V(j+1) -> vbuf[1-p]): (M0 set, load)
    pairs, then the descriptors advance one tile (gen_w4_item.dma_loads)"""
    pairs = []
    for i in range(NPIECE):
        pairs.append((salu(f"s_add_u32 m0, %[dmab], {kbuf(p + 1 + look()) + 1024 * i}"),
                      vmem(f"buffer_load_dwordx4 {KD(i)}, {SK}, 0 offen lds", r=[KD(i)])))
    for i in range(NPIECE):
        pairs.append((salu(f"s_add_u32 m0, %[dmab], {vbuf_abs(p + look()) + 1024 * i}"),
                      vmem(f"buffer_load_dwordx4 {VD(i)}, {SV}, 0 offen lds", r=[VD(i)])))
    tb = hex(TILEB)
    adv = [[salu(f"s_add_u32 s40, s40, {tb}"), salu("s_addc_u32 s41, s41, 0")],
           [salu(f"s_sub_i32 {SKREM}, {SKREM}, {tb}"), salu(f"s_max_i32 s42, {SKREM}, 0")],
           [salu(f"s_add_u32 s44, s44, {tb}"), salu("s_addc_u32 s45, s45, 0")],
           [salu(f"s_sub_i32 {SVREM}, {SVREM}, {tb}"), salu(f"s_max_i32 s46, {SVREM}, 0")]]
    return pairs, adv


# ---------------------------------------------------------------------------
# one iteration: phase A / mask / phase B
# ---------------------------------------------------------------------------
def phase_a(st, p, nq, np_, k0_issued=False):
    """QK^T(j+1) of blocks 0..nq-1 from kbuf[1-p] beside the fp16 conversion of
    P(j) of blocks 0..np-1 (each just before the chain that overwrites its
    scores), the running maxima of S(j+1), the K reads, the stage's LDS-DMA
    and the first V^T fragments of PV(j).  nq = 0 (the last tile): the
    conversions and V^T reads alone."""
    kb = kbuf(p + 1)
    va = vahead(np_)
    if nq == 0:
        for b in range(np_):
            for cb in range(4):
                for c in cvt_block(b, cb):
                    st.emit(c)
        for f in range(va):
            for r in v_reads(f, vbuf(p)):
                st.emit(r)
        return [], []
    chains = [(b, cb) for cb in range(4) for b in range(nq)]
    one = P1K2 and nq == 1 and np_ == 1 and NT == 4  # (kind (2, 1): block 1 still converts its P from v16-v31)
    mf = []
    for b, cb in chains:
        mf += qk_chain(b, cb, one)
    n = len(mf)
    gaps = {}

    def put(k, ins):
        gaps.setdefault(k, []).extend(ins if isinstance(ins, list) else [ins])

    if k0_issued:
        # key block 0's fragments were read in the previous phase B's tail
        # (pdbl: no barrier between); with P1K2 key block 1's follow now
        if one:
            put(0, [k_read(t, 1, kb, one) for t in range(NT)])
    elif one:
        put(0, [k_read(t, cb, kb, one) for cb in range(2) for t in range(NT)])
    else:
        put(0, [k_read(t, 0, kb) for t in range(NT)] if NT == 4 else k_reads_tile(kb))
    for x, (b, cb) in enumerate(chains):
        c = cvt_block(b, cb)
        if cb == 0:
            put(0, c)
        else:
            put(NT * x - 1, c[0])
            put(NT * x, c[1])
        if one:
            if cb < 2:
                for t in range(NT):
                    put(NT * x + 1 + t % 3, k_read(t, cb + 2, kb, one))
        elif b == 0 and cb < 3 and NT == 4:
            for t in range(NT):
                put(NT * x + 1 + t % 3, k_read(t, cb + 1, kb))
        if x >= lag():
            by, cby = chains[x - lag()]
            if fp32scale():
                put(min(NT * x + MAX_OFF - 1, n), scale_ops(by, cby))
            mm = max_block(by, cby, first=(cby == 0))
            put(min(NT * x + MAX_OFF, n), mm[0])
            put(min(NT * x + MAX_OFF + 1, n), mm[1])
    # conversions of the blocks with a PV(j) but no QK(j+1) (their drain): any gap
    extra = [c for b in range(nq, np_) for cb in range(4) for c in cvt_block(b, cb)]
    for i, c in enumerate(extra):
        put(1 + (i * (n - 2)) // len(extra), c)
    # LDS-DMA: an M0 write and its load are always an MFMA apart (M0 wait
    # state); two or more blocks spread them over two gaps each, one shares gaps
    pairs, adv = dma_pieces(p)
    late = []
    if nq == 1 and np_ == 1 and "p1nodma" in w4.XP:
        pairs, adv = [], []   # timing-only probe: no K/V DMA in one-block iterations
    if nq == 1 and np_ == 1 and "p1dmaa" not in w4.XP:
        # one-block iterations: the V tile's pieces and descriptor advance in
        # phase B (its buffer is free for the whole iteration) -- eight pieces
        # at ~60 issue cycles crowd phase A's 16 MFMA gaps; +2.7 % at config 1,
        # +3.3 % at H=8 S=4096, +0.5-0.9 % elsewhere (profiles/
        # r05_ab_w4p_dmab.jsonl; W4_XP=p1dmaa keeps them in phase A)
        late = [ins for pr in pairs[NPIECE:] for ins in pr] + [i for g in adv[2:] for i in g]
        pairs, adv = pairs[:NPIECE], adv[:2]
    a0, sp = (2, 2) if nq >= 2 else (1, 1)
    for i, (m0, ld) in enumerate(pairs):
        put(a0 + sp * i, m0)
        put(a0 + sp * i + 1, ld)
    g = a0 + sp * (len(pairs) - 1) + 2
    for i, ins in enumerate(adv):
        put(min(g + i, n), ins)
    # the first V^T fragments of PV(j) (V(j) is ready since the last barrier)
    for f in range(va):
        for i, r in enumerate(v_reads(f, vbuf(p))):
            put(min(max(0, n - 2 * va) + 2 * f + i, n), r)
    if fp32scale():
        for y in range(max(0, len(chains) - lag()), len(chains)):
            put(n, scale_ops(*chains[y]))
    assert max(gaps) <= n, "every filler lands in a gap"
    st.interleave(mf, gaps)
    left = []
    for y in range(max(0, len(chains) - lag()), len(chains)):
        by, cby = chains[y]
        left += max_block(by, cby, first=False)
    return left, late


def mask_pass(st, nq, causal):
    """blocks 0..nq-1 whose tile j+1 is their last (T_b = j+2): the limit mask,
    then their running maxima again (over the masked scores; phase B's
    leftover maxima re-max the masked values, a no-op).  T is sorted
    descending and every QK block has T_b >= j+2, so none is masked unless
    the last one is: one compare in the common case."""
    if nq == 0:
        return
    done = w4.newlabel("nomask")
    st.raw(f"s_cmp_eq_u32 {TB[nq - 1]}, {SJ2}")
    st.branch("s_cbranch_scc0", done)
    st.raw(f"s_lshl_b32 {KV0}, {SJ1}, 6")
    for b in range(nq):
        skip = w4.newlabel(f"nomask{b}_")
        if b < nq - 1:
            st.raw(f"s_cmp_eq_u32 {TB[b]}, {SJ2}")
            st.branch("s_cbranch_scc0", skip)
        mask_block(st, b, causal)
        full_max(st, b)
        st.label(skip)
    st.label(done)


def phase_b(st, p, nq, np_, leftover, label_slow, label_end, late=(), kpre=None):
    """PV(j) of blocks 0..np-1 from vbuf[p]; the rescale decision over the
    blocks 0..nq-1 at DEC_GAP, exp2 of their S(j+1) after it.  nq = 0: the
    PV alone."""
    vb = vbuf(p)
    mf, frag_first = pv_mfmas(np_)
    n = len(mf)
    gaps = {}

    def put(k, ins):
        gaps.setdefault(k, []).extend(ins if isinstance(ins, list) else [ins])

    # phase A's deferred DMA: (M0, load) pairs an MFMA apart, then the advance
    for i, ins in enumerate(late):
        put(1 + i, ins)
    va = vahead(np_)
    for f in range(va, 2 * NE):
        k = frag_first[f - va]
        r = v_reads(f, vb)
        put(k + 1, r[0])
        put(k + 2, r[1])
    if kpre is not None:
        # pdbl: the next phase A's key-block-0 K fragments (their image was
        # published by the barrier that opened this pair; the slots' last
        # reader was this iteration's QK^T)
        for t in range(NT):
            put(max(DEC_GAP + 1, n - 2 * NT - 2) + 2 * t, k_read(t, 0, kbuf(kpre)))
    # (head_dim 64: three chains' maxima, two per gap)
    lo = [LEFT_OFF + (i if NT == 4 else i // 2) for i in range(len(leftover))]
    for k, ins in zip(lo, leftover):
        put(k, ins)
    assert not leftover or lo[-1] <= DEC_GAP
    if nq == 0:
        st.interleave(mf, gaps)
        st.branch("s_branch", label_end)
        return
    m = RMAX[0]
    dec = []
    if nq >= 2:
        m = T[0]
        dec.append(valu(f"v_max3_f32 {T[0]}, {RMAX[0]}, {RMAX[1]}, {RMAX[2 if nq > 2 else 1]}",
                        r=RMAX[:nq], w=[T[0]]))
        if nq == 4:
            dec.append(valu(f"v_max_f32 {T[0]}, {T[0]}, {RMAX[3]}", r=[T[0], RMAX[3]], w=[T[0]]))
    dec.append(valu(f"v_cmp_lt_f32 vcc, {RESCALE}, {m}", r=[m]))
    exs = [e for b in range(nq) for e in exp_ops(b)]
    if nq == 1 and np_ == 1 and "p1noexp" in w4.XP:
        exs = []   # timing-only probe: no exp2 in one-block iterations
    n_g = n - DEC_GAP
    for i, e in enumerate(exs):
        put(DEC_GAP + 1 + (i * n_g) // len(exs), e)
    for k in range(DEC_GAP):
        for f in gaps.get(k, []):
            st.emit(f)
        st.emit(mf[k])
    for f in gaps.get(DEC_GAP, []):
        st.emit(f)
    for d in dec:
        st.emit(d)
    st.branch("s_cbranch_vccnz", label_slow)
    for k in range(DEC_GAP, n):
        if k > DEC_GAP:
            for f in gaps.get(k, []):
                st.emit(f)
        st.emit(mf[k])
    for f in gaps.get(n, []):
        st.emit(f)
    st.branch("s_branch", label_end)
    # slow path: the remaining PV MFMAs (their V reads, no exps), then rescale
    st.label(label_slow)
    for k in range(DEC_GAP, n):
        if k > DEC_GAP:
            for f in gaps.get(k, []):
                if isinstance(f, str) or f.kind != "trans":
                    st.emit(f)
        st.emit(mf[k])
    for f in gaps.get(n, []):
        if isinstance(f, str) or f.kind != "trans":
            st.emit(f)
    slow_softmax(st, range(nq), first=False)
    for e in exs:
        st.emit(e)
    st.branch("s_branch", label_end)


def slow_softmax(st, blocks, first):
    """rescale (the M16 softmax's rare branch) per 16-row block: m_ref moves
    when a lane's partial max of the block grew past RESCALE.  first: the
    item's first tile -- every row centres on its max (a fully masked row,
    max -inf, keeps m_ref = 0)."""
    for b in blocks:
        skip = w4.newlabel("pskip")
        if not first:
            st.emit(valu(f"v_cmp_lt_f32 vcc, {RESCALE}, {RMAX[b]}", r=[RMAX[b]]))
            st.branch("s_cbranch_vccz", skip)
        mx, sh = T[1], T[2]
        row_max_b(st, b, mx)
        if first:
            st.emit(valu(f"v_cmp_eq_f32 vcc, {VNINF}, {mx}", r=[VNINF, mx]))
            st.emit(valu(f"v_cndmask_b32_e64 {sh}, {mx}, 0, vcc", r=[mx], w=[sh]))
        else:
            st.emit(valu(f"v_max_f32 {sh}, 0, {mx}", r=[mx], w=[sh]))
        shift_block(st, b, sh, first)
        if not first:
            st.label(skip)


def row_max_b(st, b, dst):
    s = [f"v{16 * b + i}" for i in range(16)]
    st.emit(valu(f"v_max3_f32 {dst}, {s[0]}, {s[1]}, {s[2]}", r=s[0:3], w=[dst]))
    for i in range(3, 15, 2):
        st.emit(valu(f"v_max3_f32 {dst}, {dst}, {s[i]}, {s[i + 1]}", r=[dst, s[i], s[i + 1]], w=[dst]))
    st.emit(valu(f"v_max_f32 {dst}, {dst}, {s[15]}", r=[dst, s[15]], w=[dst]))
    tmp = T[10]
    for sw in ("v_permlane16_swap_b32", "v_permlane32_swap_b32"):
        st.emit(valu(f"v_mov_b32 {tmp}, {dst}", r=[dst], w=[tmp]))
        st.emit(valu(f"{sw} {dst}, {tmp}", r=[dst, tmp], w=[dst, tmp]))
        st.emit(valu(f"v_max_f32 {dst}, {dst}, {tmp}", r=[dst, tmp], w=[dst]))


def shift_block(st, b, sh, first):
    """m_ref moves by sh: S -= sh, m_ref += sh, negm = -m_ref; O, l *= 2^-sh"""
    if not first:
        alpha = T[3]
        st.emit(valu(f"v_exp_f32 {alpha}, -{sh}", r=[sh], w=[alpha], kind="trans"))
        regs = [O(b, e, i) for e in range(NE) for i in range(4)] + [L(b, i) for i in range(4)]
        for a in regs:
            st.emit(valu(f"v_accvgpr_read_b32 {T[4]}, {a}", r=[a], w=[T[4]]))
            st.emit(valu(f"v_mul_f32 {T[4]}, {T[4]}, {alpha}", r=[T[4], alpha], w=[T[4]]))
            st.emit(valu(f"v_accvgpr_write_b32 {a}, {T[4]}", r=[T[4]], w=[a]))
    for i in range(16):
        x = f"v{16 * b + i}"
        st.emit(valu(f"v_sub_f32 {x}, {x}, {sh}", r=[x, sh], w=[x]))
    st.emit(valu(f"v_add_f32 {MREF[b]}, {MREF[b]}, {sh}", r=[MREF[b], sh], w=[MREF[b]]))
    for i in range(4):
        if fp32scale():
            st.emit(valu(f"v_mul_f32_e32 {NEGM(b, i)}, {w4.c_lits()[1]}, {MREF[b]}", r=[MREF[b]], w=[NEGM(b, i)]))
        else:
            st.emit(valu(f"v_xor_b32 {NEGM(b, i)}, 0x80000000, {MREF[b]}", r=[MREF[b]], w=[NEGM(b, i)]))


def mask_block(st, b, causal):
    """S(b) = -inf where key >= kv_hi_b or (causal) key > query row, for the
    tile at key KV0 (key kv = KV0 + 16cb + 4sg + i, row = qr_b + r16):
    valid iff 16cb + i <= lim = min(kvh_b - KV0 - 1 - 4sg, qr_b - KV0 + r16 - 4sg).
    A tile inside both bounds gets lim >= 63: a no-op."""
    st.raw(f"s_sub_i32 {ST0}, {KVH[b]}, {KV0}")
    st.raw(f"s_sub_i32 {ST0}, {ST0}, 1")
    st.raw(f"s_sub_i32 {ST1}, {QR[b]}, {KV0}")
    lim_rag, lim = T[5], T[7]
    st.emit(valu(f"v_sub_u32 {T[6]}, %[vt], %[r16]", r=["%[vt]", "%[r16]"], w=[T[6]]))   # -4sg
    st.emit(valu(f"v_add_u32 {lim_rag}, {ST0}, {T[6]}", r=[T[6]], w=[lim_rag]))
    if causal:
        st.emit(valu(f"v_add_u32 {lim}, {ST1}, %[vt]", r=["%[vt]"], w=[lim]))
        st.emit(valu(f"v_min_i32 {lim}, {lim}, {lim_rag}", r=[lim, lim_rag], w=[lim]))
    else:
        lim = lim_rag
    for cb in range(4):
        for i in range(4):
            x = S(b, cb, i)
            st.emit(valu(f"v_cmp_le_i32 vcc, {16 * cb + i}, {lim}", r=[lim]))
            st.emit(valu(f"v_cndmask_b32 {x}, {VNINF}, {x}, vcc", r=[VNINF, x], w=[x]))


def full_max(st, b):
    for cb in range(4):
        for ins in max_block(b, cb, first=(cb == 0)):
            st.emit(ins)


def qk_plain(st, kb, nb):
    """QK^T of one tile for blocks 0..nb-1, not interleaved (prologue): each
    16-key block's four K fragments read one block ahead (head_dim 64: the
    whole tile's at once)"""
    for r in ([k_read(t, 0, kb) for t in range(NT)] if NT == 4 else k_reads_tile(kb)):
        st.emit(r)
    for cb in range(4):
        if cb < 3 and NT == 4:
            for t in range(NT):
                st.emit(k_read(t, cb + 1, kb))
        for b in range(nb):
            for m in qk_chain(b, cb):
                st.emit(m)


# iteration kinds (NP, NQ): steady, one block's drain, every block's drain
def kinds():
    n = nb()
    return [(k, k) for k in range(1, n + 1)] + [(k, k - 1) for k in range(1, n + 1)] + \
        [(k, 0) for k in range(2, n + 1)]


def kname(np_, nq):
    return f"k{np_}{nq}"


class _NoLds:
    """timing-only probe (W4_XP=p1nolds, wrong results): the one-block
    iterations issue no LDS reads (K and V^T fragments stay stale) -- what
    the iteration costs without its 128 KiB per CU of fragment reads"""

    def __init__(self, st):
        self.st = st

    def emit(self, ins):
        if isinstance(ins, str) or ins.kind != "dsr":
            self.st.emit(ins)

    def interleave(self, mfmas, gaps):
        for k, m in enumerate(mfmas):
            for f in gaps.get(k, []):
                self.emit(f)
            self.emit(m)
        for f in gaps.get(len(mfmas), []):
            self.emit(f)

    def __getattr__(self, k):
        return getattr(self.st, k)


def iteration(st, p, np_, nq, causal, Lb):
    stamp_path(st, NB - nq if nq else NPATH - 1)   # 0: 4 QK blocks .. 3: 1; 4: drain
    if "p1nolds" in w4.XP and np_ == 1:
        st = _NoLds(st)
    left, late = phase_a(st, p, nq, np_)
    mask_pass(st, nq, causal)
    phase_b(st, p, nq, np_, left, Lb["slow_" + kname(np_, nq)][p], Lb["end"][p], late)


# ---------------------------------------------------------------------------
# prologue / epilogue
# ---------------------------------------------------------------------------
def rsrc(st, dst, lo, hi, records):
    st.raw(f"s_mov_b32 s{dst}, {lo}")
    st.raw(f"s_and_b32 s{dst + 1}, {hi}, 0xffff")
    st.raw(f"s_mov_b32 s{dst + 2}, {records}")
    st.raw(f"s_mov_b32 s{dst + 3}, 0x20000")


def q_scale(st):
    """Q * c (fp32 product, then fp16: M16::scale_q) from v0-63 into a144-207,
    eight elements at a time in the (free) V^T fragment registers"""
    qregs = [16 * b + j for b in range(nb()) for j in range(4 * NT)]  # Q(b, t) raw: v[16b + 4t ..]
    for c0 in range(0, len(qregs), 8):
        xs = qregs[c0:c0 + 8]
        lo = {x: f"v{144 + 3 * i}" for i, x in enumerate(xs)}
        hi = {x: f"v{145 + 3 * i}" for i, x in enumerate(xs)}
        pk = {x: f"v{146 + 3 * i}" for i, x in enumerate(xs)}
        if w4.mix():  # one rounding: gen_w4_item.mix_pk
            for x in xs:
                for op in w4.mix_pk(pk[x], f"v{x}", f"v{x}", "%[c]", f16src=True):
                    st.raw(op.text)
            for x in xs:
                st.raw(f"v_accvgpr_write_b32 a{144 + x}, {pk[x]}")
            continue
        if fp32scale():  # Q unscaled: c applies to the fp32 scores
            for x in xs:
                st.raw(f"v_accvgpr_write_b32 a{144 + x}, v{x}")
            continue
        if DT["bf16"]:
            for x in xs:
                st.raw(f"v_lshlrev_b32_e32 {lo[x]}, 16, v{x}")
                st.raw(f"v_and_b32_e32 {hi[x]}, 0xffff0000, v{x}")
            for x in xs:
                st.raw(f"v_mul_f32_e32 {lo[x]}, %[c], {lo[x]}")
                st.raw(f"v_mul_f32_e32 {hi[x]}, %[c], {hi[x]}")
        else:
            for x in xs:
                st.raw(f"v_fma_mix_f32 {lo[x]}, v{x}, %[c], neg(0) op_sel_hi:[1,0,0]")
                st.raw(f"v_fma_mix_f32 {hi[x]}, v{x}, %[c], neg(0) op_sel:[1,0,0] op_sel_hi:[1,0,0]")
        for x in xs:
            st.raw(f"{DT['cvt_pk']} {pk[x]}, {lo[x]}, {hi[x]}")
        for x in xs:
            st.raw(f"v_accvgpr_write_b32 a{144 + x}, {pk[x]}")


def prologue(st, causal):
    """descriptors, Q (every block) / K(0) / V(0) / K(1) loads, Q scaling,
    S(0) = K(0) Q^T of the blocks with a tile, the tile-0 mask where it is a
    block's last tile, the first-tile softmax"""
    if STAMPS:
        for r in range(72, NS_DIAG):
            st.raw(f"s_mov_b32 s{r}, 0")
        stamp_now(st, 76)
    st.raw(f"s_mov_b32 {SM0}, m0")
    if pdbl():
        st.raw("v_add_u32 v214, 0x10000, %[va0]")
        st.raw("v_add_u32 v215, 0x10000, %[va1]")
        st.raw("v_add_u32 v216, 0x10000, %[vlds]")
    st.raw(f"v_mov_b32 {KD(0)}, %[kdma]")
    st.raw(f"v_mov_b32 {VD(0)}, %[vdma]")
    # DMA piece i's sources (gen_w4_item.dma_setup: head_dim 128 / 64)
    for i in range(1, 4):
        if i < NPIECE:
            st.raw(f"v_add_u32 {KD(i)}, {1024 * i}, %[kdma]")
            st.raw(f"v_xor_b32 {KD(i)}, {64 * i}, {KD(i)}")
        if i < NPIECE and NT == 2:
            st.raw(f"v_add_u32 {VD(i)}, 1024, %[vdma]")
            st.raw(f"v_xor_b32 {VD(i)}, 32, {VD(i)}")
        elif i < NPIECE:
            st.raw(f"v_add_u32 {VD(i)}, {2048 * (i >> 1) + 128 * (i & 1)}, %[vdma]")
            if i >= 2:
                st.raw(f"v_xor_b32 {VD(i)}, 32, {VD(i)}")
        if i < NPIECE:
            st.raw(f"v_add_u32 {KOFF[i]}, {4096 * i}, %[koff]")
            st.raw(f"v_add_u32 {VOFF[i]}, {4096 * i}, %[voff]")
    st.raw(f"v_mov_b32 {VNINF}, {NINF}")
    for i in range(4):
        st.raw(f"v_mov_b32 v{184 + i}, {DT['one2']}")
    rsrc(st, 56, "%[qlo]", "%[qhi]", "%[qrec]")
    rsrc(st, 40, "%[klo]", "%[khi]", "%[kvrec]")
    rsrc(st, 44, "%[vlo]", "%[vhi]", "%[kvrec]")
    rsrc(st, 60, "%[olo]", "%[ohi]", "%[qrec]")
    # Q rows qr_b + r16, chunk g of k-step t: (qr_b << 8) + qoff + 64 t
    for b in range(nb()):
        st.raw(f"s_lshl_b32 {ST0}, {QR[b]}, {ROWSH}")
        st.raw(f"v_add_u32 {T[b]}, {ST0}, %[qoff]")
    for i in range(NPIECE):
        st.raw(f"v_add_u32 {T[4 + i]}, {hex(TILEB)}, {KOFF[i]}")
    st.nop(5)
    for b in range(nb()):
        for t in range(NT):
            st.raw(f"buffer_load_dwordx4 {R('v', 16 * b + 4 * t, 4)}, {T[b]}, {RQ}, 0 offen offset:{64 * t}")
    for i in range(NPIECE):
        st.raw(f"buffer_load_dwordx4 {KF(i)}, {KOFF[i]}, {SK}, 0 offen")
    for i in range(NPIECE):
        st.raw(f"buffer_load_dwordx4 {VST1(i)}, {VOFF[i]}, {SV}, 0 offen")
    for i in range(NPIECE):
        st.raw(f"buffer_load_dwordx4 {KST1(i)}, {T[4 + i]}, {SK}, 0 offen")
    # DMA descriptors start at K(2) / V(1)
    t2, t1 = hex(2 * TILEB), hex(TILEB)
    st.raw(f"s_add_u32 s40, s40, {t2}")
    st.raw("s_addc_u32 s41, s41, 0")
    st.raw(f"s_sub_i32 {SKREM}, s42, {t2}")
    st.raw(f"s_max_i32 s42, {SKREM}, 0")
    st.raw(f"s_add_u32 s44, s44, {t1}")
    st.raw("s_addc_u32 s45, s45, 0")
    st.raw(f"s_sub_i32 {SVREM}, s46, {t1}")
    st.raw(f"s_max_i32 s46, {SVREM}, 0")
    # O, l, -m_ref, m_ref = 0 (the function's blocks)
    for x in list(range(32 * nb())) + list(range(128, 128 + 4 * nb())):
        st.raw(f"v_accvgpr_write_b32 a{x}, 0")
    for x in range(96, 96 + 4 * nb()):
        st.raw(f"v_mov_b32 v{x}, 0")
    for b in range(nb()):
        st.raw(f"v_mov_b32 {MREF[b]}, 0")
    # Q and K(0) landed; V(0), K(1) may still fly
    st.raw(f"s_waitcnt vmcnt({2 * NPIECE})")
    for i in range(NPIECE):
        st.raw(f"ds_write_b128 %[klds], {KF(i)} offset:{KBUF[0] + PASSL * i}")
    q_scale(st)
    if not LATE_V0K1:
        st.raw("s_waitcnt vmcnt(0)")
        for i in range(NPIECE):
            st.raw(f"ds_write_b128 {vlds()}, {VST1(i)} offset:{vbuf(0) + PASSL * i}")
            st.raw(f"ds_write_b128 %[klds], {KST1(i)} offset:{KBUF[1] + PASSL * i}")
    if pdbl():
        # two tiles ahead: K(2), V(1) by LDS-DMA now (iteration 0's end waits)
        for i in range(NPIECE):
            st.raw(f"s_add_u32 m0, %[dmab], {kbuf(2) + 1024 * i}")
            st.nop(1)
            st.raw(f"buffer_load_dwordx4 {KD(i)}, {SK}, 0 offen lds")
        for i in range(NPIECE):
            st.raw(f"s_add_u32 m0, %[dmab], {vbuf_abs(1) + 1024 * i}")
            st.nop(1)
            st.raw(f"buffer_load_dwordx4 {VD(i)}, {SV}, 0 offen lds")
        tb = hex(TILEB)
        for ins in (f"s_add_u32 s40, s40, {tb}", "s_addc_u32 s41, s41, 0", f"s_sub_i32 {SKREM}, {SKREM}, {tb}",
                    f"s_max_i32 s42, {SKREM}, 0", f"s_add_u32 s44, s44, {tb}", "s_addc_u32 s45, s45, 0",
                    f"s_sub_i32 {SVREM}, {SVREM}, {tb}", f"s_max_i32 s46, {SVREM}, 0"):
            st.raw(ins)
    st.raw("s_waitcnt lgkmcnt(0)")
    st.raw("s_barrier")
    st.nop(2)
    # S(0) of the blocks with a tile (a prefix: T sorted descending)
    s0done = w4.newlabel("s0done")
    lbl = {n: w4.newlabel(f"s0n{n}") for n in range(1, nb() + 1)}
    for n in range(nb(), 1, -1):
        st.raw(f"s_cmp_lg_u32 {TB[n - 1]}, 0")
        st.branch("s_cbranch_scc1", lbl[n])
    st.branch("s_branch", lbl[1])
    for n in range(nb(), 0, -1):
        st.label(lbl[n])
        qk_plain(st, KBUF[0], n)
        st.branch("s_branch", s0done)
    st.label(s0done)
    if fp32scale():
        # every block's S(0) (the blocks without a tile hold zeros: harmless)
        for b in range(nb()):
            for cb in range(4):
                for ins in scale_ops(b, cb):
                    st.emit(ins)
    st.raw(f"s_mov_b32 {KV0}, 0")
    first_done = w4.newlabel("firstdone")
    for b in range(nb()):
        if b > 0:
            st.raw(f"s_cmp_eq_u32 {TB[b]}, 0")
            st.branch("s_cbranch_scc1", first_done)
        # tile 0 needs the limit mask only when it is the block's last tile
        nomask = w4.newlabel(f"nomask0_{b}")
        st.raw(f"s_cmp_eq_u32 {TB[b]}, 1")
        st.branch("s_cbranch_scc0", nomask)
        mask_block(st, b, causal)
        st.label(nomask)
        slow_softmax(st, [b], first=True)
        for e in exp_ops(b):
            st.emit(e)
    st.label(first_done)
    if LATE_V0K1:
        # V(0), K(1) landed under S(0) and the first softmax: their images
        # (unread by S(0)) are published by the barrier below
        st.raw("s_waitcnt vmcnt(0)")
        for i in range(NPIECE):
            st.raw(f"ds_write_b128 {vlds()}, {VST1(i)} offset:{vbuf(0) + PASSL * i}")
            st.raw(f"ds_write_b128 %[klds], {KST1(i)} offset:{KBUF[1] + PASSL * i}")
    # every wave's S(0) K reads are done before iteration 0's DMA refills kbuf[0]
    st.lgkm_all()
    st.raw("s_barrier")
    st.raw(f"s_mov_b32 {SJ}, 0")
    # NP of iteration 0: the blocks with a tile
    st.raw(f"s_mov_b32 {SNP}, 0")
    for b in range(nb()):
        st.raw(f"s_cmp_lg_u32 {TB[b]}, 0")
        st.raw(f"s_cselect_b32 {STMP}, 1, 0")
        st.raw(f"s_add_u32 {SNP}, {SNP}, {STMP}")
    if STAMPS:
        stamp_now(st, 72)
        st.raw("s_sub_u32 s89, s72, s76")


def epilogue_block(st, b):
    """O / l -> fp16 rows qr_b + r16 (M16::store_o: permlane16 swaps, dwordx4
    stores, sc1)"""
    l, inv = T[0], T[1]
    st.raw(f"s_lshl_b32 {ST1}, {QR[b]}, {ROWSH}")
    st.emit(valu(f"v_accvgpr_read_b32 {l}, {L(b, 0)}", r=[L(b, 0)], w=[l]))
    # inv = l > 0 ? 1.0f / l : 0  (IEEE division, the compiler's sequence)
    st.emit(valu(f"v_div_scale_f32 {T[2]}, {DIVS}, {l}, {l}, 1.0", r=[l], w=[T[2]]))
    st.emit(valu(f"v_rcp_f32_e32 {T[3]}, {T[2]}", r=[T[2]], w=[T[3]], kind="trans"))
    st.emit(valu(f"v_fma_f32 {T[4]}, -{T[2]}, {T[3]}, 1.0", r=[T[2], T[3]], w=[T[4]]))
    st.emit(valu(f"v_fmac_f32_e32 {T[3]}, {T[4]}, {T[3]}", r=[T[3], T[4]], w=[T[3]]))
    st.emit(valu(f"v_div_scale_f32 {T[4]}, vcc, 1.0, {l}, 1.0", r=[l], w=[T[4]]))
    st.emit(valu(f"v_mul_f32_e32 {T[5]}, {T[4]}, {T[3]}", r=[T[4], T[3]], w=[T[5]]))
    st.emit(valu(f"v_fma_f32 {T[6]}, -{T[2]}, {T[5]}, {T[4]}", r=[T[2], T[5], T[4]], w=[T[6]]))
    st.emit(valu(f"v_fmac_f32_e32 {T[5]}, {T[6]}, {T[3]}", r=[T[5], T[6], T[3]], w=[T[5]]))
    st.emit(valu(f"v_fma_f32 {T[2]}, -{T[2]}, {T[5]}, {T[4]}", r=[T[2], T[5], T[4]], w=[T[2]]))
    st.emit(valu(f"v_div_fmas_f32 {T[2]}, {T[2]}, {T[3]}, {T[5]}", r=[T[2], T[3], T[5]], w=[T[2]]))
    st.emit(valu(f"v_div_fixup_f32 {T[2]}, {T[2]}, {l}, 1.0", r=[T[2], l], w=[T[2]]))
    st.emit(valu(f"v_cmp_lt_f32 vcc, 0, {l}", r=[l]))
    st.emit(valu(f"v_cndmask_b32 {inv}, 0, {T[2]}, vcc", r=[T[2]], w=[inv]))
    st.emit(valu(f"v_add_u32 {T[7]}, {ST1}, %[ooff]", r=["%[ooff]"], w=[T[7]]))
    for ep in range(NE // 2):
        for x in range(2):
            e = 2 * ep + x
            for i in range(4):
                d = EPI[4 * x + i]
                st.emit(valu(f"v_accvgpr_read_b32 {d}, {O(b, e, i)}", r=[O(b, e, i)], w=[d]))
            for i in range(4 if not w4.mix() else 0):
                d = EPI[4 * x + i]
                st.emit(valu(f"v_mul_f32_e32 {d}, {d}, {inv}", r=[d, inv], w=[d]))
        X, Y = XY[0:2], XY[2:4]
        if w4.mix():
            for k, dst in enumerate(X + Y):
                for op in w4.mix_pk(dst, EPI[2 * k], EPI[2 * k + 1], inv):
                    st.emit(op)
        else:
            st.emit(valu(f"{DT['cvt_pk']} {X[0]}, {EPI[0]}, {EPI[1]}", r=EPI[0:2], w=[X[0]]))
            st.emit(valu(f"{DT['cvt_pk']} {X[1]}, {EPI[2]}, {EPI[3]}", r=EPI[2:4], w=[X[1]]))
            st.emit(valu(f"{DT['cvt_pk']} {Y[0]}, {EPI[4]}, {EPI[5]}", r=EPI[4:6], w=[Y[0]]))
            st.emit(valu(f"{DT['cvt_pk']} {Y[1]}, {EPI[6]}, {EPI[7]}", r=EPI[6:8], w=[Y[1]]))
        for dw in range(2):
            st.emit(valu(f"v_permlane16_swap_b32 {X[dw]}, {Y[dw]}", r=[X[dw], Y[dw]], w=[X[dw], Y[dw]]))
        st.emit(vmem(f"buffer_store_dwordx4 v[152:155], {T[7]}, {RO}, 0 offen offset:{64 * ep} sc1",
                     r=["v[152:155]", T[7]]))
    st.nop(2)


# ---------------------------------------------------------------------------
def double_iter(st, p, k, causal, Lb):
    """pdbl: steady tiles j, j+1 (j mod 4 = p) of kind (k, k), one barrier"""
    q = (p + 1) % nbuf()
    stamp_path(st, NB - k)
    left, late = phase_a(st, p, k, k)
    mid = Lb[f"dmid{k}"][p]
    phase_b(st, p, k, k, left, Lb[f"dslow1_{k}"][p], mid, late, kpre=p + 2)
    st.label(mid)
    left, late = phase_a(st, q, k, k, k0_issued=True)
    phase_b(st, q, k, k, left, Lb[f"dslow2_{k}"][p], Lb[f"dend{k}"][p], late)
    st.label(Lb[f"dend{k}"][p], drain_lgkm=True)
    stamp_path_end(st)
    if STAMPS:  # two tiles: count the path twice
        st.raw(f"s_add_u32 s{83 + NB - k}, s{83 + NB - k}, 1")
    st.raw("s_waitcnt vmcnt(0)")
    st.raw("s_barrier")
    if STAMPS:
        stamp_now(st, 72)
        st.raw("s_sub_u32 s75, s72, s76")
        st.raw("s_add_u32 s88, s88, s75")
    st.raw(f"s_add_u32 {SJ}, {SJ}, 2")
    st.raw(f"s_cmp_lt_u32 {SJ}, {TB[0]}")
    st.far("s_cbranch_scc1", Lb["loop"][(p + 2) % nbuf()])
    st.far("s_branch", Lb["done"])


def body(st, p, causal, Lb):
    """iteration j (parity p = j & 1): the kind of (NP, NQ) = (#{T_b > j},
    #{T_b > j+1}) -- NP carried from the previous iteration's NQ, NQ = NP
    unless block NP-1 ends at tile j (then NP-1, or 0 when every block does:
    equal tile counts) -- then the stage's DMA wait and the barrier"""
    K = lambda np_, nq: Lb["k_" + kname(np_, nq)][p]  # noqa: E731
    st.label(Lb["loop"][p], drain_lgkm=True)
    st.raw(f"s_add_u32 {SJ1}, {SJ}, 1")
    st.raw(f"s_add_u32 {SJ2}, {SJ}, 2")
    if pdbl() and p % 2 == 1:
        # kind (k, k) twice: T[k-1] >= j + 4 (every live block has tiles
        # j+1 and j+2, neither its last: no mask, no drain) -- the block
        # tile counts are the workgroup's, so every wave takes the same path
        single = w4.newlabel("single")
        st.raw(f"s_add_u32 {STMP}, {SJ}, 3")
        for k in range(1, nb() + 1):
            nxt = w4.newlabel("dnext")
            st.raw(f"s_cmp_eq_u32 {SNP}, {k}")
            st.branch("s_cbranch_scc0", nxt)
            st.raw(f"s_cmp_lt_u32 {STMP}, {TB[k - 1]}")
            st.branch("s_cbranch_scc0", single)
            double_iter(st, p, k, causal, Lb)
            st.label(nxt)
        st.label(single)
    lbl = {k: w4.newlabel(f"np{k}_") for k in range(1, nb() + 1)}
    for k in range(nb(), 1, -1):
        st.raw(f"s_cmp_eq_u32 {SNP}, {k}")
        st.branch("s_cbranch_scc1", lbl[k])
    for k in range(1, nb() + 1):
        if k > 1:
            st.label(lbl[k])
        st.raw(f"s_cmp_gt_u32 {TB[k - 1]}, {SJ1}")   # block k-1 has tile j+1: steady
        st.branch("s_cbranch_scc1", K(k, k))
        if k > 1:
            st.raw(f"s_cmp_eq_u32 {TB[0]}, {SJ1}")   # every block ends at tile j
            st.branch("s_cbranch_scc1", K(k, 0))
        st.branch("s_branch", K(k, k - 1))
    for np_, nq in kinds():
        st.label(K(np_, nq))
        st.raw(f"s_mov_b32 {SNP}, {nq}")             # NP of iteration j+1
        iteration(st, p, np_, nq, causal, Lb)
    st.label(Lb["end"][p], drain_lgkm=True)
    stamp_path_end(st)
    st.raw("s_waitcnt vmcnt(0)")   # this iteration's LDS-DMA landed before the barrier publishes it
    st.raw("s_barrier")
    if STAMPS:
        stamp_now(st, 72)
        st.raw("s_sub_u32 s75, s72, s76")
        st.raw("s_add_u32 s88, s88, s75")
    st.raw(f"s_add_u32 {SJ}, {SJ}, 1")
    st.raw(f"s_cmp_lt_u32 {SJ}, {TB[0]}")
    jump = st.far if pdbl() else st.branch
    if p < nbuf() - 1:
        jump("s_cbranch_scc0", Lb["done"])  # else on to body p + 1
    else:
        jump("s_cbranch_scc1", Lb["loop"][0])


def generate(causal):
    st = Stream()
    dl = [f"{d}{k}" for k in range(1, nb() + 1) for d in ("dmid", "dend", "dslow1_", "dslow2_")]
    Lb = {k: [w4.newlabel(f"{k}{p}") for p in range(nbuf())]
          for k in ["loop", "end"] + [f"k_{kname(*x)}" for x in kinds()] + [f"slow_{kname(*x)}" for x in kinds()] + dl}
    Lb["done"] = w4.newlabel("done")
    prologue(st, causal)
    for p in range(nbuf()):
        body(st, p, causal, Lb)
    st.label(Lb["done"], drain_lgkm=True)
    stamp_now(st, 76)
    end = w4.newlabel("epidone")
    for b in range(nb()):
        if b > 0:
            st.raw(f"s_cmp_eq_u32 {TB[b]}, 0")
            st.branch("s_cbranch_scc1", end)
        epilogue_block(st, b)
    st.label(end)
    if STAMPS:
        st.raw("s_waitcnt vmcnt(0)")
        stamp_now(st, 72)
        st.raw("s_sub_u32 s90, s72, s76")
        st.raw(f"s_lshl_b32 {ST1}, {QR[0]}, {ROWSH}")
        for i in range(13):
            st.raw(f"v_mov_b32 v{i}, s{78 + i}")
        for i in range(13, 16):
            st.raw(f"v_mov_b32 v{i}, 0")
        st.raw(f"v_mov_b32 v16, {ST1}")
        st.nop(2)
        for i in range(4):
            st.raw(f"buffer_store_dwordx4 v[{4 * i}:{4 * i + 3}], v16, {RO}, 0 offen offset:{16 * i}")
        st.raw("s_waitcnt vmcnt(0)")
    st.raw(f"s_mov_b32 m0, {SM0}")
    return st.out


HEADER = """// GENERATED by gen_w4p_item.py -- do not edit.
// One multi-block item (up to four 64-row query blocks x all key tiles) of the
// W4P tier: see the generator's docstring for the register map and the schedule.
#pragma once
"""


def header():
    # the head_dim-128 pair programs' LDS layout (fa_w4p_kernel.hpp): 1 = four
    # K / V images per tensor (two key tiles per barrier), 128 KiB
    set_hd(128)
    CURNB["nb"] = 2
    on = pdbl()
    CURNB["nb"] = 4
    on4 = pdbl()
    return HEADER + f"#define FA_W4P_DBL {1 if on else 0}\n#define FA_W4P_DBL4 {1 if on4 else 0}\n"


def cxx(causal, bf16, lines):
    body_ = "\n".join(f'      "{ln}\\n"' for ln in lines)
    vclob = ", ".join(f'"v{i}"' for i in range(NV))
    aclob = ", ".join(f'"a{i}"' for i in range(NA))
    sclob = ", ".join(f'"s{i}"' for i in range(NS_LO, NS_DIAG if STAMPS else NS_HI))
    name = (("w4p_item_causal" if causal else "w4p_item_noncausal") + ("_d64" if NT == 2 else "")
            + ("_nb2" if nb() == 2 else "") + ("_bf16" if bf16 else "_f16"))
    blocks = ",\n        ".join(f'[qr{b}] "s"(rn.qr[{b}]), [kvh{b}] "s"(rn.kvh[{b}]), [t{b}] "s"(rn.t[{b}])'
                                 for b in range(NB))
    return f"""
__device__ __forceinline__ void {name}(const W4PRun& rn, const W4Lane& ln) {{
  asm volatile(
{body_}
      :
      : [qlo] "s"(rn.qlo), [qhi] "s"(rn.qhi), [klo] "s"(rn.klo), [khi] "s"(rn.khi),
        [vlo] "s"(rn.vlo), [vhi] "s"(rn.vhi), [olo] "s"(rn.olo), [ohi] "s"(rn.ohi),
        [qrec] "s"(rn.qrec), [kvrec] "s"(rn.kvrec),
        {blocks},
        [c] "s"(rn.c), [dmab] "s"(rn.dmab),
        [ka0] "v"(ln.ka[0]), [ka1] "v"(ln.ka[1]), [ka2] "v"(ln.ka[2]), [ka3] "v"(ln.ka[3]),
        [va0] "v"(ln.va[0]), [va1] "v"(ln.va[1]), [koff] "v"(ln.koff), [voff] "v"(ln.voff),
        [klds] "v"(ln.klds), [vlds] "v"(ln.vlds), [vt] "v"(ln.vt), [r16] "v"(ln.r16),
        [qoff] "v"(ln.qoff), [ooff] "v"(ln.ooff), [kdma] "v"(ln.kdma), [vdma] "v"(ln.vdma)
      : "memory", "vcc", "scc", {sclob},
        {vclob},
        {aclob});
}}
"""


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "fa_w4p_item.inc"
    text = header()
    for hd in (128, 64):
        set_hd(hd)
        for bf16 in (False, True):
            set_dtype(bf16)
            for causal in (False, True):
                for n in (4, 2):
                    CURNB["nb"] = n
                    w4._lbl[0] = 0
                    text += cxx(causal, bf16, generate(causal))
                CURNB["nb"] = 4
    set_dtype(False)
    set_hd(128)
    with open(out, "w") as f:
        f.write(text)


if __name__ == "__main__":
    main()
