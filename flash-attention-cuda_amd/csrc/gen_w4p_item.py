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

NB = 4                 # query blocks per workgroup (at most)
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
NV = 214


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


def vahead(np_):
    """V^T fragments read ahead of their PV MFMAs: >= 8 MFMAs of cover for the
    LDS latency (at head_dim 64 at most the tile's 8)"""
    return min({1: 6, 2: 4}.get(np_, 3), 2 * NE)


def kslot(cb, t):
    """K fragment slot: two 16-key blocks' fragments at head_dim 128 (read one
    block ahead), the whole tile's 8 at 64"""
    return 4 * (cb & 1) + t if NT == 4 else 2 * cb + t


def k_read(t, cb, kb):
    s = kslot(cb, t)
    return dsr(f"ds_read_b128 {KF(s)}, {KADDR[t]} offset:{kb + 16 * ROWB * cb}", KF(s), KADDR[t])


def k_reads_tile(kb):
    """head_dim 64: every K fragment of the tile at once (the 8 slots hold it)"""
    return [k_read(t, cb, kb) for cb in range(4) for t in range(NT)]


def v_reads(f, vb):
    u, e = divmod(f, NE)
    slot = f % 8
    off = vb + 32 * ROWB * u + 512 * (e >> 1)
    a = VADDR[e & 1]
    return [dsr(f"ds_read_b64_tr_b16 {VF(slot, 0)}, {a} offset:{off}", VF(slot, 0), a),
            dsr(f"ds_read_b64_tr_b16 {VF(slot, 1)}, {a} offset:{off + 16 * ROWB}", VF(slot, 1), a)]


def qk_chain(b, cb):
    out = []
    for t in range(NT):
        c = NEGM(b) if t == 0 else S(b, cb)
        out.append(mfma(S(b, cb), KF(kslot(cb, t)), Q(b, t), c))
    return out


def cvt_block(b, cb):
    p = 64 + 8 * b + 4 * (cb >> 1) + 2 * (cb & 1)
    s = 16 * b + 4 * cb
    return [valu(f"{DT['cvt_pk']} v{p}, v{s}, v{s + 1}", r=[f"v{s}", f"v{s + 1}"], w=[f"v{p}"]),
            valu(f"{DT['cvt_pk']} v{p + 1}, v{s + 2}, v{s + 3}", r=[f"v{s + 2}", f"v{s + 3}"], w=[f"v{p + 1}"])]


def max_block(b, cb, first):
    return max_at(RMAX[b], 16 * b + 4 * cb, first)


def max_at(m, s, first):
    """running max m over the four scores v[s .. s+3] (first: starts it)"""
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
    """LDS-DMA of K(j+2) -> kbuf[p], V(j+1) -> vbuf[1-p]: (M0 set, load)
    pairs, then the descriptors advance one tile (gen_w4_item.dma_loads)"""
    pairs = []
    for i in range(NPIECE):
        pairs.append((salu(f"s_add_u32 m0, %[dmab], {KBUF[p] + 1024 * i}"),
                      vmem(f"buffer_load_dwordx4 {KD(i)}, {SK}, 0 offen lds", r=[KD(i)])))
    for i in range(NPIECE):
        pairs.append((salu(f"s_add_u32 m0, %[dmab], {VBUF[1 - p] + 1024 * i}"),
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
def phase_a(st, p, nq, np_):
    """QK^T(j+1) of blocks 0..nq-1 from kbuf[1-p] beside the fp16 conversion of
    P(j) of blocks 0..np-1 (each just before the chain that overwrites its
    scores), the running maxima of S(j+1), the K reads, the stage's LDS-DMA
    and the first V^T fragments of PV(j).  nq = 0 (the last tile): the
    conversions and V^T reads alone."""
    kb = KBUF[1 - p]
    va = vahead(np_)
    if nq == 0:
        for b in range(np_):
            for cb in range(4):
                for c in cvt_block(b, cb):
                    st.emit(c)
        for f in range(va):
            for r in v_reads(f, VBUF[p]):
                st.emit(r)
        return [], []
    chains = [(b, cb) for cb in range(4) for b in range(nq)]
    mf = []
    for b, cb in chains:
        mf += qk_chain(b, cb)
    n = len(mf)
    gaps = {}

    def put(k, ins):
        gaps.setdefault(k, []).extend(ins if isinstance(ins, list) else [ins])

    put(0, [k_read(t, 0, kb) for t in range(NT)] if NT == 4 else k_reads_tile(kb))
    for x, (b, cb) in enumerate(chains):
        c = cvt_block(b, cb)
        if cb == 0:
            put(0, c)
        else:
            put(NT * x - 1, c[0])
            put(NT * x, c[1])
        if b == 0 and cb < 3 and NT == 4:
            for t in range(NT):
                put(NT * x + 1 + t % 3, k_read(t, cb + 1, kb))
        if x >= lag():
            by, cby = chains[x - lag()]
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
        for i, r in enumerate(v_reads(f, VBUF[p])):
            put(min(max(0, n - 2 * va) + 2 * f + i, n), r)
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


def phase_b(st, p, nq, np_, leftover, label_slow, label_end, late=()):
    """PV(j) of blocks 0..np-1 from vbuf[p]; the rescale decision over the
    blocks 0..nq-1 at DEC_GAP, exp2 of their S(j+1) after it.  nq = 0: the
    PV alone."""
    vb = VBUF[p]
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
    emit_b(st, mf, gaps, dec, exs, lambda: slow_softmax(st, range(nq), first=False),
           label_slow, label_end)


def emit_b(st, mf, gaps, dec, exs, slow, label_slow, label_end):
    """phase B's emission: the MFMAs with their fillers, the rescale decision
    dec after gap DEC_GAP, the exp2s exs spread over the later gaps; the slow
    path (slow(), then the exp2s) behind the decision's branch"""
    n = len(mf)
    n_g = n - DEC_GAP
    for i, e in enumerate(exs):
        gaps.setdefault(DEC_GAP + 1 + (i * n_g) // len(exs), []).append(e)
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
    slow()
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
    row_max_regs(st, [f"v{16 * b + i}" for i in range(16)], dst)


def row_max_regs(st, s, dst):
    """dst = the row's max over the score registers s (16 or 8) and the 4 lanes of the row"""
    n = len(s)
    st.emit(valu(f"v_max3_f32 {dst}, {s[0]}, {s[1]}, {s[2]}", r=s[0:3], w=[dst]))
    for i in range(3, n - 1, 2):
        st.emit(valu(f"v_max3_f32 {dst}, {dst}, {s[i]}, {s[i + 1]}", r=[dst, s[i], s[i + 1]], w=[dst]))
    st.emit(valu(f"v_max_f32 {dst}, {dst}, {s[n - 1]}", r=[dst, s[n - 1]], w=[dst]))
    tmp = T[10]
    for sw in ("v_permlane16_swap_b32", "v_permlane32_swap_b32"):
        st.emit(valu(f"v_mov_b32 {tmp}, {dst}", r=[dst], w=[tmp]))
        st.emit(valu(f"{sw} {dst}, {tmp}", r=[dst, tmp], w=[dst, tmp]))
        st.emit(valu(f"v_max_f32 {dst}, {dst}, {tmp}", r=[dst, tmp], w=[dst]))


def shift_block(st, b, sh, first):
    """m_ref moves by sh: S -= sh, m_ref += sh, negm = -m_ref; O, l *= 2^-sh"""
    for ins in shift_ops([f"v{16 * b + i}" for i in range(16)], b, b, sh, first):
        st.emit(ins)


def shift_ops(sregs, ob, mb, sh, first):
    """shift_block's instructions: scores sregs, accumulators O(ob) / L(ob),
    m_ref MREF[mb] / NEGM(mb)"""
    out = []
    if not first:
        alpha = T[3]
        out.append(valu(f"v_exp_f32 {alpha}, -{sh}", r=[sh], w=[alpha], kind="trans"))
        regs = [O(ob, e, i) for e in range(NE) for i in range(4)] + [L(ob, i) for i in range(4)]
        for a in regs:
            out.append(valu(f"v_accvgpr_read_b32 {T[4]}, {a}", r=[a], w=[T[4]]))
            out.append(valu(f"v_mul_f32 {T[4]}, {T[4]}, {alpha}", r=[T[4], alpha], w=[T[4]]))
            out.append(valu(f"v_accvgpr_write_b32 {a}, {T[4]}", r=[T[4]], w=[a]))
    for x in sregs:
        out.append(valu(f"v_sub_f32 {x}, {x}, {sh}", r=[x, sh], w=[x]))
    out.append(valu(f"v_add_f32 {MREF[mb]}, {MREF[mb]}, {sh}", r=[MREF[mb], sh], w=[MREF[mb]]))
    for i in range(4):
        out.append(valu(f"v_xor_b32 {NEGM(mb, i)}, 0x80000000, {MREF[mb]}", r=[MREF[mb]], w=[NEGM(mb, i)]))
    return out


def mask_block(st, b, causal, qr=None, kvh=None, sbase=None, ncb=4):
    """S(b) = -inf where key >= kv_hi_b or (causal) key > query row, for the
    tile at key KV0 (key kv = KV0 + 16cb + 4sg + i, row = qr_b + r16):
    valid iff 16cb + i <= lim = min(kvh_b - KV0 - 1 - 4sg, qr_b - KV0 + r16 - 4sg).
    A tile inside both bounds gets lim >= 63: a no-op.  (The split phase:
    ncb = 2 key blocks at v[sbase ..], its own row base and bound.)"""
    qr = QR[b] if qr is None else qr
    kvh = KVH[b] if kvh is None else kvh
    sbase = 16 * b if sbase is None else sbase
    st.raw(f"s_sub_i32 {ST0}, {kvh}, {KV0}")
    st.raw(f"s_sub_i32 {ST0}, {ST0}, 1")
    st.raw(f"s_sub_i32 {ST1}, {qr}, {KV0}")
    lim_rag, lim = T[5], T[7]
    st.emit(valu(f"v_sub_u32 {T[6]}, %[vt], %[r16]", r=["%[vt]", "%[r16]"], w=[T[6]]))   # -4sg
    st.emit(valu(f"v_add_u32 {lim_rag}, {ST0}, {T[6]}", r=[T[6]], w=[lim_rag]))
    if causal:
        st.emit(valu(f"v_add_u32 {lim}, {ST1}, %[vt]", r=["%[vt]"], w=[lim]))
        st.emit(valu(f"v_min_i32 {lim}, {lim}, {lim_rag}", r=[lim, lim_rag], w=[lim]))
    else:
        lim = lim_rag
    for cb in range(ncb):
        for i in range(4):
            x = f"v{sbase + 4 * cb + i}"
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


# ---------------------------------------------------------------------------
# the split phase (W4_XP=split1, causal items whose blocks 2 and 3 are absent:
# the pairs).  Once block 1 is done, block 0 alone would cost every wave the
# whole K and V^T tile from LDS for 16 rows (LDS-bound: 4 x 32 KiB of reads per
# tile).  With >= NS_MIN key tiles left, the waves switch layout: wave w =
# (rh, kh) = (w >> 1, w & 1) takes rows 32 rh .. 32 rh + 31 of block 0 (two
# 16-row blocks i, rows QR[2 + i] + r16, whose scaled Q the prologue loaded
# into Q(2), Q(3)) against keys 32 kh .. 32 kh + 31 of every tile: half the
# LDS reads for the same MFMAs.  Each wave keeps an independent partial
# softmax per row block (O(2 + i), L(2 + i), MREF / NEGM / RMAX[2 + i], the
# first tile centred on its own row max); at the end each wave merges, for
# its own 16 rows, its old partial (O(0), keys before the switch), its own
# split partial and its partner's (w ^ 1) through LDS.
#   kind x (entry, iteration j): PV(j) of block 0 in the old layout, QK^T(j+1)
#                                in the split one, the split's first softmax
#   kind s (steady):             PV(j) / QK^T(j+1) split, lazy rescale
#   kind sd (drain):             PV(j) split
# ---------------------------------------------------------------------------
SPLIT_XP = "split1" in w4.XP
NS_MIN = int(os.environ.get("W4P_NSMIN", "3"))   # split tiles at least
SNP_X, SNP_S, SNP_DONE = 5, 6, 7
KAS = [R("v", 32 + t) for t in range(4)]   # K / V^T read addresses of the wave's key half
VAS = [R("v", 36 + x) for x in range(2)]
RS = [RMAX[2], RMAX[3]]


def split_on(causal):
    return SPLIT_XP and causal


def ss_base(i, c=0):        # split scores: row block i, key block c (of the half): S(1, 2i + c)
    return 16 + 8 * i + 4 * c


def va_s():
    return min(4, NE)


def split_setup(st):
    """the wave's key-half read addresses: + 32 kh rows"""
    st.raw(f"s_and_b32 {STMP}, {QR[0]}, 16")
    st.raw(f"s_lshl_b32 {STMP}, {STMP}, {ROWSH + 1}")
    for t in range(NT):
        st.emit(valu(f"v_add_u32 {KAS[t]}, {STMP}, {KADDR[t]}", r=[KADDR[t]], w=[KAS[t]]))
    for x in range(2):
        st.emit(valu(f"v_add_u32 {VAS[x]}, {STMP}, {VADDR[x]}", r=[VADDR[x]], w=[VAS[x]]))


def k_read_s(t, c, kb):
    s_ = kslot(c, t)
    return dsr(f"ds_read_b128 {KF(s_)}, {KAS[t]} offset:{kb + 16 * ROWB * c}", KF(s_), KAS[t])


def v_reads_s(e, vb):
    off = vb + 512 * (e >> 1)
    a = VAS[e & 1]
    return [dsr(f"ds_read_b64_tr_b16 {VF(e, 0)}, {a} offset:{off}", VF(e, 0), a),
            dsr(f"ds_read_b64_tr_b16 {VF(e, 1)}, {a} offset:{off + 16 * ROWB}", VF(e, 1), a)]


def qk_chain_s(i, c):
    out = []
    sreg = R("v", ss_base(i, c), 4)
    for t in range(NT):
        cc = NEGM(2 + i) if t == 0 else sreg
        out.append(mfma(sreg, KF(kslot(c, t)), Q(2 + i, t), cc))
    return out


def pv_mfmas_s():
    ms, ff = [], {}
    for e in range(NE):
        ff[e] = len(ms)
        for i in range(2):
            ms.append(mfma(O(2 + i, e), VF(e), P(1, i), O(2 + i, e)))
    ms += [mfma(L(2 + i), ONES, P(1, i), L(2 + i)) for i in range(2)]
    return ms, ff


def phase_a_split(st, p, mode):
    """mode x: QK^T(j+1) split beside block 0's P(j) conversion (old layout)
    and its first V^T reads; s: QK^T(j+1) split beside the split P(j)
    conversions, maxima, V^T reads; sd: conversions and V^T reads alone.
    The DMA as the one-block kind's."""
    kb = KBUF[1 - p]
    if mode == "sd":
        for i in range(2):
            for c in range(2):
                for ins in cvt_block(1, 2 * i + c):
                    st.emit(ins)
        for e in range(va_s()):
            for r in v_reads_s(e, VBUF[p]):
                st.emit(r)
        return [], []
    chains = [(i, c) for c in range(2) for i in range(2)]
    mf = []
    for i, c in chains:
        mf += qk_chain_s(i, c)
    n = len(mf)
    gaps = {}

    def put(k, ins):
        gaps.setdefault(k, []).extend(ins if isinstance(ins, list) else [ins])

    if NT == 4:
        put(0, [k_read_s(t, 0, kb) for t in range(NT)])
        for t in range(NT):
            put(1 + t % 3, k_read_s(t, 1, kb))
    else:
        put(0, [k_read_s(t, c, kb) for c in range(2) for t in range(NT)])
    if mode == "s":
        for x, (i, c) in enumerate(chains):
            cv = cvt_block(1, 2 * i + c)
            if x == 0:
                put(0, cv)
            else:
                put(NT * x - 1, cv[0])
                put(NT * x, cv[1])
            if x >= lag():
                iy, cy = chains[x - lag()]
                mm = max_at(RS[iy], ss_base(iy, cy), first=(cy == 0))
                put(min(NT * x + MAX_OFF, n), mm[0])
                put(min(NT * x + MAX_OFF + 1, n), mm[1])
    else:
        extra = [cv for cb in range(4) for cv in cvt_block(0, cb)]
        for k, cv in enumerate(extra):
            put(1 + (k * (n - 2)) // len(extra), cv)
    pairs, adv = dma_pieces(p)
    late = []
    if "p1dmaa" not in w4.XP:
        late = [ins for pr in pairs[NPIECE:] for ins in pr] + [i for g in adv[2:] for i in g]
        pairs, adv = pairs[:NPIECE], adv[:2]
    for k, (m0, ld) in enumerate(pairs):
        put(1 + k, m0)
        put(2 + k, ld)
    g = len(pairs) + 2
    for k, ins in enumerate(adv):
        put(min(g + k, n), ins)
    if mode == "s":
        va = va_s()
        for e in range(va):
            for k, r in enumerate(v_reads_s(e, VBUF[p])):
                put(min(max(0, n - 2 * va) + 2 * e + k, n), r)
    else:
        va = vahead(1)
        for f in range(va):
            for k, r in enumerate(v_reads(f, VBUF[p])):
                put(min(max(0, n - 2 * va) + 2 * f + k, n), r)
    assert max(gaps) <= n
    st.interleave(mf, gaps)
    left = []
    if mode == "s":
        for y in range(max(0, len(chains) - lag()), len(chains)):
            iy, cy = chains[y]
            left += max_at(RS[iy], ss_base(iy, cy), first=(cy == 0))
    return left, late


def mask_pass_s(st, causal):
    """tile j+1 is block 0's last: the limit mask of both split row blocks
    (key base KV0 + 32 kh), then their maxima again"""
    done = w4.newlabel("nomasks")
    st.raw(f"s_cmp_eq_u32 {TB[0]}, {SJ2}")
    st.branch("s_cbranch_scc0", done)
    st.raw(f"s_lshl_b32 {KV0}, {SJ1}, 6")
    st.raw(f"s_and_b32 {STMP}, {QR[0]}, 16")
    st.raw(f"s_lshl_b32 {STMP}, {STMP}, 1")
    st.raw(f"s_add_u32 {KV0}, {KV0}, {STMP}")
    for i in range(2):
        mask_block(st, 0, causal, qr=QR[2 + i], kvh=KVH[0], sbase=ss_base(i), ncb=2)
        for c in range(2):
            for ins in max_at(RS[i], ss_base(i, c), first=(c == 0)):
                st.emit(ins)
    st.label(done)


def first_softmax_s_ops():
    """the split's first tile: every row of each row block centres on its
    max over the wave's key half (slow_softmax(first=True)'s arithmetic)"""
    class Sink:
        def __init__(self):
            self.ops = []

        def emit(self, ins):
            self.ops.append(ins)
    sk = Sink()
    for i in range(2):
        sregs = [f"v{ss_base(i) + k}" for k in range(8)]
        mx, sh = T[1], T[2]
        row_max_regs(sk, sregs, mx)
        sk.emit(valu(f"v_cmp_eq_f32 vcc, {VNINF}, {mx}", r=[VNINF, mx]))
        sk.emit(valu(f"v_cndmask_b32_e64 {sh}, {mx}, 0, vcc", r=[mx], w=[sh]))
        sk.ops += shift_ops(sregs, 2 + i, 2 + i, sh, first=True)
    return sk.ops


def slow_softmax_s(st):
    for i in range(2):
        skip = w4.newlabel("pskips")
        st.emit(valu(f"v_cmp_lt_f32 vcc, {RESCALE}, {RS[i]}", r=[RS[i]]))
        st.branch("s_cbranch_vccz", skip)
        sregs = [f"v{ss_base(i) + k}" for k in range(8)]
        mx, sh = T[1], T[2]
        row_max_regs(st, sregs, mx)
        st.emit(valu(f"v_max_f32 {sh}, 0, {mx}", r=[mx], w=[sh]))
        for ins in shift_ops(sregs, 2 + i, 2 + i, sh, first=False):
            st.emit(ins)
        st.label(skip)


def phase_b_split(st, p, mode, leftover, label_slow, label_end, late):
    vb = VBUF[p]
    gaps = {}

    def put(k, ins):
        gaps.setdefault(k, []).extend(ins if isinstance(ins, list) else [ins])

    for k, ins in enumerate(late):
        put(1 + k, ins)
    if mode == "x":
        mf, ff = pv_mfmas(1)
        va = vahead(1)
        for f in range(va, 2 * NE):
            r = v_reads(f, vb)
            put(ff[f - va] + 1, r[0])
            put(ff[f - va] + 2, r[1])
        n = len(mf)
        ops = first_softmax_s_ops() + exp_ops(1)
        for k, ins in enumerate(ops):
            put(1 + (k * (n - 1)) // len(ops), ins)
        st.interleave(mf, gaps)
        st.branch("s_branch", label_end)
        return
    mf, ff = pv_mfmas_s()
    va = va_s()
    for e in range(va, NE):
        r = v_reads_s(e, vb)
        put(ff[e - va] + 1, r[0])
        put(ff[e - va] + 2, r[1])
    if mode == "sd":
        st.interleave(mf, gaps)
        st.branch("s_branch", label_end)
        return
    lo = [LEFT_OFF + (i if NT == 4 else i // 2) for i in range(len(leftover))]
    for k, ins in zip(lo, leftover):
        put(k, ins)
    assert not leftover or lo[-1] <= DEC_GAP
    dec = [valu(f"v_max_f32 {T[0]}, {RS[0]}, {RS[1]}", r=RS, w=[T[0]]),
           valu(f"v_cmp_lt_f32 vcc, {RESCALE}, {T[0]}", r=[T[0]])]
    emit_b(st, mf, gaps, dec, exp_ops(1), lambda: slow_softmax_s(st), label_slow, label_end)


def iteration_split(st, p, mode, causal, Lb):
    stamp_path(st, NPATH - 1 if mode == "sd" else NB - 1)
    if mode == "x":
        split_setup(st)
    left, late = phase_a_split(st, p, mode)
    if mode == "s":
        mask_pass_s(st, causal)
    phase_b_split(st, p, mode, left, Lb["slow_s"][p], Lb["end"][p], late)


def split_merge(st):
    """after the loop (SNP = SNP_DONE): wave w hands its split partial of the
    partner's row block (1 - kh) to LDS, takes the partner's of its own, and
    merges them with its own split partial and its old one into O(0) / L(0)"""
    reg = NE * 1024 + 512                       # bytes per wave: O^T (NE x 1 KiB) then m, l
    base, wb, rb = "s40", "s41", "s42"
    st.raw(f"s_and_b32 {ST0}, {QR[0]}, 48")      # 16 w
    st.raw(f"s_lshl_b32 {base}, {ST0}, {ROWSH}")
    st.raw(f"s_sub_u32 {base}, %[dmab], {base}")  # the images' base
    st.raw(f"s_mul_i32 {wb}, {ST0}, {reg // 16}")
    st.raw(f"s_add_u32 {wb}, {wb}, {base}")
    st.raw(f"s_xor_b32 {rb}, {ST0}, 16")
    st.raw(f"s_mul_i32 {rb}, {rb}, {reg // 16}")
    st.raw(f"s_add_u32 {rb}, {rb}, {base}")
    ln, aw, ar, mw, mr = "v40", "v41", "v42", "v43", "v44"
    st.raw(f"v_mbcnt_lo_u32_b32 {ln}, -1, 0")
    st.raw(f"v_mbcnt_hi_u32_b32 {ln}, -1, {ln}")
    st.raw(f"v_lshlrev_b32 {aw}, 4, {ln}")
    st.raw(f"v_lshlrev_b32 {mw}, 3, {ln}")
    st.raw(f"v_add_u32 {ar}, {rb}, {aw}")
    st.raw(f"v_add_u32 {aw}, {wb}, {aw}")
    st.raw(f"v_add_u32 {mr}, {rb}, {mw}")
    st.raw(f"v_add_u32 {mw}, {wb}, {mw}")
    st.nop(2)
    kh1, wdone = w4.newlabel("mkh1"), w4.newlabel("mwdone")
    st.raw(f"s_and_b32 {STMP}, {QR[0]}, 16")
    st.raw(f"s_cmp_eq_u32 {STMP}, 0")
    st.branch("s_cbranch_scc0", kh1)
    for kh in range(2):
        if kh:
            st.label(kh1)
        i = 1 - kh                               # the partner's row block
        for e in range(NE):
            for k in range(4):
                st.emit(valu(f"v_accvgpr_read_b32 v{4 * e + k}, {O(2 + i, e, k)}",
                             r=[O(2 + i, e, k)], w=[f"v{4 * e + k}"]))
        st.emit(valu(f"v_mov_b32 v48, {MREF[2 + i]}", r=[MREF[2 + i]], w=["v48"]))
        st.emit(valu(f"v_accvgpr_read_b32 v49, {L(2 + i, 0)}", r=[L(2 + i, 0)], w=["v49"]))
        st.nop(1)
        for e in range(NE):
            st.emit(w4.dsw(f"ds_write_b128 {aw}, v[{4 * e}:{4 * e + 3}] offset:{1024 * e}", aw,
                           f"v[{4 * e}:{4 * e + 3}]"))
        st.emit(w4.dsw(f"ds_write_b64 {mw}, v[48:49] offset:{NE * 1024}", mw, "v[48:49]"))
        st.branch("s_branch", wdone)
    st.label(wdone)
    st.lgkm_all()
    st.raw("s_barrier")
    for e in range(NE):
        st.emit(dsr(f"ds_read_b128 v[{4 * e}:{4 * e + 3}], {ar} offset:{1024 * e}",
                    f"v[{4 * e}:{4 * e + 3}]", ar))
    st.emit(dsr(f"ds_read_b64 v[48:49], {mr} offset:{NE * 1024}", "v[48:49]", mr))
    st.lgkm_all()
    kh1, mdone = w4.newlabel("mmkh1"), w4.newlabel("mmdone")
    st.raw(f"s_cmp_eq_u32 {STMP}, 0")
    st.branch("s_cbranch_scc0", kh1)
    m, a0, a1, a2, t = T[0], T[1], T[2], T[3], T[4]
    for kh in range(2):
        if kh:
            st.label(kh1)
        ms = MREF[2 + kh]
        st.emit(valu(f"v_max3_f32 {m}, {MREF[0]}, {ms}, v48", r=[MREF[0], ms, "v48"], w=[m]))
        for dst, src in ((a0, MREF[0]), (a1, ms), (a2, "v48")):
            st.emit(valu(f"v_sub_f32 {dst}, {src}, {m}", r=[src, m], w=[dst]))
        for x in (a0, a1, a2):
            st.emit(valu(f"v_exp_f32 {x}, {x}", r=[x], w=[x], kind="trans"))
        regs = [(O(0, e, k), O(2 + kh, e, k), f"v{4 * e + k}") for e in range(NE) for k in range(4)]
        regs.append((L(0, 0), L(2 + kh, 0), "v49"))
        for o0, o1, o2 in regs:
            st.emit(valu(f"v_accvgpr_read_b32 {t}, {o0}", r=[o0], w=[t]))
            st.emit(valu(f"v_accvgpr_read_b32 {T[5]}, {o1}", r=[o1], w=[T[5]]))
            st.emit(valu(f"v_mul_f32 {t}, {t}, {a0}", r=[t, a0], w=[t]))
            st.emit(valu(f"v_fmac_f32_e32 {t}, {T[5]}, {a1}", r=[t, T[5], a1], w=[t]))
            st.emit(valu(f"v_fmac_f32_e32 {t}, {o2}, {a2}", r=[t, o2, a2], w=[t]))
            st.emit(valu(f"v_accvgpr_write_b32 {o0}, {t}", r=[t], w=[o0]))
        st.branch("s_branch", mdone)
    st.label(mdone)


# iteration kinds (NP, NQ): steady, one block's drain, every block's drain
KINDS = [(k, k) for k in range(1, NB + 1)] + [(k, k - 1) for k in range(1, NB + 1)] + \
        [(k, 0) for k in range(2, NB + 1)]


def kname(np_, nq):
    return f"k{np_}{nq}"


def iteration(st, p, np_, nq, causal, Lb):
    stamp_path(st, NB - nq if nq else NPATH - 1)   # 0: 4 QK blocks .. 3: 1; 4: drain
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
    qregs = [16 * b + j for b in range(NB) for j in range(4 * NT)]  # Q(b, t) raw: v[16b + 4t ..]
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
    for b in range(NB):
        st.raw(f"s_lshl_b32 {ST0}, {QR[b]}, {ROWSH}")
        st.raw(f"v_add_u32 {T[b]}, {ST0}, %[qoff]")
    for i in range(NPIECE):
        st.raw(f"v_add_u32 {T[4 + i]}, {hex(TILEB)}, {KOFF[i]}")
    st.nop(5)
    for b in range(NB):
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
    # O, l, -m_ref, m_ref = 0
    for x in range(144):
        st.raw(f"v_accvgpr_write_b32 a{x}, 0")
    for x in range(96, 112):
        st.raw(f"v_mov_b32 v{x}, 0")
    for b in range(NB):
        st.raw(f"v_mov_b32 {MREF[b]}, 0")
    # Q and K(0) landed; V(0), K(1) may still fly
    st.raw(f"s_waitcnt vmcnt({2 * NPIECE})")
    for i in range(NPIECE):
        st.raw(f"ds_write_b128 %[klds], {KF(i)} offset:{KBUF[0] + PASSL * i}")
    q_scale(st)
    st.raw("s_waitcnt vmcnt(0)")
    for i in range(NPIECE):
        st.raw(f"ds_write_b128 %[vlds], {VST1(i)} offset:{VBUF[0] + PASSL * i}")
        st.raw(f"ds_write_b128 %[klds], {KST1(i)} offset:{KBUF[1] + PASSL * i}")
    st.raw("s_waitcnt lgkmcnt(0)")
    st.raw("s_barrier")
    st.nop(2)
    # S(0) of the blocks with a tile (a prefix: T sorted descending)
    s0done = w4.newlabel("s0done")
    lbl = {nb: w4.newlabel(f"s0n{nb}") for nb in range(1, NB + 1)}
    for nb in range(NB, 1, -1):
        st.raw(f"s_cmp_lg_u32 {TB[nb - 1]}, 0")
        st.branch("s_cbranch_scc1", lbl[nb])
    st.branch("s_branch", lbl[1])
    for nb in range(NB, 0, -1):
        st.label(lbl[nb])
        qk_plain(st, KBUF[0], nb)
        st.branch("s_branch", s0done)
    st.label(s0done)
    st.raw(f"s_mov_b32 {KV0}, 0")
    first_done = w4.newlabel("firstdone")
    for b in range(NB):
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
    # every wave's S(0) K reads are done before iteration 0's DMA refills kbuf[0]
    st.lgkm_all()
    st.raw("s_barrier")
    st.raw(f"s_mov_b32 {SJ}, 0")
    # NP of iteration 0: the blocks with a tile
    st.raw(f"s_mov_b32 {SNP}, 0")
    for b in range(NB):
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
def body(st, p, causal, Lb):
    """iteration j (parity p = j & 1): the kind of (NP, NQ) = (#{T_b > j},
    #{T_b > j+1}) -- NP carried from the previous iteration's NQ, NQ = NP
    unless block NP-1 ends at tile j (then NP-1, or 0 when every block does:
    equal tile counts) -- then the stage's DMA wait and the barrier"""
    K = lambda np_, nq: Lb["k_" + kname(np_, nq)][p]  # noqa: E731
    st.label(Lb["loop"][p], drain_lgkm=True)
    st.raw(f"s_add_u32 {SJ1}, {SJ}, 1")
    st.raw(f"s_add_u32 {SJ2}, {SJ}, 2")
    lbl = {k: w4.newlabel(f"np{k}_") for k in range(1, NB + 1)}
    if split_on(causal):
        lsp = w4.newlabel("npsplit")
        st.raw(f"s_cmp_gt_u32 {SNP}, {NB}")
        st.branch("s_cbranch_scc1", lsp)
    for k in range(NB, 1, -1):
        st.raw(f"s_cmp_eq_u32 {SNP}, {k}")
        st.branch("s_cbranch_scc1", lbl[k])
    for k in range(1, NB + 1):
        if k > 1:
            st.label(lbl[k])
        st.raw(f"s_cmp_gt_u32 {TB[k - 1]}, {SJ1}")   # block k-1 has tile j+1: steady
        st.branch("s_cbranch_scc1", K(k, k))
        if k > 1:
            st.raw(f"s_cmp_eq_u32 {TB[0]}, {SJ1}")   # every block ends at tile j
            st.branch("s_cbranch_scc1", K(k, 0))
        st.branch("s_branch", K(k, k - 1))
    for np_, nq in KINDS:
        st.label(K(np_, nq))
        st.raw(f"s_mov_b32 {SNP}, {nq}")             # NP of iteration j+1
        if split_on(causal) and (np_, nq) == (2, 1):
            # block 1 ends here: the split phase follows when blocks 2, 3 are
            # absent and block 0 has >= NS_MIN tiles after the entry kind's
            st.raw(f"s_add_u32 {STMP}, {SJ}, {2 + NS_MIN}")
            st.raw(f"s_cmp_eq_u32 {TB[2]}, 0")
            st.raw(f"s_cselect_b32 {STMP}, {STMP}, 0x7fffffff")
            st.raw(f"s_cmp_ge_u32 {TB[0]}, {STMP}")
            st.raw(f"s_cselect_b32 {SNP}, {SNP_X}, 1")
        iteration(st, p, np_, nq, causal, Lb)
    if split_on(causal):
        st.label(lsp)
        st.raw(f"s_cmp_eq_u32 {SNP}, {SNP_X}")
        st.branch("s_cbranch_scc1", Lb["k_x"][p])
        st.raw(f"s_cmp_gt_u32 {TB[0]}, {SJ1}")
        st.branch("s_cbranch_scc1", Lb["k_s"][p])
        st.branch("s_branch", Lb["k_sd"][p])
        for mode, nxt in (("x", SNP_S), ("s", SNP_S), ("sd", SNP_DONE)):
            st.label(Lb["k_" + mode][p])
            st.raw(f"s_mov_b32 {SNP}, {nxt}")
            iteration_split(st, p, mode, causal, Lb)
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
    if p == 0:
        st.branch("s_cbranch_scc0", Lb["done"])
    else:
        st.branch("s_cbranch_scc1", Lb["loop"][0])


def generate(causal):
    st = Stream()
    Lb = {k: [w4.newlabel(f"{k}{p}") for p in range(2)]
          for k in ["loop", "end"] + [f"k_{kname(*x)}" for x in KINDS] + [f"slow_{kname(*x)}" for x in KINDS]}
    Lb["done"] = w4.newlabel("done")
    if split_on(causal):
        for k in ("k_x", "k_s", "k_sd", "slow_s"):
            Lb[k] = [w4.newlabel(f"{k}{p}") for p in range(2)]
    prologue(st, causal)
    body(st, 0, causal, Lb)
    body(st, 1, causal, Lb)
    st.label(Lb["done"], drain_lgkm=True)
    stamp_now(st, 76)
    if split_on(causal):
        nomerge = w4.newlabel("nomerge")
        st.raw(f"s_cmp_eq_u32 {SNP}, {SNP_DONE}")
        st.branch("s_cbranch_scc0", nomerge)
        split_merge(st)
        st.label(nomerge)
    end = w4.newlabel("epidone")
    for b in range(NB):
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


def cxx(causal, bf16, lines):
    body_ = "\n".join(f'      "{ln}\\n"' for ln in lines)
    vclob = ", ".join(f'"v{i}"' for i in range(NV))
    aclob = ", ".join(f'"a{i}"' for i in range(NA))
    sclob = ", ".join(f'"s{i}"' for i in range(NS_LO, NS_DIAG if STAMPS else NS_HI))
    name = (("w4p_item_causal" if causal else "w4p_item_noncausal") + ("_d64" if NT == 2 else "")
            + ("_bf16" if bf16 else "_f16"))
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
    text = HEADER
    for hd in (128, 64):
        set_hd(hd)
        for bf16 in (False, True):
            set_dtype(bf16)
            for causal in (False, True):
                w4._lbl[0] = 0
                text += cxx(causal, bf16, generate(causal))
    set_dtype(False)
    set_hd(128)
    with open(out, "w") as f:
        f.write(text)


if __name__ == "__main__":
    main()
