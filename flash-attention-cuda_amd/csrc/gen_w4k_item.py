#!/usr/bin/env python3
"""Generator of the short-launch segment program (fa_w4k_item.inc).

The short tier (fa_w4k_kernel.hpp) gives each workgroup one or two 64-row
query blocks and flattens their key tiles into one list that its four waves
split into contiguous quarters: a wave runs one "segment" (its 64 query rows
against a contiguous run of key tiles) per block its quarter touches, and
leaves a partial result in LDS that the workgroup merges at the end.  Unlike
the persistent W4 program (gen_w4_item.py), the waves of a workgroup never
read the same K/V tile, so a segment is a barrier-free pipeline of its own:

  K tiles go straight from global memory into the K operand registers (a K
  fragment row is 16 contiguous bytes of a key row), a whole 64-key tile at a
  time, single-buffered: the loads of tile j+2 are issued key block by key
  block right after the QK^T chains that read tile j+1's fragments.
  V tiles go by LDS-DMA into the wave's own double-buffered V image and are
  read transposed (ds_read_b64_tr_b16) as in W4.

Register map (per wave; the W4 map where the roles agree):

  VGPR  v0-63    S^T tile, 4 row blocks b x 4 key blocks cb x 4 (fp32 -> exp2)
        v64-95   P (fp16), B operands of PV
        v96-111  -m_ref per row block (C operand of the QK^T chains)
        v112-175 K tile: fragment (cb, t) at v112 + 16 cb + 4 t
        v176-207 V^T fragments (8 slots)
        v208-217 ones, m_ref, running maxima     v218-221 DMA source offsets
        v222-223 V^T read addresses (this iteration's image)
        v224 -inf, v225-235 temporaries
  AGPR  a0-127 O^T, a128-143 l, a144-207 Q (pre-scaled)

Per key tile j: phase A = QK^T(j+1) beside cvt P(j), the maxima of S(j+1), the
LDS-DMA of V(j+1) into the other image and the K(j+2) loads; phase B = PV(j)
beside exp2 of S(j+1) and the V^T reads.  Outstanding vector-memory operations
are tracked like LDS reads (counted vmcnt at first use).  The arithmetic is
W4's (gen_w4_item.py) operation for operation: the segment's partial result
matches what W4 computes over the same keys before the final normalisation.
The segment ends by writing its normalised O (fp16) and per-row log2-sum-exp
(m_ref + log2 l) to LDS.

usage: python3 gen_w4k_item.py [OUT.inc]      (the Makefile runs it)
"""
import itertools
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_w4_item as g  # noqa: E402
from gen_w4_item import (Ins, Stream, mfma, valu, dsr, dsw, vmem, salu, R, S, P, NEGM,  # noqa: E402
                         ONES, MREF, RMAX, VNINF, T, O, L, Q, NINF, DT, cvt_block,
                         max_block, exp_ops, slow_softmax, mask_last_tile, full_max,
                         newlabel)

XP = set(os.environ.get("W4K_XP", "").split(",")) - {""}
V_AHEAD = int(os.environ.get("W4K_V_AHEAD", "3"))
# diagnostic builds only (never the product library): W4K_DIAG=stamps writes
# s_memtime at the segment's start, after its prologue, at the drain and after
# the epilogue over its log2-sum-exp row (fa_w4k_kernel.hpp FA_W4K_STAMPS
# copies them to O instead of merging)
DIAG = os.environ.get("W4K_DIAG", "")


def kstamp(st, i):
    if DIAG == "stamps":
        st.raw(f"s_memtime s[{76 + 2 * i}:{77 + 2 * i}]")
        st.raw("s_waitcnt lgkmcnt(0)")
        st.lgkm = []
_uid = itertools.count()


class VStream(Stream):
    """Stream + outstanding vector-memory operations (vmcnt counts loads,
    stores and LDS-DMA together, in issue order)"""

    def __init__(self):
        super().__init__()
        self.vm = []  # (destination registers, tag, uid), oldest first

    def _snap(self):
        return (Stream._snap(self), list(self.vm))

    def _restore(self, snaps):
        Stream._restore(self, [s[0] for s in snaps])
        lists = [s[1] for s in snaps]
        self.vm = []
        if lists:
            # every path into a label must carry the same vector-memory
            # operations in the same order (counted waits rely on it)
            tags0 = [t for _, t, _ in lists[0]]
            for other in lists[1:]:
                assert [t for _, t, _ in other] == tags0, "vmem paths differ at a label"
            self.vm = list(lists[0])

    def wait_vm(self, regs=(), tags=()):
        need, tags = set(regs), set(tags)
        last = -1
        for i, (dst, tag, _) in enumerate(self.vm):
            if dst & need or tag in tags:
                last = i
        if last < 0:
            return
        after = len(self.vm) - 1 - last
        assert after <= 63
        self.raw(f"s_waitcnt vmcnt({after})")
        self.vm = self.vm[last + 1:]

    def vm_all(self):
        if self.vm:
            self.raw("s_waitcnt vmcnt(0)")
            self.vm = []

    def emit(self, ins):
        if isinstance(ins, Ins):
            if ins.kind == "vmwait":
                self.wait_vm(tags=ins.tags)
                return
            # a load's destination must have landed before any use or overwrite
            self.wait_vm(regs=ins.r + ins.w)
        Stream.emit(self, ins)
        if isinstance(ins, Ins) and ins.kind == "vmem":
            self.vm.append((set(ins.w), getattr(ins, "tag", None), next(_uid)))

    def retag(self, old, new):
        self.vm = [(d, new if t == old else t, u) for d, t, u in self.vm]


def vmwait(*tags):
    i = Ins("", "vmwait")
    i.tags = tags
    return i


def tagged(ins, tag):
    ins.tag = tag
    return ins


# ---------------------------------------------------------------------------
# register map (the differences from W4)
# ---------------------------------------------------------------------------
def KF(cb, t):
    return R("v", 112 + 16 * cb + 4 * t, 4)


def VF(slot, half=None):
    base = 176 + 4 * slot
    return R("v", base, 4) if half is None else R("v", base + 2 * half, 2)


VD = [R("v", 218 + i) for i in range(4)]   # DMA source offsets of pieces i (per 4-KiB group)
VA = [R("v", 222), R("v", 223)]            # V^T read addresses (current image)

# scalars (clobbered)
SK, SV = "s[40:43]", "s[44:47]"             # K / V descriptors (next tile to load)
SKREM, SVREM = "s48", "s49"                  # their remaining bytes (signed)
SJ, SJ1 = "s50", "s51"                       # j, j + 1
SN = "s52"                                   # tiles of the segment
SMASKJ = "s54"                               # n if the last tile needs a mask, else -1
ST0, ST1 = "s55", "s56"                      # (mask_last_tile's scratch)
SOFF = ["s60", "s61", "s62", "s63"]          # 0, 4 KiB, 8 KiB, 12 KiB
SIMG, SOTH, SDELTA = "s64", "s65", "s66"     # current / other V image, +-16 KiB
SKVHI, SQM = "s57", "s67"                    # key bound, first row (segment-relative)
SPSLOT, SLSLOT = "s68", "s69"                # partial O slot, log2-sum-exp row
SM0 = "s70"
RQ = "s[72:75]"
assert g.ST0 == ST0 and g.ST1 == ST1


def vtr_reads(u, e, slot):
    """V^T fragment (u, e) from the current image into slot"""
    off = 8192 * u + 512 * (e >> 1)
    a = VA[e & 1]
    return [dsr(f"ds_read_b64_tr_b16 {VF(slot, 0)}, {a} offset:{off}", VF(slot, 0), a),
            dsr(f"ds_read_b64_tr_b16 {VF(slot, 1)}, {a} offset:{off + 4096}", VF(slot, 1), a)]


def qk_chain(b, cb):
    out = []
    for t in range(4):
        c = NEGM(b) if t == 0 else S(b, cb)
        out.append(mfma(S(b, cb), KF(cb, t), Q(b, t), c))
    return out


def k_loads(cb):
    """the next tile's K fragments of key block cb (offset 4096 cb + 64 t)"""
    return [vmem(f"buffer_load_dwordx4 {KF(cb, t)}, %[kg], {SK}, {SOFF[cb]} offen offset:{64 * t}",
                 r=["%[kg]"], w=[KF(cb, t)]) for t in range(4)]


def k_advance():
    return [salu("s_add_u32 s40, s40, 0x4000"), salu("s_addc_u32 s41, s41, 0"),
            salu(f"s_sub_i32 {SKREM}, {SKREM}, 0x4000"), salu(f"s_max_i32 s42, {SKREM}, 0")]


def v_dma(target):
    """the next V tile -> image `target` (SGPR): piece p = 4 w + i covers image
    bytes [1024 p, +1024); per 4-KiB group w the descriptor moves 4 KiB, so the
    per-lane sources VD(i) are W4's (one wave's 4 pieces); M0 is set one
    instruction ahead of each piece.  Returns (m0 writes, loads) pairs."""
    out = []
    for w in range(4):
        for i in range(4):
            p = 4 * w + i
            out.append((salu(f"s_add_u32 m0, {target}, {1024 * p}"),
                        tagged(vmem(f"buffer_load_dwordx4 {VD[i]}, {SV}, 0 offen lds", r=[VD[i]]),
                               ("V", "cur"))))
        adv = [salu("s_add_u32 s44, s44, 0x1000"), salu("s_addc_u32 s45, s45, 0"),
               salu(f"s_sub_i32 {SVREM}, {SVREM}, 0x1000"), salu(f"s_max_i32 s46, {SVREM}, 0")]
        out[-1] = (out[-1][0], out[-1][1], adv)
    return out


def pv_mfmas():
    ms, frag_first = [], {}
    for u in range(2):
        for e in range(8):
            f = u * 8 + e
            frag_first[f] = len(ms)
            for b in range(4):
                ms.append(mfma(O(b, e), VF(f % 8), P(b, u), O(b, e)))
        for b in range(4):
            ms.append(mfma(L(b), ONES, P(b, u), L(b)))
    return ms, frag_first


# ---------------------------------------------------------------------------
# phases
# ---------------------------------------------------------------------------
def phase_a(st, with_max, diag=False):
    """QK^T(j+1) beside cvt P(j), maxima of S(j+1), the DMA of V(j+1) into the
    other image, the K(j+2) loads and the first V^T reads of PV(j).
    Returns the fillers left for phase B."""
    chains = [(b, cb) for cb in range(4) for b in range(4) if not diag or cb <= b]
    mf = []
    last_of_cb = {}
    for (b, cb) in chains:
        mf += qk_chain(b, cb)
        last_of_cb[cb] = len(mf) - 1
    n = len(mf)
    gaps = {}

    def put(k, ins):
        gaps.setdefault(k, []).extend(ins if isinstance(ins, list) else [ins])

    if diag:
        above = [(b, cb) for cb in range(4) for b in range(4) if cb > b]
        for k, (b, cb) in enumerate(above):
            ins = cvt_block(b, cb)
            ins += [valu(f"v_mov_b32 {S(b, cb, i)}, {VNINF}", r=[VNINF], w=[S(b, cb, i)]) for i in range(4)]
            put(5 + 5 * k, ins)
    for x, (b, cb) in enumerate(chains):
        c = cvt_block(b, cb)
        if x < 4:
            put(0, c)
        else:
            put(4 * x - 1, c[0])
            put(4 * x, c[1])
        if diag and b == cb:
            for i in range(4):
                xr = S(b, cb, i)
                put(min(4 * x + 8, n), [valu(f"v_cmp_le_i32 vcc, {i}, %[vt]", r=["%[vt]"]),
                                        valu(f"v_cndmask_b32 {xr}, {VNINF}, {xr}, vcc", r=[VNINF, xr], w=[xr])])
        if with_max and x >= 2:
            by, cby = chains[x - 2]
            mm = max_block(by, cby, first=(cby == 0 and by in (0, 2)))
            put(4 * x + 1, mm[0])
            put(4 * x + 2, mm[1])
    leftover = []
    # V(j+1) by LDS-DMA into the other image (its last reads were PV(j-1)'s)
    pos = 2
    for m0w, ld, *adv in (v_dma(SOTH) if "nodma" not in XP else []):  # (nodma, noload: timing only)
        put(pos, m0w)
        put(pos + 1, [ld] + (adv[0] if adv else []))
        pos += 2
    # K(j+2), key block by key block, >= 4 MFMAs after the last chain reading it
    for cb in (range(4) if "noload" not in XP else []):
        for i, ld in enumerate(k_loads(cb) + (k_advance() if cb == 3 else [])):
            k = max(pos, last_of_cb[cb] + 4)
            if k < n - 2:
                put(k, ld)
                pos = k + 1
            else:
                leftover.append(ld)
    # the first V^T fragments of PV(j) (V(j) landed: DMA'd in the previous iteration)
    if V_AHEAD:
        put(n - 12 - 3 * (V_AHEAD - 3) - 1, vmwait(("V", "prev")))
    for f in range(V_AHEAD):
        for i, r in enumerate(vtr_reads(0, f, f)):
            put(n - 12 - 3 * (V_AHEAD - 3) + 3 * f + i, r)
    assert max(gaps) <= n
    st.interleave(mf, gaps)
    lv = []
    if with_max:
        for y in (len(chains) - 2, len(chains) - 1):
            by, cby = chains[y]
            lv += max_block(by, cby, first=False)
    return lv, leftover


def phase_b(st, lv, leftover, dec_gap, label_slow, label_end, exps=True):
    """PV(j) from the current image; the decision at dec_gap; exp2 of S(j+1)"""
    mf, frag_first = pv_mfmas()
    gaps = {}

    def put(k, ins):
        gaps.setdefault(k, []).extend(ins if isinstance(ins, list) else [ins])

    if not V_AHEAD:
        put(0, vmwait(("V", "prev")))
    for f in range(V_AHEAD, 16):
        k = frag_first[f - V_AHEAD] if f >= V_AHEAD and V_AHEAD else 0
        u, e = divmod(f, 8)
        r = vtr_reads(u, e, f % 8)
        put(k + 1 if V_AHEAD else 2 * f, r[0])
        put(k + 2 if V_AHEAD else 2 * f + 1, r[1])
    for i, ins in enumerate(lv):
        put(1 + i, ins)
    for i, ins in enumerate(leftover):
        put(1 + i, ins)
    dec = [valu(f"v_max_f32 {T[0]}, {RMAX[0]}, {RMAX[1]}", r=[RMAX[0], RMAX[1]], w=[T[0]]),
           valu(f"v_cmp_lt_f32 vcc, 0x41000000, {T[0]}", r=[T[0]])]
    if exps:
        ex = exp_ops()
        n_g = len(mf) - dec_gap
        for i, e in enumerate(ex):
            put(dec_gap + 1 + (i * n_g) // len(ex), e)
    for k in range(dec_gap):
        for f in gaps.get(k, []):
            st.emit(f)
        st.emit(mf[k])
    for f in gaps.get(dec_gap, []):
        st.emit(f)
    if exps:
        for d in dec:
            st.emit(d)
        st.branch("s_cbranch_vccnz", label_slow)
    for k in range(dec_gap, len(mf)):
        if k > dec_gap:
            for f in gaps.get(k, []):
                st.emit(f)
        st.emit(mf[k])
    for f in gaps.get(len(mf), []):
        st.emit(f)
    if not exps:
        return
    st.branch("s_branch", label_end)
    st.label(label_slow)
    for k in range(dec_gap, len(mf)):
        if k > dec_gap:
            for f in gaps.get(k, []):
                if isinstance(f, str) or f.kind != "trans":
                    st.emit(f)
        st.emit(mf[k])
    for f in gaps.get(len(mf), []):
        if isinstance(f, str) or f.kind != "trans":
            st.emit(f)
    slow_softmax(st, first=False)
    for e in exp_ops():
        st.emit(e)
    st.branch("s_branch", label_end)


def pv_plain(st):
    """the drain's PV(j): V^T reads two fragments ahead"""
    mf, frag_first = pv_mfmas()
    gaps = {0: [vmwait(("V", "prev"))]}
    for f in range(16):
        u, e = divmod(f, 8)
        k = frag_first[f - 2] + 1 if f >= 2 else 0
        for i, r in enumerate(vtr_reads(u, e, f % 8)):
            gaps.setdefault(k + i if f >= 2 else 0, []).append(r)
    st.interleave(mf, gaps)


def q_scale(st):
    """Q * c rounded to fp16 once (W4's q_scale), staged in the V^T slots"""
    for x0 in range(0, 64, 8):
        xs = range(x0, x0 + 8)
        lo = {x: f"v{176 + 3 * (x - x0)}" for x in xs}
        hi = {x: f"v{177 + 3 * (x - x0)}" for x in xs}
        pk = {x: f"v{178 + 3 * (x - x0)}" for x in xs}
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
    """Q, K(0) and V(0) (LDS-DMA) in flight; S(0) with K(1) behind its chains;
    the first tile's softmax"""
    kstamp(st, 0)
    st.raw(f"s_mov_b32 {SM0}, m0")
    # the segment's record (fa_w4k_kernel.hpp W4kSeg, 32 dwords in LDS):
    # 0-3 K, 4-7 V, 8-11 Q descriptors, 12 n, 13 maskj, 14 kvhi, 15 qm,
    # 16 V image pair, 17 partial slot, 18 log2-sum-exp row
    st.raw("v_mov_b32 v16, %[tab]")
    for i in range(5):
        st.raw(f"ds_read_b128 v[{4 * i}:{4 * i + 3}], v16 offset:{16 * i}")
    st.raw("s_waitcnt lgkmcnt(0)")
    for i in range(12):
        st.raw(f"v_readfirstlane_b32 s{40 + i if i < 8 else 72 + i - 8}, v{i}")
    for sreg, i in ((SN, 12), (SMASKJ, 13), (SKVHI, 14), (SQM, 15), (SIMG, 16), (SPSLOT, 17), (SLSLOT, 18)):
        st.raw(f"v_readfirstlane_b32 {sreg}, v{i}")
    for i, v in enumerate((0, 0x1000, 0x2000, 0x3000)):
        st.raw(f"s_mov_b32 {SOFF[i]}, {v}")
    st.raw(f"s_mov_b32 {SKREM}, s42")
    st.raw(f"s_mov_b32 {SVREM}, s46")
    st.raw(f"s_add_u32 {SOTH}, {SIMG}, 0x4000")
    st.raw(f"s_mov_b32 {SDELTA}, 0x4000")
    st.raw(f"v_mov_b32 {VA[0]}, %[va0]")
    st.raw(f"v_mov_b32 {VA[1]}, %[va1]")
    # DMA source offsets: piece i of a 4-KiB group = vd0 + 2048 (i >> 1) + 128 (i & 1),
    # chunk bit 1 flipped for i >= 2 (the image's swizzle, as W4's dma_setup)
    st.raw(f"v_mov_b32 {VD[0]}, %[vd0]")
    for i in range(1, 4):
        st.raw(f"v_add_u32 {VD[i]}, {2048 * (i >> 1) + 128 * (i & 1)}, %[vd0]")
        if i >= 2:
            st.raw(f"v_xor_b32 {VD[i]}, 32, {VD[i]}")
    st.raw(f"v_mov_b32 {VNINF}, {NINF}")
    for i in range(4):
        st.raw(f"v_mov_b32 v{208 + i}, {DT['one2']}")
    st.nop(4)
    # Q rows 16 b + r16 -> v[16 b + 4 t]
    for b in range(4):
        for t in range(4):
            st.emit(tagged(vmem(f"buffer_load_dwordx4 {R('v', 16 * b + 4 * t, 4)}, %[qoff], {RQ}, {SOFF[b]} offen offset:{64 * t}",
                                r=["%[qoff]"], w=[R('v', 16 * b + 4 * t, 4)]), ("Q",)))
    for cb in range(4):
        for ld in k_loads(cb):
            st.emit(ld)
    for ins in k_advance():
        st.emit(ins)
    for m0w, ld, *adv in v_dma(SIMG):
        st.emit(m0w)
        st.nop(1)
        st.emit(ld)
        for a in (adv[0] if adv else []):
            st.emit(a)
    # O, l, -m_ref, m_ref = 0
    for x in range(144):
        st.raw(f"v_accvgpr_write_b32 a{x}, 0")
    for x in range(96, 112):
        st.raw(f"v_mov_b32 v{x}, 0")
    for b in range(4):
        st.raw(f"v_mov_b32 {MREF[b]}, 0")
    st.wait_vm(tags=[("Q",)])
    q_scale(st)
    st.nop(3)
    # S(0); K(1) loads behind each key block's chains
    mf, last = [], {}
    for cb in range(4):
        for b in range(4):
            mf += qk_chain(b, cb)
        last[cb] = len(mf) - 1
    gaps = {}
    for cb in range(3):
        for t, ld in enumerate(k_loads(cb)):
            gaps.setdefault(last[cb] + 4 + t, []).append(ld)
    st.interleave(mf, gaps)
    st.nop(2)
    for ld in k_loads(3) + k_advance():
        st.emit(ld)
    # the segment's only tile is its last: mask it
    skip = newlabel("k_nomask0")
    st.raw(f"s_cmp_eq_u32 {SMASKJ}, 1")
    st.branch("s_cbranch_scc0", skip)
    st.raw(f"s_sub_i32 {ST0}, {SKVHI}, 1")
    st.raw(f"s_mov_b32 {ST1}, {SQM}")
    mask_last_tile(st, causal)
    st.label(skip)
    slow_softmax(st, first=True)
    for e in exp_ops():
        st.emit(e)
    st.raw(f"s_mov_b32 {SJ}, 0")
    kstamp(st, 1)


def epilogue(st):
    """normalised O (fp16) and m_ref + log2 l per row into the LDS partial
    slot: row 16 b + r16 at %[pslot] + 256 row, 16-B chunk c at (c ^ r16)
    (conflict-free writes); log2-sum-exp at %[lslot] + 4 row"""
    st.vm_all()
    st.lgkm_all()
    LA = "v13"
    E = st.emit
    E(valu(f"v_lshlrev_b32 {LA}, 2, %[r16]", r=["%[r16]"], w=[LA]))
    E(valu(f"v_add_u32 {LA}, {SLSLOT}, {LA}", r=[LA], w=[LA]))
    for b in range(4):
        l, inv = T[0], T[1]
        E(valu(f"v_accvgpr_read_b32 {l}, {L(b, 0)}", r=[L(b, 0)], w=[l]))
        E(valu(f"v_div_scale_f32 {T[2]}, s[58:59], {l}, {l}, 1.0", r=[l], w=[T[2]]))
        E(valu(f"v_rcp_f32_e32 {T[3]}, {T[2]}", r=[T[2]], w=[T[3]], kind="trans"))
        E(valu(f"v_fma_f32 {T[4]}, -{T[2]}, {T[3]}, 1.0", r=[T[2], T[3]], w=[T[4]]))
        E(valu(f"v_fmac_f32_e32 {T[3]}, {T[4]}, {T[3]}", r=[T[3], T[4]], w=[T[3]]))
        E(valu(f"v_div_scale_f32 {T[4]}, vcc, 1.0, {l}, 1.0", r=[l], w=[T[4]]))
        E(valu(f"v_mul_f32_e32 {T[5]}, {T[4]}, {T[3]}", r=[T[4], T[3]], w=[T[5]]))
        E(valu(f"v_fma_f32 {T[6]}, -{T[2]}, {T[5]}, {T[4]}", r=[T[2], T[5], T[4]], w=[T[6]]))
        E(valu(f"v_fmac_f32_e32 {T[5]}, {T[6]}, {T[3]}", r=[T[5], T[6], T[3]], w=[T[5]]))
        E(valu(f"v_fma_f32 {T[2]}, -{T[2]}, {T[5]}, {T[4]}", r=[T[2], T[5], T[4]], w=[T[2]]))
        E(valu(f"v_div_fmas_f32 {T[2]}, {T[2]}, {T[3]}, {T[5]}", r=[T[2], T[3], T[5]], w=[T[2]]))
        E(valu(f"v_div_fixup_f32 {T[2]}, {T[2]}, {l}, 1.0", r=[T[2], l], w=[T[2]]))
        E(valu(f"v_cmp_lt_f32 vcc, 0, {l}", r=[l]))
        E(valu(f"v_cndmask_b32 {inv}, 0, {T[2]}, vcc", r=[T[2]], w=[inv]))
        # log2-sum-exp of row 16 b + r16 (-inf for an empty row)
        E(valu(f"v_log_f32_e32 {T[8]}, {l}", r=[l], w=[T[8]], kind="trans"))
        E(valu(f"v_add_f32_e32 {T[8]}, {MREF[b]}, {T[8]}", r=[MREF[b], T[8]], w=[T[8]]))
        E(dsw(f"ds_write_b32 {LA}, {T[8]} offset:{64 * b}", LA, T[8]))
        for ep in range(4):
            # two register sets, alternating, so one write's operands are not
            # overwritten by the next conversion
            r0 = 16 * (ep & 1)
            d = [f"v{r0 + i}" for i in range(8)]
            X, Y = [f"v{r0 + 8}", f"v{r0 + 9}"], [f"v{r0 + 10}", f"v{r0 + 11}"]
            AD = f"v{r0 + 12}"
            for x in range(2):
                e = 2 * ep + x
                for i in range(4):
                    E(valu(f"v_accvgpr_read_b32 {d[4 * x + i]}, {O(b, e, i)}", r=[O(b, e, i)], w=[d[4 * x + i]]))
                for i in range(4):
                    E(valu(f"v_mul_f32_e32 {d[4 * x + i]}, {d[4 * x + i]}, {inv}", r=[d[4 * x + i], inv],
                           w=[d[4 * x + i]]))
            E(valu(f"{DT['cvt_pk']} {X[0]}, {d[0]}, {d[1]}", r=d[0:2], w=[X[0]]))
            E(valu(f"{DT['cvt_pk']} {X[1]}, {d[2]}, {d[3]}", r=d[2:4], w=[X[1]]))
            E(valu(f"{DT['cvt_pk']} {Y[0]}, {d[4]}, {d[5]}", r=d[4:6], w=[Y[0]]))
            E(valu(f"{DT['cvt_pk']} {Y[1]}, {d[6]}, {d[7]}", r=d[6:8], w=[Y[1]]))
            for dw in range(2):
                E(valu(f"v_permlane16_swap_b32 {X[dw]}, {Y[dw]}", r=[X[dw], Y[dw]], w=[X[dw], Y[dw]]))
            E(valu(f"v_add_u32 {AD}, {SPSLOT}, %[pl{ep}]", r=[f"%[pl{ep}]"], w=[AD]))
            E(dsw(f"ds_write_b128 {AD}, v[{r0 + 8}:{r0 + 11}] offset:{4096 * b}", AD, f"v[{r0 + 8}:{r0 + 11}]"))
    st.lgkm_all()
    kstamp(st, 3)
    if DIAG == "stamps":
        st.raw(f"v_mov_b32 v0, {SLSLOT}")
        for i in range(4):
            st.raw(f"v_mov_b32 v{2 + 2 * i}, s{76 + 2 * i}")
            st.raw(f"v_mov_b32 v{3 + 2 * i}, s{77 + 2 * i}")
        st.raw("ds_write_b128 v0, v[2:5]")
        st.raw("ds_write_b128 v0, v[6:9] offset:16")
        st.raw("s_waitcnt lgkmcnt(0)")
    st.raw(f"s_mov_b32 m0, {SM0}")


def generate(causal):
    st = VStream()
    lab = {k: newlabel("k" + k) for k in ("loop", "drain", "masked", "general", "slow", "slow2", "slow3",
                                          "end", "done")}
    prologue(st, causal)
    # loop head invariant: outstanding = V(j)'s DMA, then K(j+1)'s loads
    st.label(lab["loop"], drain_lgkm=True)
    st.retag(("V", "cur"), ("V", "prev"))
    entry_vm = [t for _, t, _ in st.vm]
    st.raw(f"s_add_u32 {SJ1}, {SJ}, 1")
    st.raw(f"s_cmp_lt_u32 {SJ1}, {SN}")
    st.branch("s_cbranch_scc0", lab["drain"])
    st.raw(f"s_add_u32 {ST0}, {SJ}, 2")
    st.raw(f"s_cmp_eq_u32 {ST0}, {SMASKJ}")
    st.branch("s_cbranch_scc1", lab["masked"])
    lv, left = phase_a(st, with_max=True)
    phase_b(st, lv, left, dec_gap=6, label_slow=lab["slow"], label_end=lab["end"])
    # ---- masked: the segment's last tile (causal diagonal / ragged end) ----
    st.label(lab["masked"])
    st.raw(f"s_lshl_b32 {ST1}, {SJ1}, 6")
    st.raw(f"s_sub_i32 {ST0}, {SKVHI}, {ST1}")
    st.raw(f"s_sub_i32 {ST0}, {ST0}, 1")
    st.raw(f"s_sub_i32 {ST1}, {SQM}, {ST1}")
    if causal:
        st.raw(f"s_cmp_eq_u32 {ST1}, 0")
        st.branch("s_cbranch_scc0", lab["general"])
        st.raw(f"s_cmp_ge_i32 {ST0}, 63")
        st.branch("s_cbranch_scc0", lab["general"])
        lv, left = phase_a(st, with_max=True, diag=True)
        phase_b(st, lv, left, dec_gap=6, label_slow=lab["slow3"], label_end=lab["end"])
        st.label(lab["general"])
    lv, left = phase_a(st, with_max=False)
    mask_last_tile(st, causal)
    full_max(st)
    phase_b(st, [], left, dec_gap=0, label_slow=lab["slow2"], label_end=lab["end"])
    st.label(lab["end"], drain_lgkm=True)
    # next iteration reads the other image
    st.raw(f"v_add_u32 {VA[0]}, {SDELTA}, {VA[0]}")
    st.raw(f"v_add_u32 {VA[1]}, {SDELTA}, {VA[1]}")
    st.raw(f"s_add_u32 {SIMG}, {SIMG}, {SDELTA}")
    st.raw(f"s_sub_u32 {SOTH}, {SOTH}, {SDELTA}")
    st.raw(f"s_sub_i32 {SDELTA}, 0, {SDELTA}")
    st.raw(f"s_add_u32 {SJ}, {SJ}, 1")
    st.raw(f"s_branch {lab['loop']}")
    assert XP or [t for _, t, _ in st.vm] == [(("V", "cur") if t == ("V", "prev") else t) for t in entry_vm] or \
        [t for _, t, _ in st.vm][:16] == [("V", "cur")] * 16, "loop-carried vmem state"
    st.dead = True
    # ---- drain: PV(n-1) only ----
    st.label(lab["drain"], drain_lgkm=True)
    kstamp(st, 2)
    for b in range(4):
        for cb in range(4):
            for c in cvt_block(b, cb):
                st.emit(c)
    pv_plain(st)
    epilogue(st)
    return st.out


HEADER = """// GENERATED by gen_w4k_item.py -- do not edit.
// One segment (64 query rows x a run of key tiles) of the short-launch tier:
// see the generator's docstring for the register map and the schedule.
#pragma once
"""


def cxx(causal, bf16, lines):
    body = "\n".join(f'      "{l}\\n"' for l in lines)
    vclob = ", ".join(f'"v{i}"' for i in range(224 + 12))
    aclob = ", ".join(f'"a{i}"' for i in range(208))
    sclob = ", ".join(f'"s{i}"' for i in range(40, 84 if DIAG else 76))
    name = ("w4k_seg_causal" if causal else "w4k_seg_noncausal") + ("_bf16" if bf16 else "_f16")
    return f"""
__device__ __forceinline__ void {name}(unsigned tab, float c, const W4kLane& ln) {{
  asm volatile(
{body}
      :
      : [tab] "s"(tab), [c] "s"(c),
        [kg] "v"(ln.kg), [vd0] "v"(ln.vd0), [va0] "v"(ln.va[0]), [va1] "v"(ln.va[1]),
        [vt] "v"(ln.vt), [r16] "v"(ln.r16), [qoff] "v"(ln.qoff),
        [pl0] "v"(ln.pl[0]), [pl1] "v"(ln.pl[1]), [pl2] "v"(ln.pl[2]), [pl3] "v"(ln.pl[3])
      : "memory", "vcc", "scc", {sclob},
        {vclob},
        {aclob});
}}
"""


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "fa_w4k_item.inc"
    text = HEADER
    for bf16 in (False, True):
        g.set_dtype(bf16)
        for causal in (False, True):
            g._lbl[0] = 0
            text += cxx(causal, bf16, generate(causal))
    with open(out, "w") as f:
        f.write(text)


if __name__ == "__main__":
    main()
