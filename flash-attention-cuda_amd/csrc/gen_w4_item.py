#!/usr/bin/env python3
"""Generator of the one-wave-per-SIMD attention item program (fa_w4_item.inc).

The W4 kernel (fa_w4_kernel.hpp) runs 4 waves x 64 query rows on one CU, each
wave owning the whole 512-entry register file.  hipcc cannot hold that
layout (it routes the score tile through AGPRs and spills), so
one query block ("item") of the persistent kernel is a single inline-asm
statement whose registers are fixed here:

  VGPR  v0-63    S^T tile, 4 row blocks b x 4 key blocks cb x 4  (fp32 scores,
                 then exp2'd in place)
        v64-95   P, fp16, B operands of PV  (b, u) x 4
        v96-111  -m_ref broadcast per row block (C operand of QK^T chains)
        v112-143 K fragments (8 slots)      v144-175 V^T fragments (8 slots)
        v176-183 per-pass LDS-DMA source offsets of the K/V staging
        v208-235 constants, m_ref, running maxima, temporaries
  AGPR  a0-127   O^T accumulator (b, e) x 4    a128-143 row sums l (b)
        a144-207 Q (pre-scaled by log2(e)/sqrt(d)), B operands of QK^T
        a208-239 the next item's K(1) / V(0), loaded into registers during
                 the previous item's last iteration (prologue only)
  the compiler keeps v236-v255 for the lane constants passed in.

Per key tile j (after the prologue computed S(0)) every wave runs
  phase A: QK^T(j+1) -- 64 MFMAs in 16 four-deep chains; beside them the fp16
           conversion of P(j) (each block just before the chain that
           overwrites its registers), the running row maxima of S(j+1), the
           K reads, and the stage traffic (LDS-DMA of K(j+2) / V(j+1) straight
           into the LDS images the previous iteration finished reading)
  phase B: PV(j) + row sums -- 72 MFMAs; beside them the rescale decision
           (wave-uniform branch, rare slow path) and exp2 of S(j+1), one v_exp
           per MFMA gap, and the V^T transposed reads
  s_waitcnt vmcnt(0) (this iteration's DMA landed), one barrier.
The arithmetic is the M16 policy's (fa_fwd_kernel.hpp) operation for
operation, per 32-row half (the rescale decision is taken per half, as the
8-wave ping-pong's 32-row waves take it), so results match the ping-pong
kernel up to the final fp32 -> fp16 rounding of O.

Hazards are not padded by the assembler: `Stream` tracks, per register, the
last MFMA and VALU writes in wait states and inserts s_nop where a reader is
too close; LDS reads are waited for with counted lgkmcnt at their first use.

usage: python3 gen_w4_item.py [OUT.inc]      (the Makefile runs it)
"""
import os
import sys

# diagnostic builds only (never the product library): W4_DIAG=raw (store O
# unnormalised), l (store the row sums l in every column), haz (double every
# hazard window)
DIAG = os.environ.get("W4_DIAG", "")
# timing-only experiment switches for diagnostic builds (wrong results):
# nostage (no K/V staging in phase A), nomax (no running maxima), tmajor
# (QK^T chains interleaved t-major within a key block)
XP = set(os.environ.get("W4_XP", "").split(",")) - {""}

# Wait states = instructions issued BETWEEN producer and consumer (s_nop N
# counts N+1), as LLVM's hazard recognizer counts them.  Required after a
# 16x16x32 MFMA writes a register before a VALU / memory instruction reads or
# writes it:  gfx950 needs
# NumPasses + 4; the 16x16x32 f16 form is taken as 8-pass (12), the larger of
# the two plausible pass counts.
MFMA_TO_VALU = 12
VALU_TO_MFMA = 3      # VALU / accvgpr write -> MFMA operand read (needs 2)
VALU_TO_PERMLANE = 2  # VALU write -> v_permlane*_swap read
TRANS_TO_VALU = 1     # transcendental (v_exp / v_rcp) write -> non-trans VALU read (gfx940+)
if DIAG == "haz":
    MFMA_TO_VALU, VALU_TO_MFMA, VALU_TO_PERMLANE, TRANS_TO_VALU = 24, 6, 4, 2

NINF = "0xff800000"

# element type of Q/K/V/O and the MFMA operands (set per generated function):
# fp16 (the reference's type) or bf16 -- only the MFMA opcode, the fp32 <->
# 16-bit conversions and the 1.0 constant differ
DT = {"mfma": "v_mfma_f32_16x16x32_f16", "cvt_pk": "v_cvt_pk_f16_f32", "one2": "0x3c003c00"}


def set_dtype(bf16):
    DT.update({"mfma": "v_mfma_f32_16x16x32_bf16", "cvt_pk": "v_cvt_pk_bf16_f32", "one2": "0x3f803f80"}
              if bf16 else {"mfma": "v_mfma_f32_16x16x32_f16", "cvt_pk": "v_cvt_pk_f16_f32",
                            "one2": "0x3c003c00"})
    DT["bf16"] = bf16
# V^T fragments read this many fragments ahead of their PV MFMAs (4 or 5:
# level within noise at both head_dims, profiles/r04_ab_w4_wait_coalescing*)
V_AHEAD = int(os.environ.get("W4_V_AHEAD", "3"))
# counted-wait coalescing: a wait for one LDS read also retires the younger
# reads issued at least WAGE wait states earlier (0: wait for the needed read
# only), so their own first uses need no wait of their own -- half the
# s_waitcnt of a tile, +0.8-1.3 % (profiles/r04_ab_w4_wait_coalescing*.jsonl;
# stamps: tile 2929 -> 2878 cycles, r04_w4_stamps_wait_coalescing.txt)
WAGE = int(os.environ.get("W4_WAGE", "8"))

# head_dim of the generated function (set_hd): 128, the reference's, or 64.
# Q/K/V/O rows are 2*hd bytes in HBM and in the (packed) LDS tile images:
# 16 KiB per 64-key tile at 128, 8 KiB at 64 (fa_w4_kernel.hpp k_off64/v_off64)
HDC = {"hd": 128}


def set_hd(hd):
    HDC["hd"] = hd


def NT():     # k-steps of a QK^T chain = Q fragments per row block
    return HDC["hd"] // 32


def NE():     # 16-column O^T blocks per row block
    return HDC["hd"] // 16


def ROWB():   # bytes of a Q/K/V/O row
    return 2 * HDC["hd"]


def ROWSH():
    return 8 if HDC["hd"] == 128 else 7


def TILEB():  # bytes of a 64-key K or V tile
    return 64 * ROWB()


def NPASS():  # 4-KiB register-staging passes per tile and tensor (256 lanes x 16 B)
    return HDC["hd"] // 32


def PASSL():  # LDS stride of a 4-KiB staging pass (the images are packed: 4 KiB)
    return 4096
# causal diagonal tile masked block by block inside phase A (W4_DIAG_FAST=0:
# the general mask after phase A, for A/B)
DIAG_FAST = os.environ.get("W4_DIAG_FAST", "1") == "1"
# next item's loads issued before (1) or after (0) the last iteration's PV drain
PF_BEFORE_DRAIN = os.environ.get("W4_PF_BEFORE", "0") == "1"  # V^T fragments read ahead of the PV MFMAs that use them
# cross-item overlap (non-split programs): an item with a successor defers
# its epilogue (O read-out, 1/l scaling, fp16 conversion, stores) into the
# successor's prologue, beside the S(0) QK^T MFMAs, which touch no O
# register; its O descriptor and row base wait in s[60:63] / s64
XOVL = os.environ.get("W4_XOVL", "1") == "1" and DIAG not in ("stamps", "pstamps")  # (s60-s69: stamps)
ROSAVE, ROWSAVE = "s[60:63]", "s64"
# the deferred epilogue zeroes O / l with 32x32x16 MFMAs of zero operands
# instead of v_accvgpr_write: at head_dim 64 (+0.3-2.5 %); at 128 the writes
# stay (the MFMAs measured -0.1-0.2 %, profiles/r04_ab_w4_mfma_zeroing*.jsonl)
MFZ_XP = "nomfz" not in XP


def mfz():
    return MFZ_XP and HDC["hd"] == 64
# cache policy of the (non-split) O stores; the split tier's slab stores stay
# sc1 (read by other workgroups)
OPOL = " ".join([""] + os.environ.get("W4_OPOL", "sc1").split("+"))  # e.g. W4_OPOL=nt, sc1+nt, ""


def regs(spec):
    """'v12' / 'v[4:7]' / 'a[0:3]' -> ['v4','v5','v6','v7']; '%[name]' operands as is"""
    if spec.startswith("%") or spec.startswith("s"):
        return [spec]
    if "[" in spec:
        kind = spec[0]
        lo, hi = spec[2:-1].split(":")
        return [f"{kind}{i}" for i in range(int(lo), int(hi) + 1)]
    return [spec]


def R(kind, i, n=1):
    return f"{kind}{i}" if n == 1 else f"{kind}[{i}:{i + n - 1}]"


class Ins:
    """one instruction: text, kind, registers read / written"""

    def __init__(self, text, kind, r=(), w=(), lgkm_dst=False):
        self.text, self.kind = text, kind
        self.r = [x for s in r for x in regs(s)]
        self.w = [x for s in w for x in regs(s)]
        self.lgkm_dst = lgkm_dst


def mfma(d, a, b, c):
    return Ins(f"{DT['mfma']} {d}, {a}, {b}, {c}", "mfma", r=[a, b, c] if c[0] in "va" else [a, b], w=[d])


def valu(text, r=(), w=(), kind="valu"):
    return Ins(text, kind, r=r, w=w)


def dsr(text, dst, addr):
    return Ins(text, "dsr", r=[addr], w=[dst], lgkm_dst=True)


def dsw(text, addr, data):
    return Ins(text, "dsw", r=[addr, data])


def vmem(text, r=(), w=()):
    return Ins(text, "vmem", r=r, w=w)


def salu(text):
    return Ins(text, "salu")


class Stream:
    """Linear instruction stream with wait-state and lgkmcnt bookkeeping.

    pos counts wait states (one per instruction, N+1 per s_nop N).  State is
    forked at branches and merged (most conservative) at labels."""

    def __init__(self):
        self.out = []
        self.pos = 0
        self.mfma_w = {}   # reg -> pos of the last MFMA write
        self.valu_w = {}   # reg -> pos of the last VALU write
        self.trans_w = {}  # reg -> pos of the last transcendental write
        self.lgkm = []     # outstanding LDS ops, oldest first: (set of dst regs or None, pos)
        self.pending = {}  # label -> list of saved states
        self.dead = False  # after an unconditional branch

    # -- state for branches ----------------------------------------------
    def _snap(self):
        return ({r: self.pos - p for r, p in self.mfma_w.items()},
                {r: self.pos - p for r, p in self.valu_w.items()},
                [x for x in self.lgkm],
                {r: self.pos - p for r, p in self.trans_w.items()})

    def _restore(self, snaps):
        m, v, lg, tr = {}, {}, None, {}
        for sm, sv, sl, st_ in snaps:
            for r, d in sm.items():
                m[r] = min(m.get(r, 10 ** 9), d)
            for r, d in sv.items():
                v[r] = min(v.get(r, 10 ** 9), d)
            for r, d in st_.items():
                tr[r] = min(tr.get(r, 10 ** 9), d)
            if lg is None or len(sl) > len(lg):
                lg = sl
        self.mfma_w = {r: self.pos - d for r, d in m.items() if d < 64}
        self.valu_w = {r: self.pos - d for r, d in v.items() if d < 64}
        self.trans_w = {r: self.pos - d for r, d in tr.items() if d < 64}
        # merged paths may differ in LDS ops in flight: keep the longer list;
        # counted waits stay safe (they only ever wait for more than needed)
        # as long as every path's list is a suffix-compatible prefix -- assert
        self.lgkm = lg or []

    def branch(self, cond, label):
        self.raw(f"{cond} {label}")
        self.pending.setdefault(label, []).append(self._snap())
        if cond == "s_branch":
            self.dead = True

    def label(self, name, drain_lgkm=False):
        snaps = self.pending.pop(name, [])
        if not self.dead:
            snaps = snaps + [self._snap()]
        self.out.append(f"{name}:")
        self._restore(snaps)
        self.dead = False
        if drain_lgkm and self.lgkm:
            self.raw("s_waitcnt lgkmcnt(0)")
            self.lgkm = []

    # -- emission ---------------------------------------------------------
    def raw(self, text, ws=1):
        self.out.append(text)
        self.pos += ws

    def nop(self, n):
        while n > 0:
            k = min(n, 8)
            self.raw(f"s_nop {k - 1}", ws=k)
            n -= k

    def wait_lgkm_for(self, regs_needed):
        """counted lgkmcnt so every outstanding LDS read writing a needed reg is done"""
        need = set(regs_needed)
        last = -1
        for i, (op, _) in enumerate(self.lgkm):
            if op is not None and op & need:
                last = i
        if last < 0:
            return
        after = len(self.lgkm) - 1 - last
        if WAGE:
            after = sum(1 for _, at in self.lgkm[last + 1:] if at > self.pos - WAGE)
        self.raw(f"s_waitcnt lgkmcnt({min(after, 15)})")
        keep = min(after, 15)
        self.lgkm = self.lgkm[len(self.lgkm) - keep:]

    def lgkm_all(self):
        if self.lgkm:
            self.raw("s_waitcnt lgkmcnt(0)")
            self.lgkm = []

    def emit(self, ins):
        if isinstance(ins, str):
            self.raw(ins)
            return
        k = ins.kind
        touched = ins.r + ins.w
        # LDS read results must have landed before any use (or overwrite)
        self.wait_lgkm_for(touched)
        need = 0
        if k == "mfma":
            for r in ins.r:
                if r in self.valu_w:
                    need = max(need, VALU_TO_MFMA - (self.pos - self.valu_w[r] - 1))
            # an MFMA reading another MFMA's result as A/B (not used here) or
            # as C of the same chain (hardware-forwarded) needs nothing
        else:
            for r in touched:
                if r in self.mfma_w:
                    need = max(need, MFMA_TO_VALU - (self.pos - self.mfma_w[r] - 1))
            if k != "trans":
                for r in ins.r:
                    if r in self.trans_w:
                        need = max(need, TRANS_TO_VALU - (self.pos - self.trans_w[r] - 1))
            if "permlane" in ins.text:
                for r in ins.r:
                    if r in self.valu_w:
                        need = max(need, VALU_TO_PERMLANE - (self.pos - self.valu_w[r] - 1))
        if need > 0:
            self.nop(need)
        self.raw(ins.text)
        at = self.pos - 1
        for r in ins.w:
            if k == "mfma":
                self.mfma_w[r] = at
                self.valu_w.pop(r, None)
            elif k in ("valu", "trans"):
                self.valu_w[r] = at
                self.mfma_w.pop(r, None)
                if k == "trans":
                    self.trans_w[r] = at
                else:
                    self.trans_w.pop(r, None)
            else:
                self.mfma_w.pop(r, None)
                self.valu_w.pop(r, None)
        if k in ("dsr", "dsw"):
            self.lgkm.append((set(ins.w) if ins.lgkm_dst else None, self.pos - 1))

    def far(self, cond, label):
        """branch whose target may lie past the +-128 KiB of a SOPP branch
        (the dbl programs): an inverted short branch over s_getpc_b64 +
        pc-relative add + s_setpc_b64 (LLVM's own branch relaxation sequence;
        s[58:59] are free in the key loop and at item boundaries)"""
        inv = {"s_cbranch_scc0": "s_cbranch_scc1", "s_cbranch_scc1": "s_cbranch_scc0"}
        skip = None
        if cond != "s_branch":
            skip = newlabel("nofar")
            self.raw(f"{inv[cond]} {skip}")
        post = newlabel("pc")
        self.raw("s_getpc_b64 s[58:59]")
        self.out.append(f"{post}:")
        self.raw(f"s_add_u32 s58, s58, ({label}-{post})&4294967295")
        self.raw(f"s_addc_u32 s59, s59, ({label}-{post})>>32")
        self.raw("s_setpc_b64 s[58:59]")
        self.pending.setdefault(label, []).append(self._snap())
        if skip is None:
            self.dead = True
        else:
            self.label(skip)

    def jump(self, cond, label):
        """a loop-control branch: far in the dbl programs"""
        if dbl():
            self.far(cond, label)
        else:
            self.branch(cond, label)

    def interleave(self, mfmas, gaps):
        """gaps[k] = fillers issued before mfmas[k]; gaps[len(mfmas)] after the last"""
        for k, m in enumerate(mfmas):
            for f in gaps.get(k, []):
                self.emit(f)
            self.emit(m)
        for f in gaps.get(len(mfmas), []):
            self.emit(f)


# ---------------------------------------------------------------------------
# register map
# ---------------------------------------------------------------------------
def S(b, cb, i=None):
    base = 16 * b + 4 * cb
    return R("v", base, 4) if i is None else R("v", base + i)


def P(b, u, r=None):
    base = 64 + 8 * b + 4 * u
    return R("v", base, 4) if r is None else R("v", base + r)


def NEGM(b, i=None):
    return R("v", 96 + 4 * b, 4) if i is None else R("v", 96 + 4 * b + i)


def KF(slot):
    return R("v", 112 + 4 * slot, 4)


def VF(slot, half=None):
    base = 144 + 4 * slot if slot < 8 else 184 + 4 * (slot - 8)
    return R("v", base, 4) if half is None else R("v", base + 2 * half, 2)


def v14():
    """14 V^T fragment slots (the DMA build's free v184-v207 as slots 8-13):
    all of PV(j)'s first-half fragments are read at the end of phase A, after
    the last K reads, and six of the second half at the start of phase B,
    before its exp2 stream (W4_XP=v14)"""
    return "v14" in XP and dma()


def vslot(f):
    if v14():
        return f if f < 14 else f - 14
    return f % 8


def vahead():
    return 8 if v14() else V_AHEAD


def KST(i):
    return R("v", 176 + 4 * i, 4)


def VST(i):
    return R("v", 192 + 4 * i, 4)


ONES = R("v", 208, 4)
MREF = [R("v", 212 + b) for b in range(4)]
RMAX = [R("v", 216), R("v", 217)]          # running partial maxima, half 0 / 1
KOFF = ["%[koff]"] + [R("v", 218 + i) for i in range(3)]  # staging global offsets, passes 0..3
VOFF = ["%[voff]"] + [R("v", 221 + i) for i in range(3)]
VNINF = R("v", 224)
T = [R("v", 225 + i) for i in range(11)]   # v225-v235 temporaries


def O(b, e, i=None):
    base = (b * NE() + e) * 4
    return R("a", base, 4) if i is None else R("a", base + i)


def L(b, i=None):
    return R("a", 128 + 4 * b, 4) if i is None else R("a", 128 + 4 * b + i)


def Q(b, t):
    return R("a", 144 + 4 * NT() * b + 4 * t, 4)


# LDS: K buffers at 0 / 16384, V buffers at 32768 / 49152 (lane addresses
# carry the workgroup's LDS base)
KBUF = [0, 16384]
VBUF = [32768, 49152]
KADDR = [f"%[ka{t}]" for t in range(4)]
VADDR = ["%[va0]", "%[va1]"]

# Two key tiles per barrier ("dbl", head_dim 128 non-split programs under
# LDS-DMA): four K and four V images (K at 0..48K, V at 64K..112K, the item
# table after them at 128K), tiles issued two ahead (K(j+3), V(j+2) in
# iteration j), so an iteration of two steady tiles -- phase A(j), B(j),
# A(j+1), B(j+1) -- needs one vmcnt wait and one barrier, and the second
# phase A's first K fragments are read in the first phase B's tail.  The V
# images' ds offsets exceed 16 bits from the lane bases, so the V bases are
# copied + 64K into v188 / v189 (free under DMA staging), the prologue's V
# write base into v190.
# (default since round 6: bit-identical to the one-tile form, stamped tile
# 2887 -> 2784 cycles at S=8192 non-causal, 2969 -> 2899 causal; same
# process +1.0 % S=8192 non-causal, +0.75 % S=16384 causal, +0.3 % the
# headline, level S=8192 causal -- the cycles return partly as clock,
# profiles/r06_w4_dbl_stamps.jsonl, r06_ab_w4_dbl.jsonl; W4_XP=nodbl for A/B)
# (off under the experiments that use v184-v207 or s71: v14, rsa, epiwait16,
# prostamps)
DBL_XP = "nodbl" not in XP and not ({"v14", "rsa", "epiwait16"} & XP) and DIAG != "prostamps"
CUR = {"split": False}


def dbl():
    return DBL_XP and DMA_ON and HDC["hd"] == 128 and not CUR["split"]


def nbuf():   # K / V images per tensor
    return 4 if dbl() else 2


def look():   # tiles a DMA runs ahead of the iteration that reads them
    return 2 if dbl() else 1


def kbuf(i):  # ds offset of tile i's K image (from the %[ka*] lane bases)
    return 16384 * (i % nbuf())


def vbuf(i):  # ds offset of tile i's V image (from vaddr())
    return 16384 * (i % 4) if dbl() else VBUF[i % 2]


def vbuf_abs(i):  # LDS byte offset of tile i's V image (M0 of its DMA)
    return 65536 + 16384 * (i % 4) if dbl() else VBUF[i % 2]


def vaddr(k):
    return ("v188", "v189")[k] if dbl() else VADDR[k]


def vlds():
    return "v190" if dbl() else "%[vlds]"

# scalar scratch (clobbered): staging descriptors and loop state
SK = "s[40:43]"      # K stage descriptor (tile j+3 in iteration j)
SV = "s[44:47]"      # V stage descriptor (tile j+2)
SKREM, SVREM = "s48", "s49"  # remaining bytes (signed) of those descriptors
SJ, SJ1 = "s50", "s51"       # j, j+1
SNW, SNW1 = "s52", "s53"     # n_w, n_w - 1
SMASKJ = "s54"               # j+2 == n_w and the wave's last tile needs a mask
ST0, ST1 = "s55", "s56"
# item state (the item loop runs inside the asm: fa_w4_kernel.hpp's item
# table in LDS, 16 dwords per item, read at each item start)
RQ, RO, RL = "s[72:75]", "s[76:79]", "s[80:83]"   # Q / O of the head, split: LSE rows
NX = "s[84:87]"             # scratch descriptor for the next item's prefetch
QW, QM, NTILES, KVHI = "s88", "s89", "s90", "s91"  # this wave's first row, mask coordinate
ITEM, WARM = "s92", "s93"   # item index; 1 if this item's Q, K(0), V(0), K(1) were prefetched
SNWMIN = "s71"              # dbl: the item's smallest n_w over the four waves (PEND's slot: RSA is off)


def kslot(cb, t):
    """K fragment slot of (key block cb, k-step t): two key blocks' fragments
    at head_dim 128 (read one key block ahead), the whole tile's 8 at 64"""
    return 4 * (cb & 1) + t if NT() == 4 else 2 * cb + t


# K / V images hold packed rows (fa_w4_kernel.hpp: 256-B rows at head_dim
# 128, 128-B rows at 64): a 16-key block is 16 ROWB() bytes of K, a 32-key
# step 32 ROWB() of V
def k_read(t, cb, slot, kb):
    return dsr(f"ds_read_b128 {KF(slot)}, {KADDR[t]} offset:{kb + 16 * ROWB() * cb}", KF(slot), KADDR[t])


def v_reads(u, e, slot, vb):
    off = vb + 32 * ROWB() * u + 512 * (e >> 1)
    a = vaddr(e & 1)
    return [dsr(f"ds_read_b64_tr_b16 {VF(slot, 0)}, {a} offset:{off}", VF(slot, 0), a),
            dsr(f"ds_read_b64_tr_b16 {VF(slot, 1)}, {a} offset:{off + 16 * ROWB()}", VF(slot, 1), a)]


def qk_chain(b, cb, slots):
    """S(b,cb) = sum_t K[t][cb] . Q[b][t]^T, C = -m_ref on the first step"""
    out = []
    for t in range(NT()):
        c = NEGM(b) if t == 0 else S(b, cb)
        out.append(mfma(S(b, cb), KF(slots[t]), Q(b, t), c))
    return out


def cvt_block(b, cb):
    """fp16 P from the exp2'd scores of block (b, cb): pf[b][cb>>1][4(cb&1)+i]"""
    p = 64 + 8 * b + 4 * (cb >> 1) + 2 * (cb & 1)
    s = 16 * b + 4 * cb
    return [valu(f"{DT['cvt_pk']} v{p}, v{s}, v{s + 1}", r=[f"v{s}", f"v{s + 1}"], w=[f"v{p}"]),
            valu(f"{DT['cvt_pk']} v{p + 1}, v{s + 2}, v{s + 3}", r=[f"v{s + 2}", f"v{s + 3}"], w=[f"v{p + 1}"])]


def max_block(b, cb, first):
    h = b >> 1
    s = 16 * b + 4 * cb
    m = RMAX[h]
    if first:
        return [valu(f"v_max3_f32 {m}, v{s}, v{s + 1}, v{s + 2}", r=[f"v{s}", f"v{s + 1}", f"v{s + 2}"], w=[m]),
                valu(f"v_max_f32 {m}, {m}, v{s + 3}", r=[m, f"v{s + 3}"], w=[m])]
    return [valu(f"v_max3_f32 {m}, {m}, v{s}, v{s + 1}", r=[m, f"v{s}", f"v{s + 1}"], w=[m]),
            valu(f"v_max3_f32 {m}, {m}, v{s + 2}, v{s + 3}", r=[m, f"v{s + 2}", f"v{s + 3}"], w=[m])]


def exp_ops():
    return [valu(f"v_exp_f32 v{x}, v{x}", r=[f"v{x}"], w=[f"v{x}"], kind="trans") for x in range(64)]


def pv_mfmas(rowsums=True):
    """PV + row sums in M16::pv order: for u: for e: 4 b; then 4 row sums"""
    ms, frag_first = [], {}
    for u in range(2):
        for e in range(NE()):
            f = u * NE() + e
            frag_first[f] = len(ms)
            for b in range(4):
                ms.append(mfma(O(b, e), VF(vslot(f)), P(b, u), O(b, e)))
        if rowsums:
            ms += rowsum_mfmas(u)
    return ms, frag_first


def rowsum_mfmas(u):
    return [mfma(L(b), ONES, P(b, u), L(b)) for b in range(4)]


# Staging sets: stage j's K/V rows live in set j & 1 between their global
# loads and their LDS writes -- set 0 in VGPRs, set 1 in AGPRs a208-a239 --
# so the loads of stage j+1 (phase A) and the LDS writes of stage j (phase
# B) sit in different halves of an iteration.
STAGE2 = "stage1" not in XP
# first phase-A gap and spacing of the next stage's global loads (8 loads +
# 8 descriptor updates)
LD_AT = int(os.environ.get("W4_LD_AT", "18"))
LD_SP = int(os.environ.get("W4_LD_SP", "2"))
DMA_AT = int(os.environ.get("W4_DMA_AT", "2"))  # first phase-A gap of the DMA sequence
# gaps between its instructions: 1 at head_dim 128, 2 at 64 (+0.1-1.6 % over
# 1 there, profiles/r05_ab_d64var.jsonl "dsp2")
DMA_SP_ENV = os.environ.get("W4_DMA_SP")


def dma_sp():
    return int(DMA_SP_ENV) if DMA_SP_ENV else (1 if HDC["hd"] == 128 else 2)
CVT0 = "cvt0" in XP
CVT_EARLY = "cvtearly" in XP
# the 8 row-sum MFMAs of PV(j) at the start of phase A(j+1), under the K
# reads' latency, instead of at the end of the exp2-bound phase B(j)
RSA = "rsa" in XP
# head_dim 128: V(0) / K(1) written before the prologue's first barrier with
# K(0), one barrier per item seam instead of two (+0.3-0.8 %; at 64 level to
# -0.5 %, profiles/r04_ab_w4_one_barrier_seam{,_d64}.jsonl; W4_XP=twobar
# keeps two at 128 too)
ONEBAR_XP = "twobar" not in XP
ONEBAR64_XP = "onebar64" in XP


def onebar():
    return ONEBAR_XP and (HDC["hd"] == 128 or ONEBAR64_XP)
# gap of a chain's maxima within chain x + LAG, and the first phase-B gap of
# phase A's leftover maxima: one gap later than the hazard windows need
# spares 3 of a tile's 5 s_nop (profiles/r04_ab_w4_nop_trim*.jsonl)
MAX_OFF = int(os.environ.get("W4_MAX_OFF", "2"))
LEFT_OFF = int(os.environ.get("W4_LEFT_OFF", "3"))


# K/V staging by LDS-DMA (the default; W4_XP=regstage: the round-3 register
# staging, for A/B): each wave's 4+4 1-KiB pieces of the
# next K/V tiles go straight into their LDS images (buffer_load_dwordx4 ...
# lds, lane-linear destination at M0, per-lane source offsets through the
# images' inverse swizzle), so phase B carries no ds_writes and no staging
# registers are needed.  Issued in phase A of iteration j into the buffers
# iteration j-1 finished reading (K(j+2) -> kbuf[j&1], V(j+1) -> vbuf[(j+1)&1])
# and waited for (vmcnt(0)) before the iteration's barrier.
DMA_ON = "regstage" not in XP
SM0 = "s70"          # M0 of the enclosing code, restored at the end
PEND = "s71"         # 1: the last phase B's row sums are pending (RSA)


def dma():
    """LDS-DMA staging (both head dims: the images are packed, so a
    lane-linear 1-KiB piece carries no padding -- four pieces per wave and
    tensor at head_dim 128, two at 64)"""
    return DMA_ON


def npiece():  # LDS-DMA pieces per wave, tile and tensor (1 KiB each)
    return TILEB() // 4096


def sg0():  # prologue stage-0 loads in flight (none under DMA)
    return 0 if dma() else 2 * NPASS()


def nst():  # an item's O stores per wave
    return 2 * NE()


def KD(i):
    return R("v", 176 + i)   # per-pass K source offsets (DMA)


def VD(i):
    return R("v", 180 + i)   # per-pass V source offsets (DMA)


def kst(i, st_set):
    return KST(i) if st_set == 0 else R("a", 208 + 4 * i, 4)


def vst(i, st_set):
    return VST(i) if st_set == 0 else R("a", 224 + 4 * i, 4)


def stage_writes(p):
    """LDS writes of stage j (K(j+2) -> kbuf[j&1], V(j+1) -> vbuf[(j+1)&1]);
    with two sets the 8 youngest loads (stage j+1) may still be in flight"""
    if dma():
        return []
    ss = p if STAGE2 else 0
    out = [f"s_waitcnt vmcnt({2 * NPASS() if STAGE2 else 0})"]
    for i in range(NPASS()):
        out.append(dsw(f"ds_write_b128 %[klds], {kst(i, ss)} offset:{KBUF[p] + PASSL() * i}", "%[klds]", kst(i, ss)))
        out.append(dsw(f"ds_write_b128 %[vlds], {vst(i, ss)} offset:{VBUF[1 - p] + PASSL() * i}", "%[vlds]", vst(i, ss)))
    return out


def dma_loads(p):
    """LDS-DMA of K(j+1+look) and V(j+look) into their images (iteration j,
    p = j mod nbuf; two images per tensor: K(j+2) -> kbuf[p], V(j+1) ->
    vbuf[1-p]): wave w's piece i of a tile is LDS bytes [4096w + 1024i,
    +1024), M0 set per piece (one MFMA between the M0 write and the load: its
    wait state); then the descriptors advance one tile"""
    out = []
    for i in range(npiece()):
        out.append(salu(f"s_add_u32 m0, %[dmab], {kbuf(p + 1 + look()) + 1024 * i}"))
        out.append(vmem(f"buffer_load_dwordx4 {KD(i)}, {SK}, 0 offen lds", r=[KD(i)]))
    for i in range(npiece()):
        out.append(salu(f"s_add_u32 m0, %[dmab], {vbuf_abs(p + look()) + 1024 * i}"))
        out.append(vmem(f"buffer_load_dwordx4 {VD(i)}, {SV}, 0 offen lds", r=[VD(i)]))
    tb = hex(TILEB())
    out += [salu(f"s_add_u32 s40, s40, {tb}"), salu("s_addc_u32 s41, s41, 0"),
            salu(f"s_sub_i32 {SKREM}, {SKREM}, {tb}"), salu(f"s_max_i32 s42, {SKREM}, 0"),
            salu(f"s_add_u32 s44, s44, {tb}"), salu("s_addc_u32 s45, s45, 0"),
            salu(f"s_sub_i32 {SVREM}, {SVREM}, {tb}"), salu(f"s_max_i32 s46, {SVREM}, 0")]
    return out


def dma_setup(st):
    """M0 saved; per-pass DMA source offsets from the lane constants
    (kdma = piece 0's, K(i) = (kdma + 1024 i) ^ 64 i; vdma = piece 0's; head
    dim 128: V(i) = vdma + 2048 (i >> 1) + 128 (i & 1), chunk bit 1 flipped
    for i >= 2; head dim 64: V(1) = (vdma + 1024) ^ 32 -- 8 rows on, whose
    chunk XOR (row >> 2) & 3 differs by 2)"""
    st.raw(f"s_mov_b32 {SM0}, m0")
    st.raw(f"v_mov_b32 {KD(0)}, %[kdma]")
    st.raw(f"v_mov_b32 {VD(0)}, %[vdma]")
    for i in range(1, npiece()):
        st.raw(f"v_add_u32 {KD(i)}, {1024 * i}, %[kdma]")
        st.raw(f"v_xor_b32 {KD(i)}, {64 * i}, {KD(i)}")
        if HDC["hd"] == 64:
            st.raw(f"v_add_u32 {VD(i)}, 1024, %[vdma]")
            st.raw(f"v_xor_b32 {VD(i)}, 32, {VD(i)}")
            continue
        st.raw(f"v_add_u32 {VD(i)}, {2048 * (i >> 1) + 128 * (i & 1)}, %[vdma]")
        if i >= 2:
            st.raw(f"v_xor_b32 {VD(i)}, 32, {VD(i)}")
    st.nop(1)


def stage_loads(st_set=0, p=None):
    """global loads of the next stage into a staging set, then the
    descriptors advance one tile (bytes left clamp at 0: no traffic past the end)"""
    if dma():
        return dma_loads(p)
    out = []
    for i in range(NPASS()):
        out.append(vmem(f"buffer_load_dwordx4 {kst(i, st_set)}, {KOFF[i]}, {SK}, 0 offen", r=[KOFF[i]], w=[kst(i, st_set)]))
        out.append(vmem(f"buffer_load_dwordx4 {vst(i, st_set)}, {VOFF[i]}, {SV}, 0 offen", r=[VOFF[i]], w=[vst(i, st_set)]))
    if "noadv" in XP:  # timing only: every stage re-reads the same (L1-hot) tile
        return out + [salu("s_nop 0")] * 8
    tb = hex(TILEB())
    out += [salu(f"s_add_u32 s40, s40, {tb}"), salu("s_addc_u32 s41, s41, 0"),
            salu(f"s_sub_i32 {SKREM}, {SKREM}, {tb}"), salu(f"s_max_i32 s42, {SKREM}, 0"),
            salu(f"s_add_u32 s44, s44, {tb}"), salu("s_addc_u32 s45, s45, 0"),
            salu(f"s_sub_i32 {SVREM}, {SVREM}, {tb}"), salu(f"s_max_i32 s46, {SVREM}, 0")]
    return out


# ---------------------------------------------------------------------------
# program pieces
# ---------------------------------------------------------------------------
def lag():
    return 2 if NT() == 4 else 3


# bf16 scores in fp32 (verdict r05 item 5): the bf16 programs take Q into
# the MFMA unscaled (exact), start each chain from C = -m_ref / c and
# multiply every score by c = log2(e)/sqrt(d) in fp32 after its chain --
# instead of a bf16-rounded Q * c (8 mantissa bits: 4.3-5.2e-3 max error on
# peaked inputs against SDPA's 1.4-1.5e-3, profiles/r05_bf16_peaked_err.jsonl).
# fp16 keeps Q * c (11 bits: within the oracle gate).  W4_XP=bf16q: the old
# bf16 form, for A/B.
BF16_FP32SCALE = "bf16q" not in XP


def fp32scale():
    return BF16_FP32SCALE and DT.get("bf16", False)


def c_lits():
    """(c, -1/c) as fp32 hex literals, c = fp32(1/sqrt(hd)) * fp32(log2 e) as
    fa_fwd.hip computes p.c"""
    import struct
    import numpy as np
    hd = HDC["hd"]
    c = np.float32(np.float32(1.0) / np.sqrt(np.float32(hd))) * np.float32(1.4426950408889634)
    ni = np.float32(-1.0) / np.float32(c)
    h = lambda x: "0x%08x" % struct.unpack("<I", struct.pack("<f", float(x)))[0]  # noqa: E731
    return h(c), h(ni)


def scale_ops(b, cb):
    """S(b, cb) *= c in fp32 (fp32scale)"""
    cl = c_lits()[0]
    x = 16 * b + 4 * cb
    return [valu(f"v_mul_f32_e32 v{x + i}, {cl}, v{x + i}", r=[f"v{x + i}"], w=[f"v{x + i}"]) for i in range(4)]


def phase_a(st, p, with_max, diag=False, k0_issued=False):
    """QK^T(j+1) from kbuf[(j+1)&1] beside cvt P(j), maxima of S(j+1), staging.
    diag: the wave's causal diagonal tile with its keys aligned to its rows
    (kv0 = qm, a whole tile before kv_hi): 16-row block (b, cb) is all valid
    below the diagonal (cb < b), all masked above it (cb > b: no MFMAs, the
    scores set to -inf), and masked per element on it (key 4sg + i > row r16)
    -- the general mask_last_tile + full_max path, block by block, beside
    the 40 remaining MFMAs"""
    kb = kbuf(p + 1)
    chains = [(b, cb) for cb in range(4) for b in range(4) if not diag or cb <= b]
    mf = []
    if "tmajor" in XP:
        for cb in range(4):
            slots = [4 * (cb & 1) + t for t in range(4)]
            ch = [qk_chain(b, cb, slots) for b in range(4)]
            for t in range(4):
                mf += [ch[b][t] for b in range(4)]
    else:
        for x, (b, cb) in enumerate(chains):
            slots = [kslot(cb, t) for t in range(NT())]
            mf += qk_chain(b, cb, slots)
    gaps = {}

    def put(k, ins):
        ins = ins if isinstance(ins, list) else [ins]
        if "nokread" in XP:
            ins = [i for i in ins if isinstance(i, str) or "ds_read_b128" not in i.text]
        if "novread" in XP:
            ins = [i for i in ins if isinstance(i, str) or "ds_read_b64_tr" not in i.text]
        gaps.setdefault(k, []).extend(ins)

    n = len(mf)
    # K reads of cb 0 first; the conversions of cb 0's four blocks cover
    # their LDS latency  (W4_XP=kpre, timing only: read in the previous phase B)
    # (head_dim 64: all 8 fragments of the tile at once, the slots hold them)
    k0 = ([k_read(t, cb, kslot(cb, t), kb) for cb in range(4) for t in range(2)] if NT() == 2
          else [k_read(t, 0, t, kb) for t in range(NT())])
    if RSA:
        # the previous PV's row sums, deferred by its phase B's fast path,
        # ahead of this QK^T under the cb-0 K reads' latency
        for ins in k0:
            st.emit(ins)
        flush_rowsums(st)
    elif k0_issued:
        pass  # read in the previous phase B's tail (dbl: no barrier between)
    elif NT() == 2 or "kpre" not in XP or diag or not with_max:
        put(0, k0)
    if diag:
        # blocks above the diagonal: P(j) out of them, then -inf
        above = [(b, cb) for cb in range(4) for b in range(4) if cb > b]
        for k, (b, cb) in enumerate(above):
            ins = cvt_block(b, cb)
            ins += [valu(f"v_mov_b32 {S(b, cb, i)}, {VNINF}", r=[VNINF], w=[S(b, cb, i)]) for i in range(4)]
            put((5 + 5 * k) if NT() == 4 else (2 + 3 * k), ins)
    for x, (b, cb) in enumerate(chains):
        c = cvt_block(b, cb)
        if "nocvt" in XP:
            pass
        elif CVT0 and not diag and NT() == 4:
            # every conversion ahead of the first MFMA, under the cb-0 K
            # reads' LDS latency (the registers they read were written by the
            # previous phase B's exp2; the chains overwrite them later)
            put(0, c)
        elif x < 4 or ("tmajor" in XP and b > 0):
            put(4 * (x - b) if x >= 4 else 0, c)
        elif "tmajor" in XP:
            put(4 * x - 2, c[0])
            put(4 * x - 1, c[1])
        elif CVT_EARLY and NT() == 4 and not diag:
            # the first conversion two gaps earlier, into the chain's empty
            # gap: one filler per gap (maxima at +2 / +3, conversions at +1 / +4)
            put(NT() * x - 3, c[0])
            put(NT() * x, c[1])
        else:
            put(NT() * x - 1, c[0])
            put(NT() * x, c[1])
        if diag and b == cb:
            # the diagonal block: key 16cb + 4sg + i is valid iff i <= r16 - 4sg
            for i in range(4):
                xr = S(b, cb, i)
                put(min(NT() * x + 2 * NT(), n), [valu(f"v_cmp_le_i32 vcc, {i}, %[vt]", r=["%[vt]"]),
                                valu(f"v_cndmask_b32 {xr}, {VNINF}, {xr}, vcc", r=[VNINF, xr], w=[xr])])
        # next cb's K fragments early in this cb's first chain (kspread: one
        # per chain of this cb)
        if "kspread" in XP and cb < 3 and not diag:
            put(4 * x + 1, k_read(b, cb + 1, 4 * ((cb + 1) & 1) + b, kb))
        elif b == (cb if diag else 0) and cb < 3 and NT() == 4:
            for t in range(NT()):
                put(NT() * x + 1 + t % 3, k_read(t, cb + 1, kslot(cb + 1, t), kb))
        # the running maxima of chain x - LAG (its MFMA results clear of the
        # 12-wait-state MFMA -> VALU window)
        if fp32scale() and with_max and x >= lag() and "nomax" not in XP:
            put(NT() * x + MAX_OFF - 1, scale_ops(*chains[x - lag()]))
        if with_max and x >= lag() and "nomax" not in XP:
            y = x - lag()
            by, cby = chains[y]
            mm = max_block(by, cby, first=(cby == 0 and by in (0, 2)))
            mo = MAX_OFF
            put(NT() * x + mo, mm[0])
            put(min(NT() * x + mo + 1, n), mm[1])
    # stage traffic: LDS writes in cb 0, loads in cb 1
    if "nostage" not in XP and dma():
        for i, ld in enumerate(stage_loads(p=p)):
            put((4 + i) if diag else (DMA_AT + dma_sp() * i), ld)
    elif "nostage" not in XP and STAGE2:
        for i, ld in enumerate(stage_loads(1 - p)):
            if HDC["hd"] == 128:
                put((10 + 2 * i) if diag else (LD_AT + LD_SP * i), ld)
            else:
                put((2 + i) if diag else (4 + 2 * i), ld)
    if "nostage" not in XP and "stage_a" in XP and not STAGE2:
        sw = stage_writes(p)
        put(0, sw[:1])
        for i, w in enumerate(sw[1:]):
            put(3 + 2 * i, w)
        for i, ld in enumerate(stage_loads()):
            put(20 + i, ld)
    # the first V^T fragments of PV(j) (V(j) is ready since the last barrier)
    if "vinA" in XP and with_max and not diag:  # timing only: all 16, spread over phase A
        for f in range(16):
            for i, r in enumerate(v_reads(f // 8, f % 8, f % 8, vbuf(p))):
                put(6 + 3 * f + i, r)
    for f in range(vahead()):
        for i, r in enumerate(v_reads(*divmod(f, NE()), vslot(f), vbuf(p))):
            put(n - 12 - 3 * (vahead() - 3) + 3 * f + i, r)
    if fp32scale():
        rest = chains[len(chains) - lag():] if with_max and "nomax" not in XP else chains
        for y in rest:
            put(n, scale_ops(*y))
    assert max(gaps) <= n, "every filler lands in a gap"
    st.interleave(mf, gaps)
    leftover = []
    if with_max and "nomax" not in XP:
        for y in range(len(chains) - lag(), len(chains)):
            by, cby = chains[y]
            leftover += max_block(by, cby, first=False)
    return leftover


def phase_b(st, p, leftover, dec_gap, label_slow, label_end, exps=True, kpre=None):
    """PV(j) from vbuf[j&1]; decision at dec_gap; exp2 of S(j+1) after it.
    kpre (dbl): tile index whose K image the next phase A reads -- its first
    key block's fragments are read in this phase's tail"""
    vb = vbuf(p)
    mf, frag_first = pv_mfmas(rowsums=not (RSA and exps) and "norowsum" not in XP)
    gaps = {}

    def put(k, ins):
        ins = ins if isinstance(ins, list) else [ins]
        if "novread" in XP:
            ins = [i for i in ins if isinstance(i, str) or "ds_read_b64_tr" not in i.text]
        gaps.setdefault(k, []).extend(ins)

    # V fragments V_AHEAD ahead (the first V_AHEAD were read in phase A)
    if v14():
        # slots 8-13 are free: fragments 8-13 at once; 14, 15 into slots 0, 1
        # once fragments 0, 1 have been consumed (MFMAs 0-7)
        for f in range(8, 16):
            u, e = divmod(f, NE())
            r = v_reads(u, e, vslot(f), vb)
            k = 2 * (f - 8) if f < 14 else 12 + 2 * (f - 14)
            put(k, r[0])
            put(k + 1, r[1])
    for f in range(vahead(), 2 * NE() if not ("vinA" in XP and exps and dec_gap > 0 or v14()) else vahead()):
        k = frag_first[f - vahead()]
        u, e = divmod(f, NE())
        r = v_reads(u, e, vslot(f), vb)
        put(k + 1, r[0])
        put(k + 2, r[1])
    for i, ins in enumerate(leftover):
        put(LEFT_OFF + i, ins)
    if "kpre" in XP and exps:  # timing only: next phase A's cb-0 K fragments (stale buffer)
        for t in range(4):
            put(len(mf) - 12 + 2 * t, k_read(t, 0, t, kbuf(p)))
    if kpre is not None:
        # the K fragments were consumed by the previous phase A: their slots
        # are free; K(kpre) was published by the barrier before this phase
        for t in range(NT()):
            put(len(mf) - 10 + 2 * t, k_read(t, 0, kslot(0, t), kbuf(kpre)))
    # stage traffic (phase A is the denser half): LDS writes of stage j, then
    # the next stage's global loads, spread over the gaps after the decision
    if "nostage" not in XP and ("stage_a" not in XP or STAGE2):
        sw = stage_writes(p)
        put(dec_gap + 2, sw[:1])
        for i, w in enumerate(sw[1:]):
            put(dec_gap + 3 + (6 if STAGE2 else 3) * i, w)
        if not STAGE2:
            for i, ld in enumerate(stage_loads()):
                put(dec_gap + 28 + 2 * i, ld)
    dec = [valu(f"v_max_f32 {T[0]}, {RMAX[0]}, {RMAX[1]}", r=[RMAX[0], RMAX[1]], w=[T[0]])
           if "nomax" not in XP else valu(f"v_mov_b32 {T[0]}, 0", w=[T[0]]),
           valu(f"v_cmp_lt_f32 vcc, 0x41000000, {T[0]}", r=[T[0]])]
    if exps and "noexp" not in XP:
        ex = exp_ops()
        n_g = len(mf) - dec_gap
        for i, e in enumerate(ex):
            put(dec_gap + 1 + (i * n_g) // len(ex), e)
    # emit up to the decision, fork to the slow path, then the fast remainder
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
        return mf, gaps
    if RSA:
        st.raw(f"s_mov_b32 {PEND}, 1")  # this PV's row sums: the next phase A
    if dec_gap > 0:
        stamp(st, 60)
        stamp_acc(st, 65, 60, 62)
        if DIAG == "stamps":
            st.raw("s_add_u32 s67, s67, 1")
    # timing only (wrong results): the steady path skips the DMA wait
    # (novmwait) or the wait and the barrier (nobar)
    if dec_gap > 0 and "nobar" in XP:
        st.branch("s_branch", label_end.replace("Lend", "Lendnb"))
    elif dec_gap > 0 and "novmwait" in XP:
        st.branch("s_branch", label_end.replace("Lend", "Lendnw"))
    else:
        st.branch("s_branch", label_end)
    # slow path: the remaining PV MFMAs (no exps), then rescale
    st.label(label_slow)
    for k in range(dec_gap, len(mf)):
        if k > dec_gap:
            for f in gaps.get(k, []):
                if isinstance(f, str) or f.kind != "trans":
                    st.emit(f)
        st.emit(mf[k])
    if RSA:
        # l takes this PV's row sums before the rescale scales it
        for u in range(2):
            for m in rowsum_mfmas(u):
                st.emit(m)
    slow_softmax(st, first=False)
    for e in exp_ops():
        st.emit(e)
    st.branch("s_branch", label_end)
    return mf, gaps


def flush_rowsums(st):
    """the row sums a phase B's fast path left pending (PEND = 1): the
    previous P is still in v64-95 (this phase's conversions follow)"""
    if not RSA:
        return
    skip = newlabel("nors")
    st.raw(f"s_cmp_eq_u32 {PEND}, 0")
    st.branch("s_cbranch_scc1", skip)
    for u in range(2):
        for m in rowsum_mfmas(u):
            st.emit(m)
    st.label(skip)
    st.raw(f"s_mov_b32 {PEND}, 0")


def row_max_b(st, b, dst):
    """per-lane max of row block b's 16 scores, then across the 4 lane groups"""
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
        for e in range(NE()):
            for i in range(4):
                a = O(b, e, i)
                st.emit(valu(f"v_accvgpr_read_b32 {T[4]}, {a}", r=[a], w=[T[4]]))
                st.emit(valu(f"v_mul_f32 {T[4]}, {T[4]}, {alpha}", r=[T[4], alpha], w=[T[4]]))
                st.emit(valu(f"v_accvgpr_write_b32 {a}, {T[4]}", r=[T[4]], w=[a]))
        for i in range(4):
            a = L(b, i)
            st.emit(valu(f"v_accvgpr_read_b32 {T[4]}, {a}", r=[a], w=[T[4]]))
            st.emit(valu(f"v_mul_f32 {T[4]}, {T[4]}, {alpha}", r=[T[4], alpha], w=[T[4]]))
            st.emit(valu(f"v_accvgpr_write_b32 {a}, {T[4]}", r=[T[4]], w=[a]))
    for i in range(16):
        x = f"v{16 * b + i}"
        st.emit(valu(f"v_sub_f32 {x}, {x}, {sh}", r=[x, sh], w=[x]))
    st.emit(valu(f"v_add_f32 {MREF[b]}, {MREF[b]}, {sh}", r=[MREF[b], sh], w=[MREF[b]]))
    for i in range(4):
        if fp32scale():
            st.emit(valu(f"v_mul_f32_e32 {NEGM(b, i)}, {c_lits()[1]}, {MREF[b]}", r=[MREF[b]], w=[NEGM(b, i)]))
        else:
            st.emit(valu(f"v_xor_b32 {NEGM(b, i)}, 0x80000000, {MREF[b]}", r=[MREF[b]], w=[NEGM(b, i)]))


_lbl = [0]


def stamp(st, dst):
    """diagnostic (W4_DIAG=stamps): shader-cycle counter into s[dst:dst+1]"""
    if DIAG == "stamps":
        st.raw(f"s_memtime s[{dst}:{dst + 1}]")
        st.raw("s_waitcnt lgkmcnt(0)")
        st.lgkm = []


def stamp_acc(st, acc, later, earlier):
    if DIAG == "stamps":
        st.raw(f"s_sub_u32 s68, s{later}, s{earlier}")
        st.raw(f"s_add_u32 s{acc}, s{acc}, s68")


def newlabel(tag):
    _lbl[0] += 1
    return f"L{tag}_{_lbl[0]}_%="


def slow_softmax(st, first):
    """The rare rescale (M16::softmax's wave-uniform branch), per 32-row half
    h = {2h, 2h+1}: the half moves m_ref iff one of its lanes' partial maxima
    grew past RESCALE_LOG2 = 8 (the 8-wave kernel's 32-row-wave decision).
    first: the item's first tile (have_ref = false): every row centres on its
    max (a fully masked row, max -inf, keeps m_ref = 0)."""
    for h in range(2):
        skip = newlabel("skip")
        if not first:
            # the half's running partial max (this tile's scores)
            st.emit(valu(f"v_cmp_lt_f32 vcc, 0x41000000, {RMAX[h]}", r=[RMAX[h]]))
            st.branch("s_cbranch_vccz", skip)
        for b in (2 * h, 2 * h + 1):
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


def mask_last_tile(st, causal):
    """S = -inf where key >= kv_hi or (causal) key > query row, for the wave's
    last tile (key kv = kv0 + 16cb + 4sg + i, row = qw + 16b + r16).
    With c = 16cb + i: valid iff c <= lim_b, lim_b = min(kv_hi - kv0 - 1 - 4sg,
    qw - kv0 + 16b + (r16 - 4sg)).  %[vt] = r16 - 4sg."""
    # ST0 = kv_hi - kv0 - 1, ST1 = qw - kv0   (set by the caller)
    lim_rag = T[5]
    st.emit(valu(f"v_sub_u32 {T[6]}, %[vt], %[r16]", r=["%[vt]", "%[r16]"], w=[T[6]]))   # -4sg
    st.emit(valu(f"v_add_u32 {lim_rag}, {ST0}, {T[6]}", r=[T[6]], w=[lim_rag]))
    for b in range(4):
        lim = T[7]
        if causal:
            st.emit(valu(f"v_add_u32 {lim}, {ST1}, %[vt]", r=["%[vt]"], w=[lim]))
            if b:
                st.emit(valu(f"v_add_u32 {lim}, {16 * b}, {lim}", r=[lim], w=[lim]))
            st.emit(valu(f"v_min_i32 {lim}, {lim}, {lim_rag}", r=[lim, lim_rag], w=[lim]))
        else:
            lim = lim_rag
        for cb in range(4):
            for i in range(4):
                x = f"v{16 * b + 4 * cb + i}"
                st.emit(valu(f"v_cmp_le_i32 vcc, {16 * cb + i}, {lim}", r=[lim]))
                st.emit(valu(f"v_cndmask_b32 {x}, {VNINF}, {x}, vcc", r=[VNINF, x], w=[x]))


def full_max(st):
    """running partial maxima of both halves over the whole tile (masked path)"""
    for b in range(4):
        for cb in range(4):
            for ins in max_block(b, cb, first=(cb == 0 and b in (0, 2))):
                st.emit(ins)


def qk_plain(st, kb):
    """QK^T of one tile, not interleaved (prologue)"""
    for cb in range(4):
        for t in range(NT()):
            st.emit(k_read(t, cb, kslot(cb, t), kb))
        for b in range(4):
            for m in qk_chain(b, cb, [kslot(cb, t) for t in range(NT())]):
                st.emit(m)


def pv_plain(st, p):
    vb = vbuf(p)
    mf, frag_first = pv_mfmas()
    gaps = {}
    for f in range(2 * NE()):
        u, e = divmod(f, NE())
        k = frag_first[f - 2] + 1 if f >= 2 else 0
        for i, r in enumerate(v_reads(u, e, vslot(f), vb)):
            gaps.setdefault(k + i if f >= 2 else 0, []).append(r)
    st.interleave(mf, gaps)


def double_steady(st, p, labels):
    """dbl: steady tiles j and j+1 (j mod 4 = p) in one barrier interval --
    phase A(j) [QK(j+1), DMA K(j+3) / V(j+2)], phase B(j) [PV(j); QK(j+2)'s
    first K fragments in its tail], phase A(j+1) [QK(j+2), DMA K(j+4) /
    V(j+3)], phase B(j+1) [PV(j+1)]; then one DMA wait and one barrier.  The
    images it reads (K(j+1), K(j+2), V(j), V(j+1)) were published by the
    previous barrier; the ones it fills were last read before it."""
    L, nb = labels, nbuf()
    q = (p + 1) % nb
    left = phase_a(st, p, with_max=True)
    stamp(st, 62)
    stamp_acc(st, 64, 62, 60)
    phase_b(st, p, left, dec_gap=6, label_slow=L["dslow1"][p], label_end=L["dmid"][p], kpre=p + 2)
    st.label(L["dmid"][p])
    left = phase_a(st, q, with_max=True, k0_issued=True)
    stamp(st, 62)
    stamp_acc(st, 64, 62, 60)
    phase_b(st, q, left, dec_gap=6, label_slow=L["dslow2"][p], label_end=L["dend"][p])
    st.label(L["dend"][p], drain_lgkm=True)
    st.raw("s_waitcnt vmcnt(0)")
    st.raw("s_barrier")
    stamp(st, 62)
    stamp_acc(st, 66, 62, 60)
    st.raw(f"s_add_u32 {SJ}, {SJ}, 2")
    st.raw(f"s_cmp_lt_u32 {SJ}, {NTILES}")
    st.jump("s_cbranch_scc1", L["loop"][(p + 2) % nb])
    st.jump("s_branch", L["done"])


def body(st, p, causal, labels):
    """one loop iteration j of parity p = j mod nbuf (dbl, odd p: two steady
    tiles per barrier when both are steady)"""
    L = labels
    st.label(L["loop"][p], drain_lgkm=True)
    stamp(st, 60)
    st.raw(f"s_add_u32 {SJ1}, {SJ}, 1")
    st.raw(f"s_cmp_lt_u32 {SJ1}, {SNW}")
    st.branch("s_cbranch_scc0", L["notsteady"][p])
    st.raw(f"s_add_u32 {ST0}, {SJ}, 2")
    st.raw(f"s_cmp_eq_u32 {ST0}, {SMASKJ}")
    st.branch("s_cbranch_scc1", L["masked"][p])
    if dbl() and p % 2 == 1:
        # two tiles per barrier only where EVERY wave's tiles j and j+1 are
        # steady (j + 3 < the smallest n_w: no wave drains or masks QK(j+1) /
        # QK(j+2)) -- the choice must be the workgroup's, or the waves' barrier
        # counts would part (causal waves have n_w = n_0 .. n_0 + 3)
        st.raw(f"s_add_u32 {ST1}, {SJ}, 3")
        st.raw(f"s_cmp_lt_u32 {ST1}, {SNWMIN}")
        st.branch("s_cbranch_scc0", L["single"][p])
        double_steady(st, p, labels)
        st.label(L["single"][p])
    # ---- steady: QK(j+1) with maxima, PV(j) with exps ----
    left = phase_a(st, p, with_max=True)
    stamp(st, 62)
    stamp_acc(st, 64, 62, 60)
    phase_b(st, p, left, dec_gap=6, label_slow=L["slow"][p], label_end=L["end"][p])
    # ---- masked: the wave's last QK (causal diagonal / ragged end) ----
    st.label(L["masked"][p])
    # kv0 = 64 (j+1): ST0 = kv_hi - kv0 - 1, ST1 = qm - kv0
    st.raw(f"s_lshl_b32 {ST1}, {SJ1}, 6")
    st.raw(f"s_sub_i32 {ST0}, {KVHI}, {ST1}")
    st.raw(f"s_sub_i32 {ST0}, {ST0}, 1")
    st.raw(f"s_sub_i32 {ST1}, {QM}, {ST1}")
    if causal and DIAG_FAST:
        # ---- aligned causal diagonal (every causal wave's last QK unless the
        # tile is ragged): masked block by block inside phase A ----
        st.raw(f"s_cmp_eq_u32 {ST1}, 0")
        st.branch("s_cbranch_scc0", L["general"][p])
        st.raw(f"s_cmp_ge_i32 {ST0}, 63")
        st.branch("s_cbranch_scc0", L["general"][p])
        left = phase_a(st, p, with_max=True, diag=True)
        stamp(st, 62)
        stamp_acc(st, 64, 62, 60)
        phase_b(st, p, left, dec_gap=6, label_slow=L["slow3"][p], label_end=L["end"][p])
        st.label(L["general"][p])
    phase_a(st, p, with_max=False)
    mask_last_tile(st, causal)
    full_max(st)
    phase_b(st, p, [], dec_gap=0, label_slow=L["slow2"][p], label_end=L["end"][p])
    # ---- drain (j = n_w - 1: PV only) / idle (j >= n_w: staging only) ----
    st.label(L["notsteady"][p])
    flush_rowsums(st)  # before the drain's conversions overwrite that P
    st.raw(f"s_cmp_eq_u32 {SJ1}, {NTILES}")
    st.branch("s_cbranch_scc1", L["last"][p])
    if dma():
        for ins in stage_loads(p=p):
            st.emit(ins)
            if isinstance(ins, Ins) and ins.text.startswith("s_add_u32 m0"):
                st.nop(1)
    elif STAGE2:
        for ins in stage_loads(1 - p) + stage_writes(p):
            st.emit(ins)
    else:
        for ins in stage_writes(p) + stage_loads():
            st.emit(ins)
    st.raw(f"s_cmp_lt_u32 {SJ}, {SNW}")
    st.branch("s_cbranch_scc0", L["end"][p])
    for b in range(4):
        for cb in range(4):
            for c in cvt_block(b, cb):
                st.emit(c)
    pv_plain(st, p)
    st.branch("s_branch", L["end"][p])
    # ---- the item's last iteration: no staging (its tiles lie past the
    # item); with a next item, its Q, K(0), V(0), K(1) are loaded into the
    # registers the prologue would load them into, once the drain's
    # conversions have freed the S registers
    st.label(L["last"][p])
    nopf, drain_pf, done_pf = newlabel("nopf"), newlabel("drainpf"), newlabel("donepf")
    st.raw(f"s_mov_b32 {WARM}, 0")
    st.raw(f"s_add_u32 {ST0}, {ITEM}, 1")
    st.raw(f"s_cmp_lt_u32 {ST0}, %[nitems]")
    st.branch("s_cbranch_scc0", nopf)
    st.raw(f"s_mov_b32 {WARM}, 1")
    st.raw(f"s_cmp_lt_u32 {SJ}, {SNW}")
    st.branch("s_cbranch_scc1", drain_pf)
    prefetch_next(st)
    st.branch("s_branch", L["end_nowait" if dma() else "end"][p])
    st.label(drain_pf)
    for b in range(4):
        for cb in range(4):
            for c in cvt_block(b, cb):
                st.emit(c)
    if PF_BEFORE_DRAIN:
        prefetch_next(st)
        pv_plain(st, p)
    else:
        # the drain's PV first: its MFMAs would otherwise queue behind the
        # prefetch's vector-memory issue
        pv_plain(st, p)
        prefetch_next(st)
    st.branch("s_branch", L["end_nowait" if dma() else "end"][p])
    st.label(nopf)
    st.raw(f"s_cmp_lt_u32 {SJ}, {SNW}")
    st.branch("s_cbranch_scc0", L["end"][p])
    for b in range(4):
        for cb in range(4):
            for c in cvt_block(b, cb):
                st.emit(c)
    pv_plain(st, p)
    st.label(L["end"][p], drain_lgkm=True)
    if dma() and "epiwait16" in XP:
        # timing only (wrong results): iteration 0 after a deferred epilogue
        # does not wait for the epilogue's 16 O stores (nor, since they are
        # older, reliably for its own DMA) -- the O stores' ack latency
        w16, wd = newlabel("w16"), newlabel("wd")
        st.raw(f"s_cmp_eq_u32 {PEND}, 1")
        st.branch("s_cbranch_scc1", w16)
        st.raw("s_waitcnt vmcnt(0)")
        st.branch("s_branch", wd)
        st.label(w16)
        st.raw(f"s_waitcnt vmcnt({nst()})")
        st.raw(f"s_mov_b32 {PEND}, 0")
        st.label(wd)
        st.label(L["end_nowait"][p], drain_lgkm=True)
    elif dma():
        # this iteration's LDS-DMA landed before the barrier publishes it (the
        # last iteration issues none: its next-item prefetch stays in flight)
        st.raw("s_waitcnt vmcnt(0)")
        st.label(L["end_nowait"][p], drain_lgkm=True)
    if "novmwait" in XP and "nobar" not in XP:
        st.label(L["end"][p].replace("Lend", "Lendnw"), drain_lgkm=True)
    st.raw("s_barrier")
    if "nobar" in XP:
        st.label(L["end"][p].replace("Lend", "Lendnb"), drain_lgkm=True)
    stamp(st, 62)
    stamp_acc(st, 66, 62, 60)
    st.raw(f"s_add_u32 {SJ}, {SJ}, 1")
    st.raw(f"s_cmp_lt_u32 {SJ}, {NTILES}")
    if p < nbuf() - 1:
        st.jump("s_cbranch_scc0", L["done"])  # else on to body p + 1
    else:
        st.jump("s_cbranch_scc1", L["loop"][0])


def prostamp(st, i):
    """diagnostic (W4_DIAG=prostamps): per-wave accumulated cycles of the
    prologue's phases, in the DMA-freed v184-v207 (lanes identical):
    v197 = last stamp, v200 + i += cycles since it; v206 = items"""
    if DIAG != "prostamps":
        return
    st.raw("s_memtime s[58:59]")
    st.raw("s_waitcnt lgkmcnt(0)")
    st.lgkm = []
    st.raw("v_mov_b32 v198, s58")
    if i >= 0:
        st.raw("v_sub_u32 v196, v198, v197")
        st.raw(f"v_add_u32 v{200 + i}, v{200 + i}, v196")
    st.raw("v_mov_b32 v197, v198")


def pstamp(st, dst):
    """diagnostic (W4_DIAG=pstamps): shader-cycle counter into s[dst:dst+1]"""
    if DIAG == "pstamps":
        st.raw(f"s_memtime s[{dst}:{dst + 1}]")
        st.raw("s_waitcnt lgkmcnt(0)")
        st.lgkm = []


def slot_read(st, item_sgpr, dst0):
    """the 16-dword table slot of item `item_sgpr` into v[dst0:dst0+15]"""
    st.raw(f"s_lshl_b32 {ST0}, {item_sgpr}, 6")
    st.raw(f"s_add_u32 {ST0}, {ST0}, %[tab]")
    st.raw(f"v_mov_b32 {T[0]}, {ST0}")
    for i in range(4):
        st.raw(f"ds_read_b128 {R('v', dst0 + 4 * i, 4)}, {T[0]} offset:{16 * i}")
    st.raw("s_waitcnt lgkmcnt(0)")


def rsrc(st, dst, lo, hi, records):
    """buffer descriptor s[dst:dst+3] from base (lo, hi) and num_records"""
    st.raw(f"s_mov_b32 s{dst}, {lo}")
    st.raw(f"s_and_b32 s{dst + 1}, {hi}, 0xffff")
    st.raw(f"s_mov_b32 s{dst + 2}, {records}")
    st.raw(f"s_mov_b32 s{dst + 3}, 0x20000")


# item table slot (fa_w4_kernel.hpp W4Slot): 0-1 Q head, 2-3 K head (+k0
# rows), 4-5 V head (+k0 rows), 6-7 O rows base, 8 K/V bytes, 9 q0,
# 10 tiles, 11 key bound, 12 k0, 13 O bytes, 14-15 LSE rows base
def read_item(st, causal):
    """this item's scalars from its table slot, and this wave's row range,
    tile count n_w and last-tile mask flag (the C++ W4Item of round 2)"""
    slot_read(st, ITEM, 128)
    rl = lambda i: f"v{128 + i}"
    for dst, i in ((40, 2), (41, 3), (44, 4), (45, 5), (ST0, 0), (ST1, 1)):
        st.raw(f"v_readfirstlane_b32 {dst if isinstance(dst, str) else 's%d' % dst}, {rl(i)}")
    rsrc(st, 72, ST0, ST1, "%[qrec]")                     # RQ
    st.raw("v_readfirstlane_b32 s42, v136")                # K/V bytes
    st.raw("s_and_b32 s41, s41, 0xffff")
    st.raw("s_mov_b32 s43, 0x20000")
    st.raw("s_and_b32 s45, s45, 0xffff")
    st.raw("s_mov_b32 s46, s42")
    st.raw("s_mov_b32 s47, 0x20000")
    st.raw(f"v_readfirstlane_b32 {ST0}, v134")
    st.raw(f"v_readfirstlane_b32 {ST1}, v135")
    st.raw("v_readfirstlane_b32 s57, v141")               # O bytes
    rsrc(st, 76, ST0, ST1, "s57")                          # RO
    st.raw(f"v_readfirstlane_b32 {ST0}, v142")
    st.raw(f"v_readfirstlane_b32 {ST1}, v143")
    # LSE bytes = O bytes * 4 / ROWB (one fp32 per row of ROWB() O bytes)
    shift = (ROWB() // 4).bit_length() - 1
    assert 4 << shift == ROWB()
    st.raw(f"s_lshr_b32 s57, s57, {shift}")
    rsrc(st, 80, ST0, ST1, "s57")                          # RL
    st.raw(f"v_readfirstlane_b32 {QW}, v137")             # q0
    st.raw(f"s_add_u32 {QW}, {QW}, %[woff]")              # + 64 wave
    st.raw(f"v_readfirstlane_b32 {NTILES}, v138")
    st.raw(f"v_readfirstlane_b32 {KVHI}, v139")
    st.raw(f"v_readfirstlane_b32 {ST0}, v140")            # k0
    st.raw(f"s_sub_i32 {QM}, {QW}, {ST0}")
    # n_w = causal ? max(0, min(tiles, (qm >> 6) + 1)) : tiles
    if causal:
        st.raw(f"s_ashr_i32 {SNW}, {QM}, 6")
        st.raw(f"s_add_i32 {SNW}, {SNW}, 1")
        st.raw(f"s_min_i32 {SNW}, {SNW}, {NTILES}")
        st.raw(f"s_max_i32 {SNW}, {SNW}, 0")
    else:
        st.raw(f"s_mov_b32 {SNW}, {NTILES}")
    st.raw(f"s_sub_u32 {SNW1}, {SNW}, 1")
    if dbl():
        # n_w of wave 0 (qm - woff): the workgroup's smallest
        if causal:
            st.raw(f"s_sub_i32 {SNWMIN}, {QM}, %[woff]")
            st.raw(f"s_ashr_i32 {SNWMIN}, {SNWMIN}, 6")
            st.raw(f"s_add_i32 {SNWMIN}, {SNWMIN}, 1")
            st.raw(f"s_min_i32 {SNWMIN}, {SNWMIN}, {NTILES}")
            st.raw(f"s_max_i32 {SNWMIN}, {SNWMIN}, 0")
        else:
            st.raw(f"s_mov_b32 {SNWMIN}, {SNW}")
    # the wave's last tile (key kv0 = 64 (n_w - 1)) needs a mask iff it
    # reaches the key bound or (causal) the diagonal: SMASKJ = n_w, else never
    st.raw(f"s_lshl_b32 {ST0}, {SNW}, 6")                 # kv0 + 64
    st.raw(f"s_cmp_gt_i32 {ST0}, {KVHI}")
    st.raw(f"s_cselect_b32 {ST1}, 1, 0")
    if causal:
        st.raw(f"s_sub_i32 {ST0}, {ST0}, 1")
        st.raw(f"s_cmp_gt_i32 {ST0}, {QM}")
        st.raw(f"s_cselect_b32 {ST0}, 1, 0")
        st.raw(f"s_or_b32 {ST1}, {ST1}, {ST0}")
    st.raw(f"s_cmp_eq_u32 {ST1}, 0")
    st.raw(f"s_cselect_b32 {SMASKJ}, -1, {SNW}")
    st.nop(5)  # VALU-written descriptor words (readfirstlane) -> buffer loads


def prefetch_next(st):
    """the next item's Q rows (this wave's 64) into v0-63, K(0) into v112..,
    V(0) and K(1) into staging set 1 -- the cold prologue's loads, issued in
    this item's last iteration (plain loads: ~10 cycles of issue each, where
    LDS-DMA pieces cost ~100); their latency hides under the PV drain, the
    epilogue and the next item's table read"""
    slot_read(st, f"{ST0}", 112)   # ST0 = ITEM + 1 (set by the caller)
    st.raw(f"v_readfirstlane_b32 {ST0}, v112")
    st.raw(f"v_readfirstlane_b32 {ST1}, v113")
    rsrc(st, 84, ST0, ST1, "%[qrec]")
    st.raw(f"v_readfirstlane_b32 {ST0}, v121")            # next q0
    st.raw(f"s_add_u32 {ST0}, {ST0}, %[woff]")
    st.raw(f"s_lshl_b32 {ST0}, {ST0}, {ROWSH()}")
    st.raw(f"v_readfirstlane_b32 s57, v120")              # next K/V bytes
    st.raw(f"v_readfirstlane_b32 s94, v114")               # next K base
    st.raw(f"v_readfirstlane_b32 s95, v115")
    st.raw(f"v_readfirstlane_b32 s96, v116")               # next V base
    st.raw(f"v_readfirstlane_b32 s97, v117")
    for b in range(4):
        st.raw(f"v_add_u32 {T[b]}, {ST0}, %[qoff]")
        if b:
            st.raw(f"v_add_u32 {T[b]}, {16 * ROWB() * b}, {T[b]}")
    st.nop(4)
    for b in range(4):
        for t in range(NT()):
            st.raw(f"buffer_load_dwordx4 {R('v', 4 * NT() * b + 4 * t, 4)}, {T[b]}, {NX}, 0 offen offset:{64 * t}")
    rsrc(st, 84, "s94", "s95", "s57")
    st.nop(4)
    for i in range(NPASS()):
        st.raw(f"buffer_load_dwordx4 {R('v', 112 + 4 * i, 4)}, {KOFF[i]}, {NX}, 0 offen")
    for i in range(NPASS()):
        st.raw(f"v_add_u32 {T[4 + i]}, {hex(TILEB())}, {KOFF[i]}")
    st.nop(1)
    for i in range(NPASS()):
        st.raw(f"buffer_load_dwordx4 {kst(i, 1)}, {T[4 + i]}, {NX}, 0 offen")
    rsrc(st, 84, "s96", "s97", "s57")
    st.nop(4)
    for i in range(NPASS()):
        st.raw(f"buffer_load_dwordx4 {vst(i, 1)}, {VOFF[i]}, {NX}, 0 offen")


def stage0(st):
    """staging descriptors start at tiles K(2) / V(1); stage 0's loads"""
    t2, t1 = hex(2 * TILEB()), hex(TILEB())
    st.raw(f"s_add_u32 s40, s40, {t2}")
    st.raw(f"s_addc_u32 s41, s41, 0")
    st.raw(f"s_sub_i32 {SKREM}, s42, {t2}")
    st.raw(f"s_max_i32 s42, {SKREM}, 0")
    st.raw(f"s_add_u32 s44, s44, {t1}")
    st.raw(f"s_addc_u32 s45, s45, 0")
    st.raw(f"s_sub_i32 {SVREM}, s46, {t1}")
    st.raw(f"s_max_i32 s46, {SVREM}, 0")
    if dma():
        return  # iteration 0 issues K(2), V(1) by LDS-DMA
    st.nop(4)
    for ins in stage_loads():
        st.emit(ins)


def zero_state(st):
    """O, l, -m_ref, m_ref = 0"""
    for x in list(range(16 * NE())) + list(range(128, 144)):
        st.raw(f"v_accvgpr_write_b32 a{x}, 0")
    for x in range(96, 112):
        st.raw(f"v_mov_b32 v{x}, 0")
    for b in range(4):
        st.raw(f"v_mov_b32 {MREF[b]}, 0")


# fp16 Q * c and O / l rounded ONCE, by mixed-precision fmas into the two
# halves of the packed result (v_fma_mixlo/hi_f16: fma(a, s, -0), the exact
# product rounded straight to fp16, signed zeros kept) -- one VALU per two
# elements fewer than the fp32 product + v_cvt_pk, whose two roundings
# M16::scale_q / store_o use.  Experiment (W4_XP=mix), off: 128 fewer VALU
# per item measured neutral on every shape (headline 1210.8 vs 1213.1,
# S=8192 causal 1365.0 vs 1368.7, short causal W4P -0.6 to -1.3 %;
# profiles/r05_ab_mix.jsonl, 290 W4/W4P/split GPU tests green with it).
# bf16 has no mix form.
MIX_XP = "mix" in XP


def mix():
    return MIX_XP and not DT["bf16"]


def mix_pk(dst, a, b, s, f16src=False):
    """dst = fp16(a s) | fp16(b s) << 16 (f32 a, b; f16src: a = b = the
    packed fp16 pair, low then high half)"""
    if f16src:
        return [valu(f"v_fma_mixlo_f16 {dst}, {a}, {s}, neg(0) op_sel_hi:[1,0,0]", r=[a], w=[dst]),
                valu(f"v_fma_mixhi_f16 {dst}, {b}, {s}, neg(0) op_sel:[1,0,0] op_sel_hi:[1,0,0]",
                     r=[b, dst], w=[dst])]
    return [valu(f"v_fma_mixlo_f16 {dst}, {a}, {s}, neg(0)", r=[a, s], w=[dst]),
            valu(f"v_fma_mixhi_f16 {dst}, {b}, {s}, neg(0)", r=[b, s, dst], w=[dst])]


def q_scale(st):
    """Q * c (fp32 product, rounded to fp16 once: M16::scale_q) from v0-63
    into AGPRs, eight elements at a time in the (free) V^T fragment registers"""
    for x0 in range(0, 16 * NT(), 8):
        xs = range(x0, x0 + 8)
        lo = {x: f"v{144 + 3 * (x - x0)}" for x in xs}
        hi = {x: f"v{145 + 3 * (x - x0)}" for x in xs}
        pk = {x: f"v{146 + 3 * (x - x0)}" for x in xs}
        if "noqscale" in XP:  # timing only (wrong results): Q unscaled, no VALU
            continue
        if mix():
            for x in xs:
                for op in mix_pk(pk[x], f"v{x}", f"v{x}", "%[c]", f16src=True):
                    st.raw(op.text)
            for x in xs:
                st.raw(f"v_accvgpr_write_b32 a{144 + x}, {pk[x]}")
            continue
        if fp32scale():  # Q unscaled: c applies to the fp32 scores
            for x in xs:
                st.raw(f"v_accvgpr_write_b32 a{144 + x}, v{x}")
            continue
        if DT["bf16"]:
            for x in xs:  # bf16 -> fp32 is exact: the 16 bits move to the top half
                st.raw(f"v_lshlrev_b32_e32 {lo[x]}, 16, v{x}")
                st.raw(f"v_and_b32_e32 {hi[x]}, 0xffff0000, v{x}")
            for x in xs:
                st.raw(f"v_mul_f32_e32 {lo[x]}, %[c], {lo[x]}")
                st.raw(f"v_mul_f32_e32 {hi[x]}, %[c], {hi[x]}")
        else:
            # fp16 half * c in one mixed-precision fma: fma(q, c, -0) is the
            # fp32 product rounded once (= cvt + v_mul_f32, signed zeros too)
            for x in xs:
                st.raw(f"v_fma_mix_f32 {lo[x]}, v{x}, %[c], neg(0) op_sel_hi:[1,0,0]")
                st.raw(f"v_fma_mix_f32 {hi[x]}, v{x}, %[c], neg(0) op_sel:[1,0,0] op_sel_hi:[1,0,0]")
        for x in xs:
            st.raw(f"{DT['cvt_pk']} {pk[x]}, {lo[x]}, {hi[x]}")
        for x in xs:
            st.raw(f"v_accvgpr_write_b32 a{144 + x}, {pk[x]}")


def prologue(st, causal, split=False):
    """Q (scaled), K(0), K(1), V(0) into registers / LDS, stage 0 in flight,
    S(0) = K(0) Q^T with the first-tile rescale and exp2.  V(0) and K(1)
    are waited for only after S(0) (their latency under the Q scaling, the
    QK^T and the first softmax).  (Prefetching the next item's Q, K(0), K(1)
    by LDS-DMA during the previous item's last iteration cut this prologue
    from 11.4k to 6.2k cycles at the headline but added as much to the
    loop -- the DMA issue cost -- and was dropped:
    profiles/r03_ab_w4_next_item_dma.jsonl.)"""
    pstamp(st, 60)
    st.raw(f"v_mov_b32 {VNINF}, {NINF}")
    for i in range(4):
        st.raw(f"v_mov_b32 v{208 + i}, {DT['one2']}")
    for i in range(1, 4):
        st.raw(f"v_add_u32 {KOFF[i]}, {4096 * i}, %[koff]")
        st.raw(f"v_add_u32 {VOFF[i]}, {4096 * i}, %[voff]")
    cold, join = newlabel("cold"), newlabel("join")
    st.raw(f"s_cmp_eq_u32 {WARM}, 0")
    st.branch("s_cbranch_scc1", cold)
    # ---- warm: Q, K(0), V(0), K(1) were loaded in the previous item's last
    # iteration
    xovl = XOVL and not split
    stage0(st)
    if xovl:
        # O and l still hold the previous item's result (its deferred
        # epilogue zeroes them); in flight: prefetch (Q 16, K(0) 4, K(1) 4,
        # V(0) 4) then stage 0 (8): Q and K(0) landed at vmcnt(16)
        for x in range(96, 112):
            st.raw(f"v_mov_b32 v{x}, 0")
        for b in range(4):
            st.raw(f"v_mov_b32 {MREF[b]}, 0")
        st.raw(f"s_waitcnt vmcnt({2 * NPASS() + sg0()})")
        if "epiwait16" in XP:
            st.raw(f"s_mov_b32 {PEND}, 1")
    else:
        # (older than the previous item's O stores)
        zero_state(st)
        st.raw(f"s_waitcnt vmcnt({nst() + sg0()})")
    prostamp(st, 0)  # item start -> Q, K(0) landed (warm items)
    st.branch("s_branch", join)
    # ---- cold: the chunk's first item
    st.label(cold)
    if "epiwait16" in XP:
        st.raw(f"s_mov_b32 {PEND}, 0")
    # Q rows qw + 16b + r16: offset (qw + 16b) * 256 + %[qoff]
    st.raw(f"s_lshl_b32 {ST0}, {QW}, {ROWSH()}")
    for b in range(4):
        st.raw(f"v_add_u32 {T[b]}, {ST0}, %[qoff]")
        if b:
            st.raw(f"v_add_u32 {T[b]}, {16 * ROWB() * b}, {T[b]}")
    st.nop(1)
    for b in range(4):
        for t in range(NT()):
            st.raw(f"buffer_load_dwordx4 {R('v', 4 * NT() * b + 4 * t, 4)}, {T[b]}, {RQ}, 0 offen offset:{64 * t}")
    # K(0) -> v112.., then V(0) and K(1) into staging set 1 (a224.., a208..:
    # free until iteration 0's loads), waited for only after S(0)
    for i in range(NPASS()):
        st.raw(f"buffer_load_dwordx4 {R('v', 112 + 4 * i, 4)}, {KOFF[i]}, {SK}, 0 offen")
    for i in range(NPASS()):
        st.raw(f"buffer_load_dwordx4 {vst(i, 1)}, {VOFF[i]}, {SV}, 0 offen")
    for i in range(NPASS()):
        st.raw(f"v_add_u32 {T[4 + i]}, {hex(TILEB())}, {KOFF[i]}")
    st.nop(1)
    for i in range(NPASS()):
        st.raw(f"buffer_load_dwordx4 {kst(i, 1)}, {T[4 + i]}, {SK}, 0 offen")
    stage0(st)
    zero_state(st)
    # Q and K(0) landed (V(0), K(1) and stage 0 may still fly)
    st.raw(f"s_waitcnt vmcnt({2 * NPASS() + sg0()})")
    st.label(join)
    for i in range(NPASS()):
        st.raw(f"ds_write_b128 %[klds], {R('v', 112 + 4 * i, 4)} offset:{KBUF[0] + PASSL() * i}")
    q_scale(st)
    if onebar():
        # V(0), K(1) (prefetched after Q, K(0)) landed under the Q scaling:
        # into their LDS images before the same barrier as K(0) -- the
        # previous item's last barrier freed every image
        st.raw(f"s_waitcnt vmcnt({sg0()})")
        for i in range(NPASS()):
            st.raw(f"ds_write_b128 {vlds()}, {vst(i, 1)} offset:{vbuf(0) + PASSL() * i}")
            st.raw(f"ds_write_b128 %[klds], {kst(i, 1)} offset:{KBUF[1] + PASSL() * i}")
    if dbl():
        # two tiles ahead: K(2), V(1) by LDS-DMA now (the previous item's last
        # barrier freed their images); iteration 0's end waits for them
        for i in range(npiece()):
            st.raw(f"s_add_u32 m0, %[dmab], {kbuf(2) + 1024 * i}")
            st.nop(1)
            st.raw(f"buffer_load_dwordx4 {KD(i)}, {SK}, 0 offen lds")
        for i in range(npiece()):
            st.raw(f"s_add_u32 m0, %[dmab], {vbuf_abs(1) + 1024 * i}")
            st.nop(1)
            st.raw(f"buffer_load_dwordx4 {VD(i)}, {SV}, 0 offen lds")
        tb = hex(TILEB())
        for ins in (f"s_add_u32 s40, s40, {tb}", "s_addc_u32 s41, s41, 0", f"s_sub_i32 {SKREM}, {SKREM}, {tb}",
                    f"s_max_i32 s42, {SKREM}, 0", f"s_add_u32 s44, s44, {tb}", "s_addc_u32 s45, s45, 0",
                    f"s_sub_i32 {SVREM}, {SVREM}, {tb}", f"s_max_i32 s46, {SVREM}, 0"):
            st.raw(ins)
    prostamp(st, 1)  # -> K(0) written, Q scaled
    st.raw("s_waitcnt lgkmcnt(0)")
    st.raw("s_barrier")
    st.nop(2)
    # S(0)
    if xovl:
        cold_s0, s0done = newlabel("colds0"), newlabel("s0done")
        st.raw(f"s_cmp_eq_u32 {WARM}, 0")
        st.branch("s_cbranch_scc1", cold_s0)
        s0_with_epilogue(st)
        st.branch("s_branch", s0done)
        st.label(cold_s0)
        qk_plain(st, KBUF[0])
        st.label(s0done)
    else:
        qk_plain(st, KBUF[0])
    if fp32scale():
        for b in range(4):
            for cb in range(4):
                for ins in scale_ops(b, cb):
                    st.emit(ins)
    prostamp(st, 2)  # -> S(0) (+ the deferred epilogue) done
    st.raw(f"s_cmp_eq_u32 {SMASKJ}, 1")
    skip = newlabel("nomask0")
    st.branch("s_cbranch_scc0", skip)
    st.raw(f"s_sub_i32 {ST0}, {KVHI}, 1")
    st.raw(f"s_mov_b32 {ST1}, {QM}")
    mask_last_tile(st, causal)
    st.label(skip)
    if "nofirst" not in XP:  # timing only (wrong results): no first-tile softmax
        slow_softmax(st, first=True)
        for e in exp_ops():
            st.emit(e)
    prostamp(st, 3)  # -> first softmax + exp2 done
    # V(0), K(1) landed: into their LDS images (warm with the deferred
    # epilogue: its 16 O stores are the youngest, behind stage 0's 8 loads)
    if onebar():
        pass
    elif xovl:
        cw, cd = newlabel("coldw"), newlabel("waitdone")
        st.raw(f"s_cmp_eq_u32 {WARM}, 0")
        st.branch("s_cbranch_scc1", cw)
        st.raw(f"s_waitcnt vmcnt({nst() + sg0()})")
        st.branch("s_branch", cd)
        st.label(cw)
        st.raw(f"s_waitcnt vmcnt({sg0()})")
        st.label(cd)
    else:
        st.raw(f"s_waitcnt vmcnt({sg0()})")
    if not (onebar()):
        for i in range(NPASS()):
            st.raw(f"ds_write_b128 {vlds()}, {vst(i, 1)} offset:{vbuf(0) + PASSL() * i}")
            st.raw(f"ds_write_b128 %[klds], {kst(i, 1)} offset:{KBUF[1] + PASSL() * i}")
        st.raw("s_waitcnt lgkmcnt(0)")
        st.lgkm = []
        st.raw("s_barrier")
    prostamp(st, 4)  # -> V(0), K(1) written, loop start
    pstamp(st, 62)
    if RSA:
        st.raw(f"s_mov_b32 {PEND}, 0")
    st.raw(f"s_mov_b32 {SJ}, 0")
    if DIAG == "stamps":
        for r in range(64, 68):
            st.raw(f"s_mov_b32 s{r}, 0")


def epilogue_ops(split, ro=RO, rowbase=ST1, zero_o=False):
    """O / l -> fp16 rows (M16::store_o: permlane16 swaps, dwordx4 stores, sc1)
    as a list of instructions (strings: raw SALU / padding).
    split: the item is one key piece of its query block -- the normalised
    partial O goes to the workspace slab (%[ro] points there) and the row's
    log2-sum-exp, m_ref + log2(l), to %[rl] (4-B sc1 stores), for the merge.
    zero_o: each O / l register is zeroed right after it is read (the
    deferred epilogue runs inside the next item's prologue, which owns them
    next)."""
    ops = []
    E = ops.append
    if split:
        E(f"s_lshl_b32 s57, {QW}, 2")
        E("s_nop 0")
        E(valu(f"v_lshlrev_b32 {T[9]}, 2, %[r16]", r=["%[r16]"], w=[T[9]]))
        E(valu(f"v_add_u32 {T[9]}, s57, {T[9]}", r=[T[9]], w=[T[9]]))
    for b in range(4):
        l, inv = T[0], T[1]
        E(valu(f"v_accvgpr_read_b32 {l}, {L(b, 0)}", r=[L(b, 0)], w=[l]))
        if zero_o and not mfz():
            for i in range(4):
                E(valu(f"v_accvgpr_write_b32 {L(b, i)}, 0", w=[L(b, i)]))
        # inv = l > 0 ? 1.0f / l : 0  (IEEE division, the compiler's sequence)
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
        if split:
            # log2(l) + m_ref (-inf for an empty row), row qw + 16b + r16
            E(valu(f"v_log_f32_e32 {T[8]}, {l}", r=[l], w=[T[8]], kind="trans"))
            E(valu(f"v_add_f32_e32 {T[8]}, {MREF[b]}, {T[8]}", r=[MREF[b], T[8]], w=[T[8]]))
            E(valu(f"v_add_u32 {T[10]}, {64 * b}, {T[9]}", r=[T[9]], w=[T[10]]))
            E(vmem(f"buffer_store_dword {T[8]}, {T[10]}, {RL}, 0 offen sc1", r=[T[8], T[10]]))
            E("s_nop 1")
        # row offset: (qw + 16b + r16) * 256 + 2 * dlane
        if "epilines" in XP:
            # timing only (wrong layout): each store one contiguous KiB = 8
            # whole 128-B lines of the block's rows, lane-linear
            E(valu(f"v_mbcnt_lo_u32_b32 {T[7]}, -1, 0", w=[T[7]]))
            E(valu(f"v_mbcnt_hi_u32_b32 {T[7]}, -1, {T[7]}", r=[T[7]], w=[T[7]]))
            E(valu(f"v_lshlrev_b32 {T[7]}, 4, {T[7]}", r=[T[7]], w=[T[7]]))
            E(valu(f"v_add_u32 {T[7]}, {rowbase}, {T[7]}", r=[T[7]], w=[T[7]]))
        else:
            E(valu(f"v_add_u32 {T[7]}, {rowbase}, %[ooff]", r=["%[ooff]"], w=[T[7]]))
        if b:
            E(valu(f"v_add_u32 {T[7]}, {16 * ROWB() * b}, {T[7]}", r=[T[7]], w=[T[7]]))
        for ep in range(NE() // 2):
            d = [f"v{144 + i}" for i in range(8)]  # O staging: the (free) V^T fragment slots
            for x in range(2):
                e = 2 * ep + x
                for i in range(4):
                    src = L(b, i) if DIAG == "l" else O(b, e, i)
                    E(valu(f"v_accvgpr_read_b32 {d[4 * x + i]}, {src}", r=[src], w=[d[4 * x + i]]))
                    if zero_o and not mfz():
                        E(valu(f"v_accvgpr_write_b32 {O(b, e, i)}, 0", w=[O(b, e, i)]))
                if DIAG in ("raw", "l") or mix():
                    continue
                for i in range(4):
                    E(valu(f"v_mul_f32_e32 {d[4 * x + i]}, {d[4 * x + i]}, {inv}", r=[d[4 * x + i], inv], w=[d[4 * x + i]]))
            # X = e even pair -> v152,153 ; Y = e odd -> v154,155
            X, Y = ["v152", "v153"], ["v154", "v155"]
            if mix() and DIAG not in ("raw", "l"):
                for k, dst in enumerate(X + Y):
                    for op in mix_pk(dst, d[2 * k], d[2 * k + 1], inv):
                        E(op)
            else:
                E(valu(f"{DT['cvt_pk']} {X[0]}, {d[0]}, {d[1]}", r=d[0:2], w=[X[0]]))
                E(valu(f"{DT['cvt_pk']} {X[1]}, {d[2]}, {d[3]}", r=d[2:4], w=[X[1]]))
                E(valu(f"{DT['cvt_pk']} {Y[0]}, {d[4]}, {d[5]}", r=d[4:6], w=[Y[0]]))
                E(valu(f"{DT['cvt_pk']} {Y[1]}, {d[6]}, {d[7]}", r=d[6:8], w=[Y[1]]))
            for dw in range(2):
                E(valu(f"v_permlane16_swap_b32 {X[dw]}, {Y[dw]}", r=[X[dw], Y[dw]], w=[X[dw], Y[dw]]))
            pol = OPOL if not split else " sc1"
            E(vmem(f"buffer_store_dwordx4 v[152:155], {T[7]}, {ro}, 0 offen "
                   f"offset:{(1024 if 'epilines' in XP else 64) * ep}{pol}",
                   r=["v[152:155]", T[7]]))
            # (no pad: the next write of v[152:155] is the next pair's
            # conversion, 20+ instructions on)
        if zero_o and mfz():
            # this row block's O (and, after the last one, every l) zeroed by
            # 32x32x16 MFMAs of zero operands (v96-99 = 0 here): 16 AGPRs per
            # instruction on the otherwise idle matrix pipe
            for z in range(0, 4 * NE(), 16):
                E(zero_mfma(4 * NE() * b + z))
            if b == 3:
                E(zero_mfma(128))
    E("s_nop 1")
    return ops


def zero_mfma(a0):
    """a[a0:a0+15] = 0 by one 32x32x16 MFMA (A = B = v[96:99] = 0, C = 0)"""
    op = "v_mfma_f32_32x32x16_" + ("bf16" if DT["bf16"] else "f16")
    return Ins(f"{op} a[{a0}:{a0 + 15}], v[96:99], v[96:99], 0", "mfma",
               r=["v[96:99]"], w=[f"a[{a0}:{a0 + 15}]"])


def epilogue(st, split):
    for op in epilogue_ops(split):
        st.emit(op)


def s0_with_epilogue(st):
    """S(0) = K(0) Q^T (qk_plain's chains) with the previous item's deferred
    epilogue (zeroing O and l behind itself) spread over the MFMA gaps"""
    kb = KBUF[0]
    mf, gaps = [], {}
    for cb in range(4):
        for b in range(4):
            mf += qk_chain(b, cb, [kslot(cb, t) for t in range(NT())])
    gaps[0] = [k_read(t, 0, t, kb) for t in range(NT())]
    for cb in range(3):
        for t in range(NT()):
            gaps.setdefault(4 * NT() * cb + 1 + t, []).append(k_read(t, cb + 1, kslot(cb + 1, t), kb))
    ops = epilogue_ops(False, ro=ROSAVE, rowbase=ROWSAVE, zero_o=True)
    if "noepi" in XP:  # timing only (wrong results): no deferred epilogue at all
        ops = []
    # timing only (wrong results): the epilogue without its O stores / with
    # only its O, l zeroing / without the zeroing
    if "epinostore" in XP:
        ops = [o for o in ops if isinstance(o, str) or not o.text.startswith("buffer_store")]
    if "epizonly" in XP:
        ops = [o for o in ops if isinstance(o, Ins) and o.text.startswith("v_accvgpr_write")]
    if "epinozero" in XP:
        ops = [o for o in ops if isinstance(o, str) or not o.text.startswith("v_accvgpr_write")]
    n = len(mf)
    for i, op in enumerate(ops):
        gaps.setdefault((i * n) // len(ops), []).append(op)
    st.interleave(mf, gaps)


def generate(causal, split=False):
    CUR["split"] = split
    st = Stream()
    nb = nbuf()
    labels = {k: [newlabel(f"{k}{p}") for p in range(nb)]
              for k in ("loop", "notsteady", "masked", "general", "slow", "slow2", "slow3", "end",
                        "single", "dmid", "dend", "dslow1", "dslow2")}
    labels["last"] = [newlabel(f"last{p}") for p in range(nb)]
    labels["end_nowait"] = [newlabel(f"endnw{p}") for p in range(nb)]
    labels["done"] = newlabel("done")
    item = newlabel("item")
    # the workgroup's items (a chunk of fa_w4_kernel.hpp's table) in one
    # statement, so the next item's operands can be loaded in this one's
    # last iteration
    # code-placement experiment (MI355X_MICROARCH.md, two waves per SIMD,
    # item 8): W4_XP=shiftN moves the whole program by N bytes
    for x in XP:
        if x.startswith("shift"):
            for _ in range(int(x[5:]) // 4):
                st.raw("s_nop 0")
    st.raw(f"s_mov_b32 {ITEM}, 0")
    st.raw(f"s_mov_b32 {WARM}, 0")
    if dma():
        dma_setup(st)
    if dbl():
        st.raw("v_add_u32 v188, 0x10000, %[va0]")
        st.raw("v_add_u32 v189, 0x10000, %[va1]")
        st.raw("v_add_u32 v190, 0x10000, %[vlds]")
    if DIAG == "prostamps":
        for r in range(200, 208):
            st.raw(f"v_mov_b32 v{r}, 0")
    st.label(item)
    prostamp(st, -1)
    if DIAG == "prostamps":
        st.raw("v_add_u32 v206, 1, v206")
    read_item(st, causal)
    prologue(st, causal, split)
    for p in range(nb):
        body(st, p, causal, labels)
    st.label(labels["done"], drain_lgkm=True)
    prostamp(st, 5)  # loop (every iteration incl. the last one's prefetch)
    pstamp(st, 64)
    if XOVL and not split:
        # a successor follows: defer this item's epilogue into its prologue
        last = newlabel("lastepi")
        st.raw(f"s_add_u32 {ST0}, {ITEM}, 1")
        st.raw(f"s_cmp_lt_u32 {ST0}, %[nitems]")
        st.branch("s_cbranch_scc0", last)
        for i in range(4):
            st.raw(f"s_mov_b32 s{60 + i}, s{76 + i}")
        st.raw(f"s_lshl_b32 {ROWSAVE}, {QW}, {ROWSH()}")
        st.raw(f"s_mov_b32 {ITEM}, {ST0}")
        if dbl():
            st.far("s_branch", item)
            st.dead = False  # (the label below is reached by its own branch)
        else:
            st.raw(f"s_branch {item}")
        st.label(last)
    # ST1 = qw * row bytes: the epilogue's row base
    st.raw(f"s_lshl_b32 {ST1}, {QW}, {ROWSH()}")
    st.nop(1)
    epilogue(st, split)
    if DIAG == "pstamps":
        # [prologue, loop, epilogue issue, store drain] cycles of this wave's
        # item, in O[qw][0:8] (every lane the same 16 bytes)
        pstamp(st, 66)
        st.raw("s_waitcnt vmcnt(0)")
        pstamp(st, 68)
        for i, (a, b) in enumerate(((62, 60), (64, 62), (66, 64), (68, 66))):
            st.raw(f"s_sub_u32 s57, s{a}, s{b}")
            st.raw(f"v_mov_b32 v{120 + i}, s57")
        st.raw(f"v_mov_b32 v124, s{ST1[1:]}")
        st.nop(2)
        st.raw(f"buffer_store_dwordx4 v[120:123], v124, {RO}, 0 offen")
        st.nop(2)
    if DIAG == "prostamps":
        # the wave's sums over its items: [Q wait, q_scale, S(0) + deferred
        # epilogue, first softmax, V(0)/K(1) writes, loop] + items, in
        # O[qw][0:16] of the chunk's last item
        st.raw("s_waitcnt vmcnt(0)")
        st.raw(f"v_mov_b32 v199, s{ST1[1:]}")
        st.nop(2)
        st.raw(f"buffer_store_dwordx4 v[200:203], v199, {RO}, 0 offen")
        st.raw(f"buffer_store_dwordx4 v[204:207], v199, {RO}, 0 offen offset:16")
        st.nop(2)
    if DIAG == "stamps":
        # [phase A, phase B, barrier (wait + skew), steady iterations] of
        # this wave, in O[qw][0:8] (every lane the same 16 bytes)
        for i, r in enumerate(range(64, 68)):
            st.raw(f"v_mov_b32 v{120 + i}, s{r}")
        st.raw(f"v_mov_b32 v124, s{ST1[1:]}")
        st.nop(2)
        st.raw(f"buffer_store_dwordx4 v[120:123], v124, {RO}, 0 offen")
        st.nop(2)
    st.raw(f"s_add_u32 {ITEM}, {ITEM}, 1")
    st.raw(f"s_cmp_lt_u32 {ITEM}, %[nitems]")
    st.jump("s_cbranch_scc1", item)
    if dma():
        st.raw(f"s_mov_b32 m0, {SM0}")
    CUR["split"] = False
    return st.out


HEADER = """// GENERATED by gen_w4_item.py -- do not edit.
// One item (256 query rows x all key tiles) of the one-wave-per-SIMD kernel:
// see the generator's docstring for the register map and the schedule.
#pragma once
"""


def header():
    # the head_dim-128 persistent programs' LDS layout (fa_w4_kernel.hpp):
    # 1 = four K / V images per tensor and the item table at 128 KiB (dbl)
    return HEADER + f"#define FA_W4_DBL {1 if DBL_XP and DMA_ON else 0}\n"


def cxx(causal, bf16, lines, split=False):
    body = "\n".join(f'      "{l}\\n"' for l in lines)
    vclob = ", ".join(f'"v{i}"' for i in range(236))
    aclob = ", ".join(f'"a{i}"' for i in range(240 if STAGE2 else 208))
    sclob = ", ".join(f'"s{i}"' for i in range(40, 98))
    dma_ops = (',\n        [kdma] "v"(ln.kdma), [vdma] "v"(ln.vdma), [dmab] "s"(rn.dmab)' if dma() else "")
    name = (("w4_item_causal" if causal else "w4_item_noncausal") + ("_split" if split else "")
            + ("_d64" if HDC["hd"] == 64 else "") + ("_bf16" if bf16 else "_f16"))
    return f"""
__device__ __forceinline__ void {name}(const W4Run& rn, const W4Lane& ln) {{
  asm volatile(
{body}
      :
      : [tab] "s"(rn.tab), [nitems] "s"(rn.nitems), [woff] "s"(rn.woff), [qrec] "s"(rn.qrec),
        [c] "s"(rn.c),
        [ka0] "v"(ln.ka[0]), [ka1] "v"(ln.ka[1]), [ka2] "v"(ln.ka[2]), [ka3] "v"(ln.ka[3]),
        [va0] "v"(ln.va[0]), [va1] "v"(ln.va[1]), [koff] "v"(ln.koff), [voff] "v"(ln.voff),
        [klds] "v"(ln.klds), [vlds] "v"(ln.vlds), [vt] "v"(ln.vt), [r16] "v"(ln.r16),
        [qoff] "v"(ln.qoff), [ooff] "v"(ln.ooff){dma_ops}
      : "memory", "vcc", "scc", {sclob},
        {vclob},
        {aclob});
}}
"""


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "fa_w4_item.inc"
    text = header()
    for bf16 in (False, True):
        set_dtype(bf16)
        for causal in (False, True):
            _lbl[0] = 0
            text += cxx(causal, bf16, generate(causal))
        # one key piece of a causal query block (fa_w4_kernel.hpp: split tier)
        _lbl[0] = 0
        text += cxx(True, bf16, generate(True, split=True), split=True)
    # head_dim 64 (non-split)
    set_hd(64)
    for bf16 in (False, True):
        set_dtype(bf16)
        for causal in (False, True):
            _lbl[0] = 0
            text += cxx(causal, bf16, generate(causal))
    set_hd(128)
    with open(out, "w") as f:
        f.write(text)


if __name__ == "__main__":
    main()
