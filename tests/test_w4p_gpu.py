"""Multi-block short-sequence tier (bm128_bn64_w4x32_m16_asm_pair_*: two 64-row
query blocks per workgroup, bm256_bn64_w4x64_m16_asm_quad_*: four,
bm64_bn64_w4x16_m16_asm_single_*: one, on the pair program;
fa_w4p_kernel.hpp + the generated item program fa_w4p_item.inc).

A workgroup holds two or four 64-row query blocks of one head (causal: pairs
of the heavy block nqb-1-r with the light block r) on one shared K/V stream,
16 rows of each per wave.  Its rescale decision is per 16-row block (the 8-wave kernels
take it per 32-row wave), so outputs are compared with the oracle (the
reference's cpu_attention restatement) on sampled heads and with an fp32
torch attention on every head, both at the 1e-3 gate; bf16 against the fp32
torch reference at 5e-3 (no reference oracle exists for bf16).
"""
import math

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import oracle  # noqa: E402  (test infrastructure)

pytestmark = pytest.mark.gpu
TOL = 1e-3
PAIR = "bm128_bn64_w4x32_m16_asm_pair"
QUAD = "bm256_bn64_w4x64_m16_asm_quad"
SINGLE = "bm64_bn64_w4x16_m16_asm_single"


def _fa():
    import fa_mi355x

    return fa_mi355x


def _ids(prefix):
    out = {c.causal: c.id for c in _fa().configs() if c.name in (f"{prefix}_noncausal", f"{prefix}_causal")}
    assert set(out) == {False, True}, prefix
    return out


def _rand(shape, seed, scale=1.0, dtype=torch.float16):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    t = torch.empty(shape, dtype=torch.float32, device="cuda")
    t.uniform_(-0.5 * scale, 0.5 * scale, generator=g)
    return t.to(dtype)


def _bits(t):
    return t.detach().cpu().contiguous().view(torch.int16).numpy().view(np.uint16)


def _torch_ref(q, k, v, causal):
    """fp32 attention of the 16-bit inputs, head by head (bounded memory)"""
    b, h, s, d = q.shape
    out = torch.empty((b, h, s, d), dtype=torch.float32, device=q.device)
    mask = torch.ones((s, s), dtype=torch.bool, device=q.device).tril() if causal else None
    for bi in range(b):
        for hi in range(h):
            sc = (q[bi, hi].float() @ k[bi, hi].float().t()) / math.sqrt(d)
            if causal:
                sc = sc.masked_fill(~mask, float("-inf"))
            out[bi, hi] = torch.softmax(sc, dim=-1) @ v[bi, hi].float()
    return out


def _check(b, h, s, causal, seed, scale=1.0, dtype=torch.float16, oracle_heads=True, tier=PAIR, d=128):
    fa = _fa()
    pre = ("d64_" if d == 64 else "") + tier
    pre = pre if dtype == torch.float16 else "bf16_" + pre
    q, k, v = (_rand((b, h, s, d), seed + i, scale if i < 2 else 1.0, dtype) for i in range(3))
    out = fa.flash_attention_fwd(q, k, v, causal=causal, config=_ids(pre)[causal])
    torch.cuda.synchronize()
    assert torch.isfinite(out.float()).all()
    ref = _torch_ref(q, k, v, causal)
    d = (out.float() - ref).abs().max().item()
    tol = TOL if dtype == torch.float16 else 5e-3
    assert d <= tol, f"max diff vs fp32 torch {d}"
    if oracle_heads and dtype == torch.float16:
        for flat in sorted({0, b * h // 2, b * h - 1}):
            bi, hi = divmod(flat, h)
            sl = (slice(bi, bi + 1), slice(hi, hi + 1))
            ro = oracle.attention(*(_bits(x[sl]) for x in (q, k, v)), causal)
            dd = oracle.max_abs_diff(_bits(out[sl]), ro)
            assert dd <= TOL, f"head {flat}: max_diff vs oracle {dd}"
    return d


SHAPES = [
    (1, 32, 1024),   # BASELINE config 1: 256 pairs, one per CU
    (1, 8, 1000),    # ragged S: the last block 40 rows, its last tile 40 keys
    (2, 3, 320),     # 5 query blocks (odd: the middle one unpaired), 6 heads (not % 8)
    (1, 4, 64),      # one block per head: single-tile items
    (1, 2, 65),      # two blocks, the second 1 row
    (1, 1, 130),     # three blocks, one head
    (1, 16, 2048),   # 512 pairs: two rounds of workgroups
    (3, 40, 777),    # 120 heads, ragged
    (1, 8, 256),     # 4 blocks: pairs (3, 0), (2, 1)
    (4, 32, 512),
]


TIERS = [PAIR, QUAD, SINGLE]
TIER_IDS = ["pair", "quad", "single"]


@pytest.mark.parametrize("tier", TIERS, ids=TIER_IDS)
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_pair_matches_oracle(shape, causal, tier):
    _check(*shape, causal, seed=700, tier=tier)


@pytest.mark.parametrize("tier", TIERS, ids=TIER_IDS)
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("s", [256, 1000, 2048])
def test_pair_peaked_rescale(s, causal, tier):
    # Q, K x4: row maxima keep growing past the 2^8 threshold -> the slow paths
    _check(1, 8, s, causal, seed=710, scale=4.0, tier=tier)


def _random_shapes(n, seed):
    rng = np.random.default_rng(seed)
    return [(int(rng.integers(1, 3)), int(rng.integers(1, 41)), int(rng.integers(1, 2049)))
            for _ in range(n)]


@pytest.mark.parametrize("tier", TIERS, ids=TIER_IDS)
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("shape", _random_shapes(6, 2027), ids=lambda s: "x".join(map(str, s)))
def test_pair_random_shapes(shape, causal, tier):
    _check(*shape, causal, seed=720, tier=tier)


@pytest.mark.parametrize("tier", TIERS, ids=TIER_IDS)
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("shape", [(1, 32, 1024), (1, 8, 1000), (2, 3, 320)], ids=lambda s: "x".join(map(str, s)))
def test_pair_bf16(shape, causal, tier):
    _check(*shape, causal, seed=730, dtype=torch.bfloat16, tier=tier)


def _sample_rows(s, n=12):
    rng = np.random.default_rng(s)
    return sorted({0, 63, 64, s // 2, s - 64, s - 1} | set(int(x) for x in rng.integers(0, s, n)))


@pytest.mark.parametrize("b,h,s,causal", [(1, 8, 4096, True), (1, 8, 4096, False), (2, 8, 2048, True),
                                           (1, 4, 8192, False), (1, 1, 32768, False)])
def test_pair_long_heads(b, h, s, causal):
    """the dispatcher's long few-head shapes (one round of pairs): sampled rows
    of every head against an fp32 torch reference of those rows, head 0's
    against the oracle's row-sampled entry"""
    fa = _fa()
    assert "_asm_pair_" in fa.configs()[fa.select_config(b, h, s, causal)].name
    q, k, v = (_rand((b, h, s, 128), 760 + i) for i in range(3))
    out = fa.flash_attention_fwd(q, k, v, causal=causal)
    torch.cuda.synchronize()
    rows = _sample_rows(s)
    r = torch.tensor(rows, device=q.device)
    for bi in range(b):
        sc = q[bi][:, r].float() @ k[bi].float().transpose(-1, -2) / math.sqrt(128)
        if causal:
            keep = torch.arange(s, device=q.device)[None, :] <= r[:, None]
            sc = sc.masked_fill(~keep, float("-inf"))
        ref = torch.softmax(sc, dim=-1) @ v[bi].float()
        err = (out[bi][:, r].float() - ref).abs().max().item()
        assert err <= TOL, f"batch {bi}: max err {err}"
    ro = oracle.attention_rows(_bits(q[0, 0]), _bits(k[0, 0]), _bits(v[0, 0]), rows, causal)
    assert oracle.max_abs_diff(_bits(out[0, 0])[rows], ro) <= TOL


def test_pair_causal_row0_and_ones():
    """causal row 0 sees key 0 only: O[0] = V[0] exactly; V = 1 -> O = 1"""
    fa = _fa()
    q, k = (_rand((1, 4, 1024, 128), 740 + i) for i in range(2))
    v = _rand((1, 4, 1024, 128), 742)
    out = fa.flash_attention_fwd(q, k, v, causal=True, config=_ids(PAIR)[True])
    assert torch.equal(out[:, :, 0], v[:, :, 0])
    ones = torch.ones_like(v)
    for causal in (False, True):
        o1 = fa.flash_attention_fwd(q, k, ones, causal=causal, config=_ids(PAIR)[causal])
        assert torch.equal(o1, ones)


@pytest.mark.parametrize("tier", TIERS, ids=TIER_IDS)
def test_pair_deterministic(tier):
    fa = _fa()
    q, k, v = (_rand((1, 32, 1024, 128), 750 + i) for i in range(3))
    a = fa.flash_attention_fwd(q, k, v, causal=True, config=_ids(tier)[True])
    b = fa.flash_attention_fwd(q, k, v, causal=True, config=_ids(tier)[True])
    assert torch.equal(a, b)


def test_quad_matches_pair_causal_row0_and_ones():
    """the quad grouping: causal row 0 = V[0], V = 1 -> O = 1, and within the
    1e-3 gate of the pair grouping (same arithmetic per block)"""
    fa = _fa()
    q, k, v = (_rand((1, 8, 2048, 128), 770 + i) for i in range(3))
    a = fa.flash_attention_fwd(q, k, v, causal=True, config=_ids(QUAD)[True])
    b = fa.flash_attention_fwd(q, k, v, causal=True, config=_ids(PAIR)[True])
    assert torch.equal(a[:, :, 0], v[:, :, 0])
    assert (a.float() - b.float()).abs().max().item() <= TOL
    ones = torch.ones_like(v)
    o1 = fa.flash_attention_fwd(q, k, ones, causal=True, config=_ids(QUAD)[True])
    assert torch.equal(o1, ones)


# head_dim 64 (configs 56-63: the generator's set_hd(64) -- QK^T chains of two
# k-steps, four O^T column blocks, the whole tile's K fragments read at once,
# two 1-KiB LDS-DMA pieces per wave and tensor into W4's packed 128-B-row
# images)
D64_SHAPES = [(1, 32, 1024), (1, 8, 1000), (2, 3, 320), (1, 4, 64), (1, 2, 65), (1, 1, 130),
              (1, 16, 2048), (3, 40, 777), (4, 32, 512)]


@pytest.mark.parametrize("tier", TIERS, ids=TIER_IDS)
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("shape", D64_SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_pair_d64_matches_oracle(shape, causal, tier):
    _check(*shape, causal, seed=800, tier=tier, d=64)


@pytest.mark.parametrize("tier", TIERS, ids=TIER_IDS)
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("s", [256, 1000, 2048])
def test_pair_d64_peaked_rescale(s, causal, tier):
    _check(1, 8, s, causal, seed=810, scale=4.0, tier=tier, d=64)


@pytest.mark.parametrize("tier", TIERS, ids=TIER_IDS)
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("shape", [(1, 32, 1024), (1, 8, 1000), (2, 3, 320)], ids=lambda s: "x".join(map(str, s)))
def test_pair_d64_bf16(shape, causal, tier):
    _check(*shape, causal, seed=830, dtype=torch.bfloat16, tier=tier, d=64)


@pytest.mark.parametrize("d", [128, 64])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["fp16", "bf16"])
@pytest.mark.parametrize("causal", [False, True])
def test_single_matches_pair_bitwise(causal, dtype, d):
    """one block per workgroup runs the pair program with block 1 absent: every
    block's arithmetic is the pair grouping's (the rescale test per 16-row
    block), so the outputs are bit-identical"""
    fa = _fa()
    pre = ("bf16_" if dtype == torch.bfloat16 else "") + ("d64_" if d == 64 else "")
    for b, h, s in ((1, 32, 512), (2, 3, 1000), (1, 5, 513), (1, 2, 64)):
        q, k, v = (_rand((b, h, s, d), 880 + i, 4.0 if i < 2 else 1.0, dtype) for i in range(3))
        a = fa.flash_attention_fwd(q, k, v, causal=causal, config=_ids(pre + SINGLE)[causal])
        p = fa.flash_attention_fwd(q, k, v, causal=causal, config=_ids(pre + PAIR)[causal])
        assert torch.equal(a, p), (b, h, s)


@pytest.mark.parametrize("b,h,s", [(1, 32, 512), (1, 32, 256), (1, 16, 1024), (1, 8, 2048), (1, 4, 4096),
                                   (2, 16, 512), (1, 64, 256), (4, 32, 128), (1, 3, 1), (2, 5, 100)])
def test_single_dispatched(b, h, s):
    """launches of at most one 64-row block per CU (heads of <= 64 blocks) run
    the single grouping, both masks: against fp32 torch on every head"""
    fa = _fa()
    for causal in (False, True):
        assert "_asm_single_" in fa.configs()[fa.select_config(b, h, s, causal)].name, (b, h, s, causal)
        q, k, v = (_rand((b, h, s, 128), 890 + i) for i in range(3))
        out = fa.flash_attention_fwd(q, k, v, causal=causal)
        torch.cuda.synchronize()
        assert (out.float() - _torch_ref(q, k, v, causal)).abs().max().item() <= TOL


MIXED = "bm64_bn64_w4x16_m16_asm_mixed_causal"


@pytest.mark.parametrize("d", [128, 64])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["fp16", "bf16"])
def test_mixed_matches_pair_bitwise(dtype, d):
    """causal launches of one to two blocks per CU: the heaviest blocks alone,
    the rest paired (the pair program either way): bit-identical to the pairs"""
    fa = _fa()
    pre = ("bf16_" if dtype == torch.bfloat16 else "") + ("d64_" if d == 64 else "")
    mixed = next(c.id for c in fa.configs() if c.name == pre + MIXED)
    for b, h, s in ((1, 32, 768), (1, 24, 1000), (2, 3, 1000), (1, 5, 513), (1, 1, 4095), (1, 32, 1024)):
        q, k, v = (_rand((b, h, s, d), 900 + i, 4.0 if i < 2 else 1.0, dtype) for i in range(3))
        a = fa.flash_attention_fwd(q, k, v, causal=True, config=mixed)
        p = fa.flash_attention_fwd(q, k, v, causal=True, config=_ids(pre + PAIR)[True])
        assert torch.equal(a, p), (b, h, s)


@pytest.mark.parametrize("b,h,s", [(1, 32, 768), (1, 24, 1024), (3, 8, 1024), (1, 12, 2048), (1, 32, 640),
                                   (1, 9, 2000)])
def test_mixed_dispatched(b, h, s):
    """the dispatched mixed grouping against fp32 torch on every head and the
    oracle on sampled heads"""
    fa = _fa()
    assert "_asm_mixed_" in fa.configs()[fa.select_config(b, h, s, True)].name, (b, h, s)
    q, k, v = (_rand((b, h, s, 128), 910 + i) for i in range(3))
    out = fa.flash_attention_fwd(q, k, v, causal=True)
    torch.cuda.synchronize()
    assert (out.float() - _torch_ref(q, k, v, True)).abs().max().item() <= TOL
    for flat in sorted({0, b * h - 1}):
        bi, hi = divmod(flat, h)
        sl = (slice(bi, bi + 1), slice(hi, hi + 1))
        ro = oracle.attention(*(_bits(x[sl]) for x in (q, k, v)), True)
        assert oracle.max_abs_diff(_bits(out[sl]), ro) <= TOL


PLANNED = "bm64_bn64_w4x16_m16_asm_planned_causal"


@pytest.mark.parametrize("d", [128, 64])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16], ids=["fp16", "bf16"])
def test_planned_matches_pair_bitwise(dtype, d):
    """causal launches of two to four blocks per CU short of whole quads:
    groups of one to four blocks planned on the host, each on the two- or the
    four-block program -- every block's arithmetic is the pairs', bit for bit"""
    fa = _fa()
    pre = ("bf16_" if dtype == torch.bfloat16 else "") + ("d64_" if d == 64 else "")
    planned = next(c.id for c in fa.configs() if c.name == pre + PLANNED)
    for b, h, s in ((1, 32, 1536), (1, 25, 2048), (2, 3, 1000), (1, 16, 3000), (1, 32, 1280), (1, 1, 4096)):
        q, k, v = (_rand((b, h, s, d), 920 + i, 4.0 if i < 2 else 1.0, dtype) for i in range(3))
        a = fa.flash_attention_fwd(q, k, v, causal=True, config=planned)
        p = fa.flash_attention_fwd(q, k, v, causal=True, config=_ids(pre + PAIR)[True])
        assert torch.equal(a, p), (b, h, s)


@pytest.mark.parametrize("b,h,s", [(1, 32, 1280), (1, 32, 1536), (1, 16, 2560), (1, 25, 2048), (1, 13, 3500)])
def test_planned_dispatched(b, h, s):
    """the dispatched planned grouping against fp32 torch on every head and
    the oracle on sampled heads"""
    fa = _fa()
    assert "_asm_planned_" in fa.configs()[fa.select_config(b, h, s, True)].name, (b, h, s)
    q, k, v = (_rand((b, h, s, 128), 930 + i) for i in range(3))
    out = fa.flash_attention_fwd(q, k, v, causal=True)
    torch.cuda.synchronize()
    assert (out.float() - _torch_ref(q, k, v, True)).abs().max().item() <= TOL
    for flat in sorted({0, b * h - 1}):
        bi, hi = divmod(flat, h)
        sl = (slice(bi, bi + 1), slice(hi, hi + 1))
        ro = oracle.attention(*(_bits(x[sl]) for x in (q, k, v)), True)
        assert oracle.max_abs_diff(_bits(out[sl]), ro) <= TOL


def test_pair_d64_row0_ones_deterministic():
    fa = _fa()
    q, k, v = (_rand((1, 8, 2048, 64), 840 + i) for i in range(3))
    for tier in TIERS:
        ids = _ids("d64_" + tier)
        a = fa.flash_attention_fwd(q, k, v, causal=True, config=ids[True])
        b = fa.flash_attention_fwd(q, k, v, causal=True, config=ids[True])
        assert torch.equal(a, b)
        assert torch.equal(a[:, :, 0], v[:, :, 0])
        ones = torch.ones_like(v)
        for causal in (False, True):
            assert torch.equal(fa.flash_attention_fwd(q, k, ones, causal=causal, config=ids[causal]), ones)


@pytest.mark.parametrize("b,h,s,tier", [(1, 8, 4096, "pair"), (1, 16, 4096, "quad"), (2, 32, 1024, "quad")])
def test_pair_d64_dispatched_long_heads(b, h, s, tier):
    """head_dim-64 causal launches the dispatcher sends to the W4P twins:
    sampled rows of every head against fp32 torch, head 0's against the
    oracle's row-sampled entry"""
    fa = _fa()
    q, k, v = (_rand((b, h, s, 64), 860 + i) for i in range(3))
    out = fa.flash_attention_fwd(q, k, v, causal=True)
    torch.cuda.synchronize()
    rows = _sample_rows(s)
    r = torch.tensor(rows, device=q.device)
    for bi in range(b):
        sc = q[bi][:, r].float() @ k[bi].float().transpose(-1, -2) / math.sqrt(64)
        keep = torch.arange(s, device=q.device)[None, :] <= r[:, None]
        sc = sc.masked_fill(~keep, float("-inf"))
        ref = torch.softmax(sc, dim=-1) @ v[bi].float()
        assert (out[bi][:, r].float() - ref).abs().max().item() <= TOL
    ro = oracle.attention_rows(_bits(q[0, 0]), _bits(k[0, 0]), _bits(v[0, 0]), rows, True)
    assert oracle.max_abs_diff(_bits(out[0, 0])[rows], ro) <= TOL
    # the launch ran the paired tier's d64 twin (the dispatcher's d128 tier name)
    name = fa.configs()[fa.select_config(b, h, s, True)].name
    assert f"_asm_{tier}_" in name, name
