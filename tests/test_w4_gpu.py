"""One-wave-per-SIMD persistent kernel (bm256_bn64_w4x64_m16_asm_persistent_*,
fa_w4_kernel.hpp + the generated item program fa_w4_item.inc).

Its arithmetic is the 8-wave kernels' operation for operation, with the
rescale decision taken per 32-row half as the ping-pong's 32-row waves take
it, so against the per-item ping-pong (bm256_bn64_w8_m16_pingpong_*) every
score, P and O accumulator is identical; only the final fp32 -> fp16
rounding of O may differ (the compiler builds some of the ping-pong's
roundings as one fused v_fma_mix, the asm rounds the fp32 product), at most
one fp16 ulp on rare elements.  Sampled heads are checked against the oracle
(reference cpu_attention restatement) at the 1e-3 gate, on the shapes that
stress the item order, ragged tiles, the causal diagonal and the rare rescale
branch (peaked scores).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import oracle  # noqa: E402  (test infrastructure)

pytestmark = pytest.mark.gpu
TOL = 1e-3


def _fa():
    import fa_mi355x

    return fa_mi355x


def _rand(shape, seed, scale=1.0):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    t = torch.empty(shape, dtype=torch.float16, device="cuda")
    t.uniform_(-0.5 * scale, 0.5 * scale, generator=g)
    return t


def _bits(t):
    return t.detach().cpu().contiguous().view(torch.int16).numpy().view(np.uint16)


def _ids(prefix):
    """{causal: config id} of the tier named prefix (fp16, or bf16 with a bf16_ prefix)."""
    out = {c.causal: c.id for c in _fa().configs() if c.name in (f"{prefix}_noncausal", f"{prefix}_causal")}
    assert set(out) == {False, True}, prefix
    return out


W4 = "bm256_bn64_w4x64_m16_asm_persistent"
BASE = "bm256_bn64_w8_m16_pingpong"

SHAPES = [
    (1, 8, 512),     # 2 items per head
    (2, 64, 2048),   # 16 query blocks x 128 heads: 4+ items per workgroup
    (3, 40, 1000),   # ragged S (last tile 40 keys), 120 heads
    (1, 203, 300),   # odd head count, 2 query blocks, the last one mostly past S
    (4, 50, 64),     # single-tile items
    (1, 7, 4096),    # fewer heads than XCD groups (non-affine item split)
    (1, 2, 4096),
    (1, 32, 2048),   # causal pair order
    (1, 16, 1280),   # odd query-block count: snake
    (1, 72, 1024),   # > 64 heads: band-16 snake
    (1, 4, 77),      # tiny ragged
]


def _compare(b, h, s, causal, seed, scale=1.0, oracle_heads=True, d=128, w4=W4, base_tier=BASE,
             max_frac=2e-3):
    fa = _fa()
    q, k, v = (_rand((b, h, s, d), seed + i, scale if i < 2 else 1.0) for i in range(3))
    base = fa.flash_attention_fwd(q, k, v, causal=causal, config=_ids(base_tier)[causal])
    out = fa.flash_attention_fwd(q, k, v, causal=causal, config=_ids(w4)[causal])
    torch.cuda.synchronize()
    assert torch.isfinite(out.float()).all()
    diff = (out.float() - base.float()).abs()
    assert diff.max().item() <= TOL, f"max diff vs ping-pong {diff.max().item()}"
    frac = (out != base).float().mean().item()
    if max_frac is not None:
        assert frac <= max_frac, f"{frac:.2e} of the elements differ from the ping-pong"
    if oracle_heads:
        for flat in sorted({0, b * h // 2, b * h - 1}):
            bi, hi = divmod(flat, h)
            sl = (slice(bi, bi + 1), slice(hi, hi + 1))
            ref = oracle.attention(*(_bits(x[sl]) for x in (q, k, v)), causal)
            d = oracle.max_abs_diff(_bits(out[sl]), ref)
            assert d <= TOL, f"head {flat}: max_diff={d}"
    return frac


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_w4_matches_pingpong_and_oracle(shape, causal):
    _compare(*shape, causal, seed=500)


def _random_shapes(n, seed):
    """seeded (batch, heads, seq) draws: ragged seq (any residue mod 64),
    1-48 heads, 1-3 batches -- item tables, tails and diagonals the fixed
    list does not hit"""
    rng = np.random.default_rng(seed)
    return [(int(rng.integers(1, 4)), int(rng.integers(1, 49)), int(rng.integers(65, 2049)))
            for _ in range(n)]


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("shape", _random_shapes(6, 2026), ids=lambda s: "x".join(map(str, s)))
def test_w4_random_shapes(shape, causal):
    _compare(*shape, causal, seed=900)


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("s", [256, 1000, 2048])
def test_w4_peaked_rescale(s, causal):
    # Q, K x4: row maxima keep growing past the 2^8 threshold -> the slow path
    _compare(1, 8, s, causal, seed=600, scale=4.0)


def test_w4_causal_row0_and_ones():
    fa = _fa()
    b, h, s = 1, 4, 1024
    q, k, v = (_rand((b, h, s, 128), 700 + i) for i in range(3))
    o = fa.flash_attention_fwd(q, k, v, causal=True, config=_ids(W4)[True])
    torch.cuda.synchronize()
    assert torch.equal(o[:, :, 0], v[:, :, 0])  # row 0 sees key 0 only
    ones = torch.ones_like(v)
    o1 = fa.flash_attention_fwd(q, k, ones, causal=False, config=_ids(W4)[False])
    torch.cuda.synchronize()
    assert torch.equal(o1, ones)


def test_w4_deterministic():
    fa = _fa()
    q, k, v = (_rand((2, 16, 1536, 128), 800 + i) for i in range(3))
    a = fa.flash_attention_fwd(q, k, v, causal=True, config=_ids(W4)[True])
    b = fa.flash_attention_fwd(q, k, v, causal=True, config=_ids(W4)[True])
    torch.cuda.synchronize()
    assert torch.equal(a, b)


BF16_W4 = "bf16_" + W4
BF16_BASE = "bf16_bm256_bn64_w8_m16_pingpong_persistent"


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("shape", [(1, 8, 512), (3, 40, 1000), (1, 72, 1024), (1, 4, 77)],
                         ids=lambda s: "x".join(map(str, s)))
def test_w4_bf16_matches_pingpong(shape, causal):
    """bf16 twin: the same item program on the bf16 MFMA; against the bf16
    persistent ping-pong the arithmetic is identical up to O's final rounding
    (one bf16 ulp = 2^-8 relative, |O| < 0.5 here) except in its tail split,
    and the fp32
    torch reference bounds both at test_bf16_gpu.py's 5e-3."""
    fa = _fa()
    b, h, s = shape
    q, k, v = (_rand((b, h, s, 128), 900 + i).to(torch.bfloat16) for i in range(3))
    base = fa.flash_attention_fwd(q, k, v, causal=causal, config=_ids(BF16_BASE)[causal])
    out = fa.flash_attention_fwd(q, k, v, causal=causal, config=_ids(BF16_W4)[causal])
    torch.cuda.synchronize()
    assert out.dtype == torch.bfloat16
    diff = (out.float() - base.float()).abs()
    assert diff.max().item() <= 2.0 ** -9, diff.max().item()
    # (no bit-match fraction here: the bf16 ping-pong runs a short
    # non-causal last round as KV-pair halves, whose key-split merge rounds
    # differently -- 1x72x1024 -- and there is no per-item bf16 ping-pong)
    sc = q.float() @ k.float().transpose(-1, -2) / 128 ** 0.5
    if causal:
        sc = sc + torch.full((s, s), float("-inf"), device="cuda").triu(1)
    ref = torch.softmax(sc, -1) @ v.float()
    assert (out.float() - ref).abs().max().item() <= 5e-3


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("b,h,s", [(2100, 32, 64), (1100, 32, 300)])
def test_w4_second_item_chunk(b, h, s, causal):
    # > 256 rounds per workgroup (67,200 / 70,400 items on 256 CUs): the
    # kernel's second item table (kW4Chunk = 256 slots per asm statement)
    # starts cold -- ITEM/WARM reset, stale K/V images, the cross-item
    # epilogue deferral stopped at the first chunk's last item
    _compare(b, h, s, causal, seed=900)


# head_dim 64: the same item program with 2-step QK^T chains, 4 O^T column
# blocks per row block, K/V by LDS-DMA into packed 128-B-row images (round
# 5; register-staged into half-filled 256-B slots before); against the
# head_dim-64 persistent ping-pong (same arithmetic) and the oracle
D64_W4 = "d64_" + W4
D64_BASE = "d64_bm256_bn64_w8_m16_pingpong_persistent"
D64_SHAPES = [(1, 8, 512), (2, 64, 2048), (3, 40, 1000), (1, 203, 300), (4, 50, 64), (1, 7, 4096),
              (1, 32, 2048), (1, 72, 1024), (1, 4, 77)]


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("shape", D64_SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_w4_d64_matches_pingpong_and_oracle(shape, causal):
    b, h, s = shape
    # the persistent ping-pong runs a short non-causal last round as KV-pair
    # halves (a different merge rounding): compare values, not bits, there
    _compare(b, h, s, causal, seed=1000, d=64, w4=D64_W4, base_tier=D64_BASE,
             max_frac=2e-3 if causal else None)


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("shape", _random_shapes(4, 2064), ids=lambda s: "x".join(map(str, s)))
def test_w4_d64_random_shapes(shape, causal):
    _compare(*shape, causal, seed=1200, d=64, w4=D64_W4, base_tier=D64_BASE,
             max_frac=2e-3 if causal else None)


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("s", [256, 1000, 2048])
def test_w4_d64_peaked_rescale(s, causal):
    _compare(1, 8, s, causal, seed=1100, scale=4.0, d=64, w4=D64_W4, base_tier=D64_BASE,
             max_frac=2e-3 if causal else None)


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("b,h,s", [(2100, 32, 64), (1, 2, 8192)])
def test_w4_d64_long_and_second_chunk(b, h, s, causal):
    _compare(b, h, s, causal, seed=1200, d=64, w4=D64_W4, base_tier=D64_BASE,
             max_frac=2e-3 if causal else None)


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("shape", [(1, 8, 512), (3, 40, 1000), (1, 4, 77)], ids=lambda s: "x".join(map(str, s)))
def test_w4_d64_bf16(shape, causal):
    fa = _fa()
    b, h, s = shape
    q, k, v = (_rand((b, h, s, 64), 1300 + i).to(torch.bfloat16) for i in range(3))
    out = fa.flash_attention_fwd(q, k, v, causal=causal, config=_ids("bf16_" + D64_W4)[causal])
    torch.cuda.synchronize()
    sc = q.float() @ k.float().transpose(-1, -2) / 64 ** 0.5
    if causal:
        sc = sc + torch.full((s, s), float("-inf"), device="cuda").triu(1)
    ref = torch.softmax(sc, -1) @ v.float()
    assert (out.float() - ref).abs().max().item() <= 5e-3


BF16_D64_BASE = "bf16_d64_bm256_bn64_w8_m16_pingpong_persistent"


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("shape", [(1, 8, 512), (3, 40, 1000), (2, 64, 2048), (1, 4, 77), (1, 2, 8192),
                                   (2100, 32, 64)], ids=lambda s: "x".join(map(str, s)))
def test_w4_d64_bf16_matches_pingpong(shape, causal):
    """bf16 at head_dim 64 (the packed-image LDS-DMA program on the bf16
    MFMA) against the bf16 head_dim-64 persistent ping-pong -- the same
    arithmetic up to O's final rounding, within two bf16 ulps at |O| < 0.5
    (the ping-pong's short non-causal tail runs as KV-pair halves) -- and
    the fp32 torch reference at 5e-3; a long head and a second item chunk
    (2100 x 32 heads of 64 rows: > 256 items per workgroup) included"""
    fa = _fa()
    b, h, s = shape
    q, k, v = (_rand((b, h, s, 64), 1400 + i).to(torch.bfloat16) for i in range(3))
    base = fa.flash_attention_fwd(q, k, v, causal=causal, config=_ids(BF16_D64_BASE)[causal])
    out = fa.flash_attention_fwd(q, k, v, causal=causal, config=_ids("bf16_" + D64_W4)[causal])
    torch.cuda.synchronize()
    assert out.dtype == torch.bfloat16
    assert (out.float() - base.float()).abs().max().item() <= 2.0 ** -8
    for bi in range(min(b, 2)):
        sc = q[bi].float() @ k[bi].float().transpose(-1, -2) / 64 ** 0.5
        if causal:
            sc = sc + torch.full((s, s), float("-inf"), device="cuda").triu(1)
        ref = torch.softmax(sc, -1) @ v[bi].float()
        assert (out[bi].float() - ref).abs().max().item() <= 5e-3


@pytest.mark.parametrize("causal", [False, True])
def test_w4_d64_bf16_peaked(causal):
    fa = _fa()
    q, k = (_rand((1, 8, 1000, 64), 1450 + i, scale=4.0).to(torch.bfloat16) for i in range(2))
    v = _rand((1, 8, 1000, 64), 1452).to(torch.bfloat16)
    out = fa.flash_attention_fwd(q, k, v, causal=causal, config=_ids("bf16_" + D64_W4)[causal])
    torch.cuda.synchronize()
    sc = q.float() @ k.float().transpose(-1, -2) / 64 ** 0.5
    if causal:
        sc = sc + torch.full((1000, 1000), float("-inf"), device="cuda").triu(1)
    ref = torch.softmax(sc, -1) @ v.float()
    assert (out.float() - ref).abs().max().item() <= 5e-3
