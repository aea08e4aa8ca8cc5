"""Persistent kernels (one workgroup per CU walking its XCD's query blocks;
register-staged K/V, and the LDS-DMA variant with three rotating buffers):
shapes where every workgroup walks SEVERAL query blocks, including ragged
sequence lengths, head counts that are not a multiple of the 8 XCD groups,
and single-tile items.

It runs exactly the per-tile arithmetic of the one-workgroup-per-item
ping-pong kernel (bm256_bn64_w8_m16_pingpong_*) in the same order, so its output must be
bit-identical to it; sampled heads are also checked against the oracle
(reference cpu_attention restatement) at the 1e-3 gate.
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


def _rand(shape, seed):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    t = torch.empty(shape, dtype=torch.float16, device="cuda")
    t.uniform_(-0.5, 0.5, generator=g)
    return t


def _bits(t):
    return t.detach().cpu().contiguous().view(torch.int16).numpy().view(np.uint16)


def _base_ids():
    """the per-item 8-wave ping-pong (the bit-identity baseline)"""
    out = {c.causal: c.id for c in _fa().configs()
           if c.name in ("bm256_bn64_w8_m16_pingpong_noncausal", "bm256_bn64_w8_m16_pingpong_causal")}
    assert set(out) == {False, True}
    return out


def _ids(kind_name):
    fa = _fa()
    out = {}
    for c in fa.configs():
        if c.dtype == "float16" and c.head_dim == 128 and c.name in (
                f"bm256_bn64_w8_m16_pingpong_{kind_name}_noncausal",
                f"bm256_bn64_w8_m16_pingpong_{kind_name}_causal"):
            out[c.causal] = c.id
    assert set(out) == {False, True}, kind_name
    return out


SHAPES = [
    (2, 64, 2048),   # 16 query blocks x 128 heads: 4+ items per workgroup
    (3, 40, 1000),   # ragged S, 120 heads (15 per XCD group)
    (1, 203, 300),   # odd head count, 2 query blocks, last one ragged
    (4, 50, 64),     # single-tile items (n = 1)
    (1, 7, 4096),    # fewer heads than XCD groups
    (1, 2, 4096),    # 2 heads: non-affine split of the items over all 8 XCDs
    # causal work orders (fa_fwd.hip persistent kernel): pair order at <= 64
    # heads with an even number of query blocks, else the rank-band snake
    (1, 32, 2048),   # pairs: 8 query blocks, 4 heads per XCD group
    (1, 64, 1536),   # pairs at the 64-head boundary, 6 query blocks
    (1, 16, 1280),   # odd query-block count (5): band-1 snake fallback
    (1, 72, 1024),   # 72 heads (> 64): band-16 snake, 4 query blocks
]


def _nc_tail_split(kind, b, h, s, causal, cus=256):
    """The persistent non-causal register-staged kernel runs an XCD's last
    round as KV-pair halves when it holds <= C/2 items (fa_fwd.hip): those
    rows are not bit-identical to the ping-pong (key split + LSE merge)."""
    if causal or kind != "persistent":
        return False
    bh, nqb = b * h, (s + 255) // 256
    per_xcd = (bh // 8) * nqb if bh % 8 == 0 else (bh * nqb + 7) // 8
    c = min(cus // 8, per_xcd)
    tail = per_xcd - (per_xcd // c) * c
    return 0 < tail and 2 * tail <= c


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("kind", ["persistent", "persistent_dma"])
def test_persistent_bit_identical(kind, shape, causal):
    fa = _fa()
    b, h, s = shape
    q, k, v = (_rand((b, h, s, 128), 100 + i) for i in range(3))
    out_base = fa.flash_attention_fwd(q, k, v, causal=causal, config=_base_ids()[causal])
    out = fa.flash_attention_fwd(q, k, v, causal=causal, config=_ids(kind)[causal])
    torch.cuda.synchronize()
    cus = torch.cuda.get_device_properties(q.device).multi_processor_count
    if _nc_tail_split(kind, b, h, s, causal, cus):
        assert (out.float() - out_base.float()).abs().max().item() <= TOL
    else:
        assert torch.equal(out, out_base)
    # sampled heads against the oracle: first, last, and one in the middle
    for flat in sorted({0, b * h // 2, b * h - 1}):
        bi, hi = divmod(flat, h)
        sl = (slice(bi, bi + 1), slice(hi, hi + 1))
        ref = oracle.attention(*(_bits(x[sl]) for x in (q, k, v)), causal)
        d = oracle.max_abs_diff(_bits(out[sl]), ref)
        assert d <= TOL, f"head {flat}: max_diff={d}"


# Non-causal tail split: B=1 H=48 S=2048 gives 48 items per XCD on 32 CUs; the
# last 16 run as 32 KV-pair halves (key range split, LSE merge), so those rows
# are not bit-identical to the ping-pong -- compare within the 1e-3 gate, and
# the tail heads (the last items of each XCD) against the oracle.
@pytest.mark.parametrize("kind", ["persistent"])
def test_persistent_nc_tail_split(kind):
    fa = _fa()
    b, h, s = 1, 48, 2048
    q, k, v = (_rand((b, h, s, 128), 300 + i) for i in range(3))
    out_base = fa.flash_attention_fwd(q, k, v, causal=False, config=_base_ids()[False])
    out = fa.flash_attention_fwd(q, k, v, causal=False, config=_ids(kind)[False])
    torch.cuda.synchronize()
    assert (out.float() - out_base.float()).abs().max().item() <= TOL
    for flat in (0, 40, 47):  # heads 40..47 hold each XCD's last items
        sl = (slice(0, 1), slice(flat, flat + 1))
        ref = oracle.attention(*(_bits(x[sl]) for x in (q, k, v)), False)
        d = oracle.max_abs_diff(_bits(out[sl]), ref)
        assert d <= TOL, f"head {flat}: max_diff={d}"


def _torch_ref(q, k, v, causal):
    """fp32 reference of the same op (for bf16 / head_dim 64, which the
    reference's fp16 d128 oracle does not cover)."""
    qf, kf, vf = q.float(), k.float(), v.float()
    sc = qf @ kf.transpose(-1, -2) / (q.shape[-1] ** 0.5)
    if causal:
        s = q.shape[2]
        sc = sc + torch.full((s, s), float("-inf"), device=q.device).triu(1)
    return (torch.softmax(sc, dim=-1) @ vf).to(q.dtype)


def _cfg(dtype, head_dim, causal):
    fa = _fa()
    for c in fa.configs():
        if (c.dtype == dtype and c.head_dim == head_dim and c.causal == causal
                and "pingpong_persistent" in c.name and "dma" not in c.name):
            return c.id
    raise AssertionError((dtype, head_dim, causal))


# Ragged tail split: S=1900 gives 8 query blocks of 256 rows, the last one
# ragged; B=1 H=48 puts 48 items on each XCD's 32 CUs, so the last 16 (heads
# 32..47) run as KV-pair halves -- half 14 partly and half 15 entirely past S.
@pytest.mark.parametrize("dtype,head_dim", [("float16", 128), ("bfloat16", 128),
                                            ("float16", 64), ("bfloat16", 64)])
def test_persistent_nc_tail_split_ragged(dtype, head_dim):
    fa = _fa()
    b, h, s = 1, 48, 1900
    tdt = torch.float16 if dtype == "float16" else torch.bfloat16
    q, k, v = (_rand((b, h, s, head_dim), 400 + i).to(tdt) for i in range(3))
    out = fa.flash_attention_fwd(q, k, v, causal=False, config=_cfg(dtype, head_dim, False))
    torch.cuda.synchronize()
    ref = _torch_ref(q, k, v, False)
    tol = TOL if dtype == "float16" else 5e-3  # bf16: 8 significant bits (tests/test_bf16_gpu.py)
    err = (out.float() - ref.float()).abs()
    assert err.max().item() <= tol, f"max err {err.max().item()}"
    if dtype == "float16" and head_dim == 128:
        for flat in (32, 47):  # tail items, against the oracle too
            sl = (slice(0, 1), slice(flat, flat + 1))
            r = oracle.attention(*(_bits(x[sl]) for x in (q, k, v)), False)
            assert oracle.max_abs_diff(_bits(out[sl]), r) <= TOL
