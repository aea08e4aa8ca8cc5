"""GPU checks specific to the KV-pair kernel (attention_kvpair, configs
*_kvpair_*): the two waves of a SIMD split one row block's key range and merge
(O, m, l) through LDS, so the cases that stress the merge are the ones where
one partner sees no key of a row (causal rows 0..63, single-tile sequences),
odd / even tile counts, and rows whose maxima differ strongly between the two
halves (peaked softmax).  Oracle: the reference's cpu_attention restatement
(flash_attention.cu:668-697), gate 1e-3.
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


def _kvpair(causal, dtype="float16", head_dim=128, kind="kvpair"):
    return next(c.id for c in _fa().configs() if f"_{kind}_" in c.name and c.causal == causal
                and c.dtype == dtype and c.head_dim == head_dim)


# kvpair: two waves per 32 query rows (2-way key split, 128-row blocks);
# kvquad: four waves per 32 rows (4-way split, 64-row blocks, 128-key stages)
KINDS = ["kvpair", "kvquad"]


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int16)).view(torch.float16).cuda()


def _bits(t):
    return t.detach().cpu().contiguous().view(torch.int16).numpy().view(np.uint16)


def _check(b, h, s, causal, seed, qk_scale=1.0, kind="kvpair"):
    q, k, v = oracle.gen_inputs(b, h, s, 128, seed)
    if qk_scale != 1.0:
        f = lambda a: (oracle.f16_bits_to_f32(a) * qk_scale).astype(np.float16).view(np.uint16)
        q, k = f(q), f(k)
    ref = oracle.attention(q, k, v, causal)
    o = _fa().flash_attention_fwd(_dev(q), _dev(k), _dev(v), causal=causal,
                                  config=_kvpair(causal, kind=kind))
    torch.cuda.synchronize()
    d = oracle.max_abs_diff(_bits(o), ref)
    assert d <= TOL, f"{kind} b={b} h={h} s={s} causal={causal}: max_diff={d}"


# tile counts 1 (partners idle), 2, 3 (odd: group A has one more), 5 (quad:
# three stages, the last half-full), 16, 17; ragged tails
@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("s", [64, 128, 192, 320, 1024, 1088, 1000])
@pytest.mark.parametrize("causal", [False, True])
def test_kvpair_tile_counts(s, causal, kind):
    _check(1, 3, s, causal, seed=21, kind=kind)


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("causal", [False, True])
def test_kvpair_peaked_merge(causal, kind):
    # Q,K x8: row maxima differ by many units between the key splits, so the
    # merge's 2^(m_a - M) / 2^(m_b - M) weights are far from 1
    _check(1, 2, 768, causal, seed=5, qk_scale=8.0, kind=kind)


@pytest.mark.parametrize("kind", KINDS)
def test_kvpair_batch_ragged(kind):
    _check(2, 3, 77, True, seed=8, kind=kind)
    _check(2, 3, 300, False, seed=9, kind=kind)


@pytest.mark.parametrize("kind", KINDS)
def test_kvpair_causal_row0_is_v0(kind):
    # row 0 sees key 0 only; its partner (odd tiles) sees nothing and must
    # contribute weight 0: O[0] == V[0] exactly
    fa = _fa()
    g = torch.Generator(device="cuda")
    g.manual_seed(9)
    q, k, v = (torch.empty(2, 4, 1024, 128, dtype=torch.float16, device="cuda")
               .uniform_(-0.5, 0.5, generator=g) for _ in range(3))
    o = fa.flash_attention_fwd(q, k, v, causal=True, config=_kvpair(True, kind=kind))
    torch.cuda.synchronize()
    assert torch.equal(o[:, :, 0], v[:, :, 0])


def test_kvpair_is_a_short_tier():
    fa = _fa()
    cfgs = fa.configs()
    # between the KV-quad's and the paired tier's non-causal shapes, causal
    # launches past S=4096 short of the KV-quad's and the persistent tier's
    assert "_kvpair_" in cfgs[fa.select_config(1, 5, 4160, False)].name  # long heads (65 blocks)
    assert "_kvpair_" in cfgs[fa.select_config(1, 6, 8192, True)].name
    # dispatched at such a shape: same result as the forced config
    g = torch.Generator(device="cuda")
    g.manual_seed(4)
    q, k, v = (torch.empty(1, 6, 8192, 128, dtype=torch.float16, device="cuda")
               .uniform_(-0.5, 0.5, generator=g) for _ in range(3))
    a = fa.flash_attention_fwd(q, k, v, causal=True, config=fa.select_config(1, 6, 8192, True))
    b = fa.flash_attention_fwd(q, k, v, causal=True, config=_kvpair(True))
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("dtype,head_dim", [("bfloat16", 128), ("float16", 64), ("bfloat16", 64)])
def test_kvpair_twins_vs_fp32(dtype, head_dim, kind):
    fa = _fa()
    tdt = torch.bfloat16 if dtype == "bfloat16" else torch.float16
    g = torch.Generator(device="cuda")
    g.manual_seed(13)
    for causal in (False, True):
        q, k, v = (torch.empty(1, 4, 640, head_dim, dtype=tdt, device="cuda")
                   .uniform_(-0.5, 0.5, generator=g) for _ in range(3))
        o = fa.flash_attention_fwd(q, k, v, causal=causal,
                                   config=_kvpair(causal, dtype, head_dim, kind))
        ref = torch.nn.functional.scaled_dot_product_attention(q.float(), k.float(), v.float(),
                                                               is_causal=causal)
        tol = 5e-3 if dtype == "bfloat16" else 1e-3
        assert (o.float() - ref).abs().max().item() <= tol

