"""Short tier (fa_w4k_kernel.hpp, gen_w4k_item.py): a workgroup's one or two
64-row query blocks, their key tiles flattened and split into quarters over
the four waves, one segment per (wave, block), merged in LDS -- the
reference's split-K log-sum-exp merge (flash_attention.cu:559-598) inside
the workgroup.

Gate: the oracle (reference cpu_attention restatement) at 1e-3 on sampled
heads, every head against an fp32 torch reference at 1e-3; bf16 against the
fp32 torch reference at test_bf16_gpu.py's 5e-3.  Shapes cover one block per
workgroup (launches within the CU count) and two (causal heavy/light pairs,
pairs across heads when a head has an odd block count, a last workgroup with
one block), ragged S (masked last tiles, partial Q blocks), segments of one
tile, long segments (S=4096 single head), and the rescale path (peaked
softmax).
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


def _cfg(causal, bf16=False):
    name = ("bf16_" if bf16 else "") + "bm64_bn64_w4x64_asm_keysplit_" + ("causal" if causal else "noncausal")
    ids = [c.id for c in _fa().configs() if c.name == name]
    assert len(ids) == 1, name
    return ids[0]


def _rand(shape, seed, scale=1.0, dtype=torch.float16):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    t = torch.empty(shape, dtype=torch.float32, device="cuda")
    t.uniform_(-0.5 * scale, 0.5 * scale, generator=g)
    return t.to(dtype)


def _bits(t):
    return t.detach().cpu().contiguous().view(torch.int16).numpy().view(np.uint16)


def _torch_ref(q, k, v, causal):
    s = q.shape[2]
    sc = q.float() @ k.float().transpose(-1, -2) / q.shape[-1] ** 0.5
    if causal:
        sc = sc + torch.full((s, s), float("-inf"), device=q.device).triu(1)
    return torch.softmax(sc, -1) @ v.float()


# (B, H, S): 64-row blocks B*H*ceil(S/64) -- <= 256: one per workgroup, else two
SHAPES = [(1, 32, 512), (1, 32, 1024), (1, 8, 1024), (1, 32, 768), (1, 3, 1), (1, 2, 7),
          (2, 3, 65), (1, 4, 100), (1, 5, 300), (2, 2, 777), (1, 16, 2000), (1, 20, 960),
          (1, 19, 960), (1, 1, 4096), (4, 8, 640)]


@pytest.mark.parametrize("causal", [False, True], ids=["noncausal", "causal"])
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_w4k_matches_oracle(shape, causal):
    fa = _fa()
    b, h, s = shape
    q, k, v = (_rand((b, h, s, 128), 2000 + 7 * s + i) for i in range(3))
    out = fa.flash_attention_fwd(q, k, v, causal=causal, config=_cfg(causal))
    torch.cuda.synchronize()
    assert torch.isfinite(out.float()).all()
    for flat in sorted({0, b * h // 2, b * h - 1}):
        bi, hi = divmod(flat, h)
        sl = (slice(bi, bi + 1), slice(hi, hi + 1))
        ref = oracle.attention(*(_bits(x[sl]) for x in (q, k, v)), causal)
        d = oracle.max_abs_diff(_bits(out[sl]), ref)
        assert d <= TOL, f"head {flat}: max_diff={d}"
    err = (out.float() - _torch_ref(q, k, v, causal)).abs().max().item()
    assert err <= TOL, err


@pytest.mark.parametrize("causal", [False, True], ids=["noncausal", "causal"])
def test_w4k_peaked_softmax(causal):
    """Q, K x4: scores spread past the lazy-rescale threshold (slow path)"""
    fa = _fa()
    b, h, s = 1, 32, 1024
    q, k = (_rand((b, h, s, 128), 31 + i, scale=4.0) for i in range(2))
    v = _rand((b, h, s, 128), 33)
    out = fa.flash_attention_fwd(q, k, v, causal=causal, config=_cfg(causal))
    torch.cuda.synchronize()
    err = (out.float() - _torch_ref(q, k, v, causal)).abs().max().item()
    assert err <= TOL, err
    ref = oracle.attention(*(_bits(x[:1, 5:6]) for x in (q, k, v)), causal)
    assert oracle.max_abs_diff(_bits(out[:1, 5:6]), ref) <= TOL


@pytest.mark.parametrize("causal", [False, True], ids=["noncausal", "causal"])
@pytest.mark.parametrize("shape", [(1, 32, 1024), (1, 5, 300), (1, 32, 512)], ids=lambda s: "x".join(map(str, s)))
def test_w4k_bf16(shape, causal):
    fa = _fa()
    b, h, s = shape
    q, k, v = (_rand((b, h, s, 128), 50 + i, dtype=torch.bfloat16) for i in range(3))
    out = fa.flash_attention_fwd(q, k, v, causal=causal, config=_cfg(causal, bf16=True))
    torch.cuda.synchronize()
    err = (out.float() - _torch_ref(q, k, v, causal)).abs().max().item()
    assert err <= 5e-3, err


def test_w4k_repeatable():
    """same inputs, same bits (no cross-workgroup state)"""
    fa = _fa()
    q, k, v = (_rand((1, 32, 1024, 128), 70 + i) for i in range(3))
    a = fa.flash_attention_fwd(q, k, v, causal=True, config=_cfg(True))
    b = fa.flash_attention_fwd(q, k, v, causal=True, config=_cfg(True))
    torch.cuda.synchronize()
    assert torch.equal(a, b)
