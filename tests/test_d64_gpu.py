"""head_dim 64 (the reference hard-codes 128,
flash_attention.cu:613).  fp16 is checked against the oracle -- the
reference's cpu_attention restatement, which is head_dim-generic -- at the
same 1e-3 gate as head_dim 128; bf16 against a torch fp32 reference at 5e-3
(tests/test_bf16_gpu.py explains that bound).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import oracle  # noqa: E402  (test infrastructure)

pytestmark = pytest.mark.gpu
D = 64


def _fa():
    import fa_mi355x

    return fa_mi355x


def _rand(shape, seed, dtype=torch.float16, scale=1.0):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    t = torch.empty(shape, dtype=torch.float32, device="cuda").uniform_(-0.5, 0.5, generator=g)
    return (t * scale).to(dtype)


def _bits(t):
    return t.detach().cpu().contiguous().view(torch.int16).numpy().view(np.uint16)


def _ids(dtype, causal):
    return [c.id for c in _fa().configs()
            if c.head_dim == D and c.dtype == dtype and c.causal == causal]


def _ref32(q, k, v, causal):
    q, k, v = q.float(), k.float(), v.float()
    s = (q @ k.transpose(-1, -2)) / (D ** 0.5)
    if causal:
        n = q.shape[-2]
        s = s.masked_fill(~torch.ones(n, n, device=q.device, dtype=torch.bool).tril(), float("-inf"))
    return torch.softmax(s, -1) @ v


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("s", [1, 77, 256, 1000, 2048])
def test_d64_fp16_every_config_vs_oracle(causal, s):
    fa = _fa()
    shape = (1, 2, s, D)
    q, k, v = _rand(shape, 1), _rand(shape, 2), _rand(shape, 3)
    ref = oracle.attention(_bits(q), _bits(k), _bits(v), causal)
    for cid in _ids("float16", causal):
        out = fa.flash_attention_fwd(q, k, v, causal=causal, config=cid)
        d = oracle.max_abs_diff(_bits(out), ref)
        assert d <= 1e-3, f"config {cid}: max_diff={d}"


@pytest.mark.parametrize("causal", [False, True])
def test_d64_peaked_and_dispatch(causal):
    """Q,K x4 (rescale branch) through every config, and the default dispatch
    at a size that selects the persistent ping-pong tier."""
    fa = _fa()
    shape = (1, 2, 1024, D)
    q, k, v = _rand(shape, 4, scale=4.0), _rand(shape, 5, scale=4.0), _rand(shape, 6)
    ref = oracle.attention(_bits(q), _bits(k), _bits(v), causal)
    for cid in _ids("float16", causal):
        out = fa.flash_attention_fwd(q, k, v, causal=causal, config=cid)
        assert oracle.max_abs_diff(_bits(out), ref) <= 1e-3, cid
    shape = (4, 32, 2048, D)
    q, k, v = _rand(shape, 7), _rand(shape, 8), _rand(shape, 9)
    out = fa.flash_attention_fwd(q, k, v, causal=causal)
    assert (out.float() - _ref32(q, k, v, causal)).abs().max().item() <= 1e-3


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("s", [77, 1000])
def test_d64_bf16_every_config(causal, s):
    fa = _fa()
    shape = (2, 3, s, D)
    q, k, v = (_rand(shape, 10 + i, torch.bfloat16) for i in range(3))
    ref = _ref32(q, k, v, causal)
    for cid in _ids("bfloat16", causal):
        out = fa.flash_attention_fwd(q, k, v, causal=causal, config=cid)
        assert out.dtype == torch.bfloat16
        d = (out.float() - ref).abs().max().item()
        assert d <= 5e-3, f"config {cid}: max_diff={d}"


def test_d64_torch_op():
    import fa_mi355x.torch_op  # noqa: F401

    shape = (1, 8, 512, D)
    q, k, v = _rand(shape, 20), _rand(shape, 21), _rand(shape, 22)
    out = torch.ops.fa_mi355x.fwd(q, k, v, True)
    assert out.shape == q.shape
    assert (out.float() - _ref32(q, k, v, True)).abs().max().item() <= 1e-3
