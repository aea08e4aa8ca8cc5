"""bf16 forward (not in the reference, which is fp16
only, flash_attention.cu:613).  Parity is against a torch fp32 reference of
the same op on the same bf16 inputs -- the reference repo has no bf16 oracle,
so this path is "parity unpinned" against the reference itself.

Tolerance: 5e-3 max-abs.  bf16 keeps 8 mantissa bits: Q*scale and P are
rounded to bf16 (relative error 2^-9 each) before the fp32-accumulated
products, so errors are ~8x the fp16 path's.  Measured on the box
(tools/dtype_error.py, profiles/r01_dtype_error.jsonl): worst config 1.9e-3,
PyTorch SDPA in bf16 1.4e-3 on the same inputs.
"""
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu
TOL = 5e-3


def _fa():
    import fa_mi355x

    return fa_mi355x


def _rand(shape, seed, scale=1.0):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    t = torch.empty(shape, dtype=torch.float32, device="cuda").uniform_(-0.5, 0.5, generator=g)
    return (t * scale).to(torch.bfloat16)


def _ref(q, k, v, causal):
    q, k, v = q.float(), k.float(), v.float()
    s = (q @ k.transpose(-1, -2)) / (q.shape[-1] ** 0.5)
    if causal:
        n = q.shape[-2]
        s = s.masked_fill(~torch.ones(n, n, device=q.device, dtype=torch.bool).tril(), float("-inf"))
    return torch.softmax(s, -1) @ v


def _bf16_configs(causal):
    return [c.id for c in _fa().configs()
            if c.dtype == "bfloat16" and c.causal == causal and c.head_dim == 128]


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("s", [1, 77, 512, 1000, 2048])
def test_every_bf16_config(causal, s):
    fa = _fa()
    shape = (1, 4, s, 128)
    q, k, v = _rand(shape, 1), _rand(shape, 2), _rand(shape, 3)
    ref = _ref(q, k, v, causal)
    for cid in _bf16_configs(causal):
        out = fa.flash_attention_fwd(q, k, v, causal=causal, config=cid)
        assert out.dtype == torch.bfloat16
        d = (out.float() - ref).abs().max().item()
        assert d <= TOL, f"config {cid}: max_diff={d}"


@pytest.mark.parametrize("causal", [False, True])
def test_bf16_peaked_softmax(causal):
    """Q, K x4: large logits exercise the running-max rescale branch."""
    fa = _fa()
    shape = (2, 4, 1024, 128)
    q, k, v = _rand(shape, 4, 4.0), _rand(shape, 5, 4.0), _rand(shape, 6)
    ref = _ref(q, k, v, causal)
    for cid in _bf16_configs(causal):
        out = fa.flash_attention_fwd(q, k, v, causal=causal, config=cid)
        assert (out.float() - ref).abs().max().item() <= TOL, cid


@pytest.mark.parametrize("causal", [False, True])
def test_bf16_dispatch_and_sdpa(causal):
    """Default dispatch (persistent ping-pong tier at this size) vs the fp32
    reference and vs PyTorch SDPA in bf16."""
    fa = _fa()
    shape = (2, 32, 2048, 128)
    q, k, v = _rand(shape, 7), _rand(shape, 8), _rand(shape, 9)
    out = fa.flash_attention_fwd(q, k, v, causal=causal)
    ref = _ref(q, k, v, causal)
    sd = torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=causal)
    assert (out.float() - ref).abs().max().item() <= TOL
    assert (out.float() - sd.float()).abs().max().item() <= 2 * TOL


def test_bf16_torch_op():
    import fa_mi355x.torch_op  # noqa: F401

    shape = (1, 8, 512, 128)
    q, k, v = _rand(shape, 10), _rand(shape, 11), _rand(shape, 12)
    out = torch.ops.fa_mi355x.fwd(q, k, v, True)
    assert out.dtype == torch.bfloat16
    assert (out.float() - _ref(q, k, v, True)).abs().max().item() <= TOL


def test_mixed_dtypes_rejected():
    fa = _fa()
    q = _rand((1, 1, 64, 128), 1)
    with pytest.raises(fa.FlashAttentionError):
        fa.flash_attention_fwd(q, q.half(), q, causal=False)
