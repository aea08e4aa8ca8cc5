"""torch.library custom op (fa_mi355x/torch_op.py).

CPU: the op registers, shape-propagates on meta tensors (fake impl), and
refuses CPU tensors (no CPU path).  GPU: it is the product kernel (bit-equal
to the ctypes entry point), agrees with PyTorch SDPA and the oracle, works
under torch.compile and inside a captured HIP graph.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import oracle  # noqa: E402  (test infrastructure)


def _op():
    import fa_mi355x.torch_op  # noqa: F401

    return torch.ops.fa_mi355x.fwd


def test_op_registered_and_meta_shapes():
    op = _op()
    for causal in (False, True):
        q = torch.empty((2, 3, 77, 128), dtype=torch.float16, device="meta")
        o = op(q, q, q, causal)
        assert o.shape == q.shape and o.dtype == torch.float16 and o.device.type == "meta"


def test_op_rejects_cpu_tensors():
    op = _op()
    q = torch.zeros((1, 1, 8, 128), dtype=torch.float16)
    with pytest.raises(ValueError):
        op(q, q, q, False)


def test_op_is_forward_only():
    # no backward formula: refuse loudly instead of zero gradients
    op = _op()
    q = torch.empty((1, 2, 64, 128), dtype=torch.float16, device="meta", requires_grad=True)
    with pytest.raises(RuntimeError, match="forward-only"):
        op(q, q, q, True)
    with torch.no_grad():
        assert op(q, q, q, True).shape == q.shape
    assert op(q.detach(), q.detach(), q.detach(), False).shape == q.shape


def _rand(shape, seed):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    return torch.empty(shape, dtype=torch.float16, device="cuda").uniform_(-0.5, 0.5, generator=g)


def _bits(t):
    return t.detach().cpu().contiguous().view(torch.int16).numpy().view(np.uint16)


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True])
def test_op_matches_entry_point_sdpa_and_oracle(causal):
    import fa_mi355x as fa

    op = _op()
    shape = (2, 4, 1000, 128)
    q, k, v = _rand(shape, 1), _rand(shape, 2), _rand(shape, 3)
    o = op(q, k, v, causal)
    o_ref = fa.flash_attention_fwd(q, k, v, causal=causal)
    sd = torch.nn.functional.scaled_dot_product_attention(q.float(), k.float(), v.float(),
                                                          is_causal=causal)
    torch.cuda.synchronize()
    assert torch.equal(o, o_ref)
    assert (o.float() - sd).abs().max().item() <= 1e-3
    sl = (slice(1, 2), slice(3, 4))
    ref = oracle.attention(*(_bits(x[sl]) for x in (q, k, v)), causal)
    assert oracle.max_abs_diff(_bits(o[sl]), ref) <= 1e-3


@pytest.mark.gpu
def test_op_under_torch_compile():
    op = _op()

    def f(q, k, v):
        return op(q, k, v, True) * 2.0

    shape = (1, 8, 512, 128)
    q, k, v = _rand(shape, 4), _rand(shape, 5), _rand(shape, 6)
    eager = f(q, k, v)
    compiled = torch.compile(f, backend="eager", fullgraph=True)(q, k, v)
    torch.cuda.synchronize()
    assert torch.equal(eager, compiled)


@pytest.mark.gpu
def test_op_in_hip_graph():
    op = _op()
    shape = (1, 32, 1024, 128)
    q, k, v = _rand(shape, 7), _rand(shape, 8), _rand(shape, 9)
    want = op(q, k, v, True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        op(q, k, v, True)  # warm-up on the capture stream
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = op(q, k, v, True)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, want)
