"""Causal split tier (fa_fwd_f16_ws / fa_fwd_bf16_ws, fa_w4_kernel.hpp
fa_fwd_f16_w4s_kernel): short causal launches cut each 256-row query block's
key range into pieces run by separate workgroups and merged in the same
launch through a caller-owned workspace -- the reference's split-K log-sum-exp
merge (flash_attention.cu:559-598) without its second kernel.

Gate: the oracle (reference cpu_attention restatement) at 1e-3 for fp16 on
sampled heads; bf16 against an fp32 torch reference at test_bf16_gpu.py's
5e-3.  The partials are normalised fp16 / bf16 rows plus an fp32
log2-sum-exp, so the merged output can differ from the unsplit kernels by
about one ulp of the element type; the tolerance is the same as every tier's.
Also: the workspace is reused across launches (arrival counters reset by the
last arriver), two streams with their own workspaces, and the C entry's
workspace checks.
"""
import ctypes

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import oracle  # noqa: E402  (test infrastructure)

pytestmark = pytest.mark.gpu
TOL = 1e-3


def _fa():
    import fa_mi355x

    return fa_mi355x


def _rand(shape, seed, scale=1.0, dtype=torch.float16):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    t = torch.empty(shape, dtype=torch.float32, device="cuda")
    t.uniform_(-0.5 * scale, 0.5 * scale, generator=g)
    return t.to(dtype)


def _bits(t):
    return t.detach().cpu().contiguous().view(torch.int16).numpy().view(np.uint16)


def _torch_ref(q, k, v):
    s = q.shape[2]
    sc = q.float() @ k.float().transpose(-1, -2) / q.shape[-1] ** 0.5
    sc = sc + torch.full((s, s), float("-inf"), device=q.device).triu(1)
    return torch.softmax(sc, -1) @ v.float()


SHAPES = [(1, 32, 512), (1, 32, 768), (1, 32, 1024), (2, 8, 1000), (1, 16, 2048), (1, 4, 4096),
          (3, 5, 1500), (1, 1, 512)]


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_split_matches_oracle(shape):
    fa = _fa()
    b, h, s = shape
    assert fa.load_library().fa_fwd_split_pieces(b, h, s, 128, 1) > 0, "shape must split"
    q, k, v = (_rand((b, h, s, 128), 1000 + i) for i in range(3))
    out = fa.flash_attention_fwd(q, k, v, causal=True)
    torch.cuda.synchronize()
    assert torch.isfinite(out.float()).all()
    for flat in sorted({0, b * h // 2, b * h - 1}):
        bi, hi = divmod(flat, h)
        sl = (slice(bi, bi + 1), slice(hi, hi + 1))
        ref = oracle.attention(*(_bits(x[sl]) for x in (q, k, v)), True)
        d = oracle.max_abs_diff(_bits(out[sl]), ref)
        assert d <= TOL, f"head {flat}: max_diff={d}"
    # every head against the fp32 torch reference
    err = (out.float() - _torch_ref(q, k, v)).abs().max().item()
    assert err <= TOL, err


@pytest.mark.parametrize("shape", [(1, 32, 1024), (2, 8, 1000)], ids=lambda s: "x".join(map(str, s)))
def test_split_peaked(shape):
    # Q, K x4: row maxima grow past the lazy-rescale threshold inside pieces
    fa = _fa()
    b, h, s = shape
    q, k = (_rand((b, h, s, 128), 1100 + i, scale=4.0) for i in range(2))
    v = _rand((b, h, s, 128), 1102)
    out = fa.flash_attention_fwd(q, k, v, causal=True)
    torch.cuda.synchronize()
    err = (out.float() - _torch_ref(q, k, v)).abs().max().item()
    assert err <= TOL, err


@pytest.mark.parametrize("shape", [(1, 32, 1024), (2, 8, 1000), (1, 16, 2048)],
                         ids=lambda s: "x".join(map(str, s)))
def test_split_bf16(shape):
    fa = _fa()
    b, h, s = shape
    q, k, v = (_rand((b, h, s, 128), 1200 + i, dtype=torch.bfloat16) for i in range(3))
    out = fa.flash_attention_fwd(q, k, v, causal=True)
    torch.cuda.synchronize()
    assert out.dtype == torch.bfloat16
    err = (out.float() - _torch_ref(q, k, v)).abs().max().item()
    assert err <= 5e-3, err


def test_split_workspace_reuse_and_streams():
    """Back-to-back launches of different shapes on one workspace, then two
    streams with their own workspaces: every result equals the first launch's
    (the arrival counters are back at zero after each launch)."""
    fa = _fa()
    shapes = [(1, 32, 1024), (1, 32, 512), (2, 8, 1000)]
    data = {sh: [_rand(sh + (128,), 1300 + 3 * n + i) for i in range(3)] for n, sh in enumerate(shapes)}
    first = {sh: fa.flash_attention_fwd(*data[sh], causal=True) for sh in shapes}
    for _ in range(3):
        for sh in shapes:
            o = fa.flash_attention_fwd(*data[sh], causal=True)
            torch.cuda.synchronize()
            assert torch.equal(o, first[sh]), sh
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    torch.cuda.synchronize()
    for st in (s1, s2):
        with torch.cuda.stream(st):
            for sh in shapes:
                outs.append((sh, fa.flash_attention_fwd(*data[sh], causal=True)))
    torch.cuda.synchronize()
    for sh, o in outs:
        assert torch.equal(o, first[sh]), sh


def test_split_c_entry_workspace_checks():
    fa = _fa()
    lib = fa.load_library()
    b, h, s = 1, 32, 1024
    need = lib.fa_fwd_ws_bytes(b, h, s, 128, 1)
    assert need > 0
    q, k, v = (_rand((b, h, s, 128), 1400 + i) for i in range(3))
    o = torch.empty_like(q)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    ws = torch.zeros(need, dtype=torch.uint8, device="cuda")
    assert lib.fa_fwd_f16_ws(p(q), p(k), p(v), p(o), b, h, s, 128, 1, None, need, st) == fa.FA_ERR_WORKSPACE
    assert lib.fa_fwd_f16_ws(p(q), p(k), p(v), p(o), b, h, s, 128, 1, p(ws), need - 1, st) == \
        fa.FA_ERR_WORKSPACE
    assert lib.fa_fwd_f16_ws(p(q), p(k), p(v), p(o), b, h, s, 128, 1, p(ws), need, st) == fa.FA_OK
    torch.cuda.synchronize()
    ref = fa.flash_attention_fwd(q, k, v, causal=True, config=fa.select_config(b, h, s, True))
    torch.cuda.synchronize()
    assert (o.float() - ref.float()).abs().max().item() <= 2 * TOL
    # a shape that does not split ignores the workspace and runs fa_fwd_f16
    assert lib.fa_fwd_ws_bytes(b, h, 8192, 128, 1) == 0
    assert lib.fa_fwd_ws_bytes(b, h, s, 128, 0) == 0
