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


# (B, H, S, piece_tiles): 0 = the dispatcher's own split (long causal
# launches short of the persistent tier); > 0 forces that piece length, so
# short and ragged shapes, 2..8 pieces per block and pieces shorter than the
# diagonal's 4 tiles are covered too
SHAPES = [(1, 12, 4096, 44), (1, 8, 4096, 22), (2, 3, 5000, 0), (1, 4, 8192, 0), (1, 32, 512, 4), (1, 32, 768, 4),
          (1, 32, 1024, 6), (2, 8, 1000, 5), (1, 16, 2048, 12), (3, 5, 1500, 4), (1, 1, 512, 4),
          (1, 2, 2048, 4), (2, 2, 700, 2), (1, 3, 512, 1)]


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_split_matches_oracle(shape):
    fa = _fa()
    b, h, s, pt = shape
    if pt == 0:
        assert fa.load_library().fa_fwd_split_pieces(b, h, s, 128, 1) > 0, "shape must split"
    q, k, v = (_rand((b, h, s, 128), 1000 + i) for i in range(3))
    out = fa.flash_attention_fwd(q, k, v, causal=True, piece_tiles=pt)
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


@pytest.mark.parametrize("shape", [(1, 32, 1024, 6), (2, 8, 1000, 4), (1, 4, 4096, 22)],
                         ids=lambda s: "x".join(map(str, s)))
def test_split_peaked(shape):
    # Q, K x4: row maxima grow past the lazy-rescale threshold inside pieces
    fa = _fa()
    b, h, s, pt = shape
    q, k = (_rand((b, h, s, 128), 1100 + i, scale=4.0) for i in range(2))
    v = _rand((b, h, s, 128), 1102)
    out = fa.flash_attention_fwd(q, k, v, causal=True, piece_tiles=pt)
    torch.cuda.synchronize()
    err = (out.float() - _torch_ref(q, k, v)).abs().max().item()
    assert err <= TOL, err


@pytest.mark.parametrize("shape", [(1, 32, 1024, 6), (2, 8, 1000, 4), (1, 12, 4096, 44)],
                         ids=lambda s: "x".join(map(str, s)))
def test_split_bf16(shape):
    fa = _fa()
    b, h, s, pt = shape
    q, k, v = (_rand((b, h, s, 128), 1200 + i, dtype=torch.bfloat16) for i in range(3))
    out = fa.flash_attention_fwd(q, k, v, causal=True, piece_tiles=pt)
    torch.cuda.synchronize()
    assert out.dtype == torch.bfloat16
    err = (out.float() - _torch_ref(q, k, v)).abs().max().item()
    assert err <= 5e-3, err


def test_split_workspace_reuse_and_streams():
    """Back-to-back launches of different shapes on one workspace, then two
    streams with their own workspaces: every result equals the first launch's
    (the arrival counters are back at zero after each launch)."""
    fa = _fa()
    shapes = [(1, 4, 4096, 22), (1, 32, 1024, 6), (1, 32, 512, 4), (2, 8, 1000, 5)]
    data = {sh: [_rand(sh[:3] + (128,), 1300 + 3 * n + i) for i in range(3)] for n, sh in enumerate(shapes)}
    run = lambda sh: fa.flash_attention_fwd(*data[sh], causal=True, piece_tiles=sh[3])
    first = {sh: run(sh) for sh in shapes}
    for _ in range(3):
        for sh in shapes:
            o = run(sh)
            torch.cuda.synchronize()
            assert torch.equal(o, first[sh]), sh
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    torch.cuda.synchronize()
    for st in (s1, s2):
        with torch.cuda.stream(st):
            for sh in shapes:
                outs.append((sh, run(sh)))
    torch.cuda.synchronize()
    for sh, o in outs:
        assert torch.equal(o, first[sh]), sh


def test_split_c_entry_workspace_checks():
    fa = _fa()
    lib = fa.load_library()
    b, h, s = 1, 4, 8192  # a shape the dispatcher splits (S=4096 at H<=8: the paired tier)
    need = lib.fa_fwd_ws_bytes(b, h, s, 128, 1, 0)
    assert need > 0
    q, k, v = (_rand((b, h, s, 128), 1400 + i) for i in range(3))
    o = torch.empty_like(q)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    b2, h2, s2, pt2 = 2, 16, 1000, 3  # a second shape on the same buffer (below)
    need2 = lib.fa_fwd_ws_bytes(b2, h2, s2, 128, 1, pt2)
    assert need2 > 0
    ws = torch.zeros(max(need, need2), dtype=torch.uint8, device="cuda")
    assert lib.fa_fwd_f16_ws(p(q), p(k), p(v), p(o), b, h, s, 128, 1, 0, None, need, st) == \
        fa.FA_ERR_WORKSPACE
    assert lib.fa_fwd_f16_ws(p(q), p(k), p(v), p(o), b, h, s, 128, 1, 0, p(ws), need - 1, st) == \
        fa.FA_ERR_WORKSPACE
    # only the first 64 KB (the arrival counters) must be zero: poison the rest
    ws[65536:] = 0xFF
    assert lib.fa_fwd_f16_ws(p(q), p(k), p(v), p(o), b, h, s, 128, 1, 0, p(ws), need, st) == fa.FA_OK
    torch.cuda.synchronize()
    ref = fa.flash_attention_fwd(q, k, v, causal=True, config=fa.select_config(b, h, s, True))
    torch.cuda.synchronize()
    assert (o.float() - ref.float()).abs().max().item() <= 2 * TOL
    assert not ws[:65536].any()  # counters back at zero
    # another shape (more query blocks, other piece count) on the same buffer
    q2, k2, v2 = (_rand((b2, h2, s2, 128), 1410 + i) for i in range(3))
    o2 = torch.empty_like(q2)
    assert lib.fa_fwd_f16_ws(p(q2), p(k2), p(v2), p(o2), b2, h2, s2, 128, 1, pt2, p(ws), need2,
                             st) == fa.FA_OK
    torch.cuda.synchronize()
    assert (o2.float() - _torch_ref(q2, k2, v2)).abs().max().item() <= TOL
    assert not ws[:65536].any()
    # shapes that do not split ignore the workspace and run fa_fwd_f16
    assert lib.fa_fwd_ws_bytes(b, 32, 8192, 128, 1, 0) == 0
    assert lib.fa_fwd_ws_bytes(b, h, s, 128, 0, 0) == 0
