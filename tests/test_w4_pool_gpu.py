"""W4 tier's cross-XCD tail pool (fa_w4_kernel.hpp; workspace launches).

The workspace entry (and the Python / torch path, which always passes one)
runs the last rounds/16 rounds of every XCD's item list (>= 64 rounds) from per-XCD claim
counters in the workspace's counter region: own pool first (from its
front), then the other XCDs' (from their backs).  Which workgroup runs an item does not change its arithmetic, so the
pooled launch must be bit-identical to the static order (fa_fwd_f16, no
workspace), leave the counters at zero, and stay so over repeated launches
and shape changes on one workspace.  Sampled heads are checked against the
oracle as well.
"""
import ctypes

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import oracle  # noqa: E402  (test infrastructure)

pytestmark = pytest.mark.gpu
TOL = 1e-3
CTR = 65536


def _fa():
    import fa_mi355x

    return fa_mi355x


def _rand(shape, seed, dtype=torch.float16):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    t = torch.empty(shape, dtype=torch.float32, device="cuda")
    t.uniform_(-0.5, 0.5, generator=g)
    return t.to(dtype)


def _bits(t):
    return t.detach().cpu().contiguous().view(torch.int16).numpy().view(np.uint16)


def _static(q, k, v, causal):
    """the workspace-free entry: the static item order"""
    fa = _fa()
    lib = fa.load_library()
    o = torch.empty_like(q)
    b, h, s, d = q.shape
    fn = lib.fa_fwd_bf16 if q.dtype == torch.bfloat16 else lib.fa_fwd_f16
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert fn(p(q), p(k), p(v), p(o), b, h, s, d, int(causal), st) == fa.FA_OK
    return o


def _pooled(q, k, v, causal, ws):
    fa = _fa()
    lib = fa.load_library()
    o = torch.empty_like(q)
    b, h, s, d = q.shape
    fn = lib.fa_fwd_bf16_ws if q.dtype == torch.bfloat16 else lib.fa_fwd_f16_ws
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert fn(p(q), p(k), p(v), p(o), b, h, s, d, int(causal), 0, p(ws), ws.numel(), st) == fa.FA_OK
    return o


# (B, H, S, causal, head_dim): >= 64 rounds per XCD list in the snake order
POOL_SHAPES = [
    (32, 32, 4096, True, 128),   # half the headline: 64 rounds, 4 pooled
    (16, 32, 8192, False, 128),  # non-causal, 64 rounds
    (128, 24, 2048, True, 128),  # 3072 heads, 8 items per head: 96 rounds
    (32, 32, 4096, True, 64),    # the head_dim-64 program
    (96, 16, 3000, True, 128),   # ragged S (last item 184 rows): 72 rounds
]


@pytest.mark.parametrize("b,h,s,causal,d", POOL_SHAPES)
def test_pool_matches_static_order(b, h, s, causal, d):
    fa = _fa()
    lib = fa.load_library()
    assert lib.fa_fwd_ws_bytes(b, h, s, d, int(causal), 0) == CTR
    q, k, v = (_rand((b, h, s, d), 900 + i) for i in range(3))
    ws = torch.zeros(CTR, dtype=torch.uint8, device="cuda")
    ref = _static(q, k, v, causal)
    for rep in range(3):  # the counters come back to zero: launches repeat
        out = _pooled(q, k, v, causal, ws)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), rep
        assert not ws.any(), rep
    # the Python entry passes a workspace: it runs the pool too
    assert torch.equal(fa.flash_attention_fwd(q, k, v, causal), ref)
    if d == 128:
        for flat in (0, b * h // 2 + 1, b * h - 1):
            bi, hi = divmod(flat, h)
            sl = (slice(bi, bi + 1), slice(hi, hi + 1))
            rows = sorted({0, 255, 256, s // 2, s - 1})
            ro = oracle.attention_rows(*(_bits(x[sl][0, 0]) for x in (q, k, v)), rows, causal)
            assert oracle.max_abs_diff(_bits(out[sl][0, 0])[rows], ro) <= TOL, flat


def test_pool_bf16_and_shape_change_on_one_workspace():
    fa = _fa()
    ws = torch.zeros(CTR, dtype=torch.uint8, device="cuda")
    for (b, h, s, causal), dt in (((32, 32, 4096, True), torch.bfloat16), ((16, 32, 8192, False), torch.float16),
                                  ((128, 24, 2048, True), torch.bfloat16)):
        q, k, v = (_rand((b, h, s, 128), 950 + i, dt) for i in range(3))
        ref = _static(q, k, v, causal)
        out = _pooled(q, k, v, causal, ws)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), (b, h, s, causal, dt)
        assert not ws.any()


def test_pool_without_counters_is_static():
    """a workspace short of the counter region: the static order, no error"""
    fa = _fa()
    lib = fa.load_library()
    b, h, s = 32, 32, 4096
    q, k, v = (_rand((b, h, s, 128), 970 + i) for i in range(3))
    o = torch.empty_like(q)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    small = torch.zeros(1024, dtype=torch.uint8, device="cuda")
    assert lib.fa_fwd_f16_ws(p(q), p(k), p(v), p(o), b, h, s, 128, 1, 0, p(small), 1024, st) == fa.FA_OK
    assert lib.fa_fwd_f16_ws(p(q), p(k), p(v), p(o), b, h, s, 128, 1, 0, None, 0, st) == fa.FA_OK
    torch.cuda.synchronize()
    assert torch.equal(o, _static(q, k, v, True))


def test_pool_misaligned_workspace_is_static():
    """the 64-bit claim counters need an 8-byte aligned workspace: a misaligned
    one (here 4 bytes in, holding garbage that would make a pool skip items)
    runs the static order and is never touched; the split tier rejects a
    workspace that is not 16-byte aligned (advice r05)"""
    fa = _fa()
    lib = fa.load_library()
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    b, h, s = 32, 32, 4096
    q, k, v = (_rand((b, h, s, 128), 980 + i) for i in range(3))
    o = torch.empty_like(q)
    ws = torch.full((CTR + 64,), 0xFF, dtype=torch.uint8, device="cuda")
    mis = ctypes.c_void_p(ws.data_ptr() + 4)
    assert lib.fa_fwd_f16_ws(p(q), p(k), p(v), p(o), b, h, s, 128, 1, 0, mis, CTR, st) == fa.FA_OK
    torch.cuda.synchronize()
    assert torch.equal(o, _static(q, k, v, True))
    assert bool((ws == 0xFF).all())
    # a split shape (B=1 H=4 S=8192 causal) with an 8-byte (not 16) aligned workspace
    b, h, s = 1, 4, 8192
    need = lib.fa_fwd_ws_bytes(b, h, s, 128, 1, 0)
    assert need > CTR and lib.fa_fwd_split_pieces(b, h, s, 128, 1) > 0
    q, k, v = (_rand((b, h, s, 128), 990 + i) for i in range(3))
    o = torch.empty_like(q)
    ws = torch.zeros(need + 64, dtype=torch.uint8, device="cuda")
    assert lib.fa_fwd_f16_ws(p(q), p(k), p(v), p(o), b, h, s, 128, 1, 0, ctypes.c_void_p(ws.data_ptr() + 8),
                             need, st) == fa.FA_ERR_WORKSPACE
    assert lib.fa_fwd_f16_ws(p(q), p(k), p(v), p(o), b, h, s, 128, 1, 0, ctypes.c_void_p(ws.data_ptr() + 16),
                             need, st) == fa.FA_OK
    torch.cuda.synchronize()
    assert torch.equal(o, fa.flash_attention_fwd(q, k, v, True))
