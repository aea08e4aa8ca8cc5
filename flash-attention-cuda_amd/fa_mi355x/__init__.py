"""fa_mi355x -- Python host side of the MI355X flash-attention forward path.

A thin ctypes binding over the C ABI in ``include/fa_mi355x.h`` (the drop-in
for the reference's ``flash_attention_v9_dispatch``,
/root/reference/flash_attention.cu:606-663).  PyTorch supplies device memory
and the current HIP stream; all arithmetic runs in the hand-written gfx950
kernels of ``libfa_mi355x.so``.  There is no fallback: if the library is
missing, every entry point raises :class:`FlashAttentionError`.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import List, Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
# FA_MI355X_LIB: another in-tree build of the library (experiment variants,
# tools/w4_variant.sh) for a test or tool run; default the product library
LIB_PATH = os.environ.get("FA_MI355X_LIB") or os.path.join(PKG_ROOT, "lib", "libfa_mi355x.so")

HEAD_DIM = 128

FA_OK = 0
FA_ERR_NULL_POINTER = 1
FA_ERR_UNSUPPORTED_HEAD_DIM = 2
FA_ERR_BAD_SHAPE = 3
FA_ERR_LAUNCH = 4
FA_ERR_BAD_CONFIG = 5
FA_ERR_HIP = 6
FA_ERR_WORKSPACE = 7

# every symbol include/fa_mi355x.h declares (tests check the .so exports them)
FA_DTYPE_F16 = 0
FA_DTYPE_BF16 = 1

EXPORTED_SYMBOLS = (
    "fa_fwd_f16",
    "fa_fwd_f16_config",
    "fa_fwd_bf16",
    "fa_fwd_bf16_config",
    "fa_fwd_f16_splitkv",
    "fa_splitkv_num_splits",
    "fa_splitkv_o_bytes",
    "fa_splitkv_ml_bytes",
    "fa_fwd_f16_ws",
    "fa_fwd_bf16_ws",
    "fa_fwd_ws_bytes",
    "fa_fwd_split_pieces",
    "fa_select_config",
    "fa_num_configs",
    "fa_config_info",
    "fa_kernel_attrs",
    "fa_status_string",
    "fa_version",
)


class FlashAttentionError(RuntimeError):
    """Raised for a nonzero fa_status_t (the reference exit()s instead)."""

    def __init__(self, status: int, msg: str):
        super().__init__(f"fa_mi355x error {status}: {msg}")
        self.status = status


class _ConfigInfo(ctypes.Structure):
    _fields_ = [
        ("id", ctypes.c_int),
        ("block_m", ctypes.c_int),
        ("block_n", ctypes.c_int),
        ("waves", ctypes.c_int),
        ("causal", ctypes.c_int),
        ("split_kv", ctypes.c_int),
        ("lds_bytes", ctypes.c_int),
        ("name", ctypes.c_char_p),
        ("dtype", ctypes.c_int),
        ("head_dim", ctypes.c_int),
    ]


class _KernelAttrs(ctypes.Structure):
    _fields_ = [
        ("num_regs", ctypes.c_int),
        ("local_size_bytes", ctypes.c_int),
        ("shared_size_bytes", ctypes.c_int),
        ("max_threads_per_block", ctypes.c_int),
        ("blocks_per_cu", ctypes.c_int),
    ]


@dataclass(frozen=True)
class TileConfig:
    id: int
    block_m: int
    block_n: int
    waves: int
    causal: bool
    split_kv: bool
    lds_bytes: int
    name: str
    dtype: str = "float16"  # element type of Q/K/V/O: "float16" or "bfloat16"
    head_dim: int = 128


_lib = None


def library_path() -> str:
    return LIB_PATH


def load_library() -> ctypes.CDLL:
    """Load libfa_mi355x.so (in-tree build). Raises loudly when absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FlashAttentionError(
            FA_ERR_HIP,
            f"{LIB_PATH} not built (run `make -C {PKG_ROOT}` or __graft_entry__.build())",
        )
    lib = ctypes.CDLL(LIB_PATH)
    vp, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_float)
    ull = ctypes.c_ulonglong
    lib.fa_fwd_f16.argtypes = [vp, vp, vp, vp, i, i, i, i, i, vp]
    lib.fa_fwd_f16.restype = i
    lib.fa_fwd_f16_config.argtypes = [vp, vp, vp, vp, i, i, i, i, i, i, vp]
    lib.fa_fwd_f16_config.restype = i
    lib.fa_fwd_bf16.argtypes = [vp, vp, vp, vp, i, i, i, i, i, vp]
    lib.fa_fwd_bf16.restype = i
    lib.fa_fwd_bf16_config.argtypes = [vp, vp, vp, vp, i, i, i, i, i, i, vp]
    lib.fa_fwd_bf16_config.restype = i
    lib.fa_fwd_f16_splitkv.argtypes = [vp, vp, vp, vp, i, i, i, i, i, i, vp, vp, vp]
    lib.fa_fwd_f16_splitkv.restype = i
    lib.fa_splitkv_num_splits.argtypes = [i, i, i, i]
    lib.fa_splitkv_num_splits.restype = i
    lib.fa_splitkv_o_bytes.argtypes = [i, i, i, i, i]
    lib.fa_splitkv_o_bytes.restype = ull
    lib.fa_splitkv_ml_bytes.argtypes = [i, i, i, i, i]
    lib.fa_splitkv_ml_bytes.restype = ull
    lib.fa_fwd_f16_ws.argtypes = [vp, vp, vp, vp, i, i, i, i, i, i, vp, ull, vp]
    lib.fa_fwd_f16_ws.restype = i
    lib.fa_fwd_bf16_ws.argtypes = [vp, vp, vp, vp, i, i, i, i, i, i, vp, ull, vp]
    lib.fa_fwd_bf16_ws.restype = i
    lib.fa_fwd_ws_bytes.argtypes = [i, i, i, i, i, i]
    lib.fa_fwd_ws_bytes.restype = ull
    lib.fa_fwd_split_pieces.argtypes = [i, i, i, i, i]
    lib.fa_fwd_split_pieces.restype = i
    lib.fa_select_config.argtypes = [i, i, i, i]
    lib.fa_select_config.restype = i
    lib.fa_num_configs.argtypes = []
    lib.fa_num_configs.restype = i
    lib.fa_config_info.argtypes = [i, ctypes.POINTER(_ConfigInfo)]
    lib.fa_config_info.restype = i
    lib.fa_kernel_attrs.argtypes = [i, ctypes.POINTER(_KernelAttrs)]
    lib.fa_kernel_attrs.restype = i
    lib.fa_status_string.argtypes = [i]
    lib.fa_status_string.restype = ctypes.c_char_p
    lib.fa_version.argtypes = []
    lib.fa_version.restype = ctypes.c_char_p
    del f
    _lib = lib
    return lib


def _check(status: int) -> None:
    if status != FA_OK:
        msg = load_library().fa_status_string(status).decode()
        raise FlashAttentionError(status, msg)


def version() -> str:
    return load_library().fa_version().decode()


def configs() -> List[TileConfig]:
    lib = load_library()
    out = []
    for cid in range(lib.fa_num_configs()):
        ci = _ConfigInfo()
        _check(lib.fa_config_info(cid, ctypes.byref(ci)))
        out.append(
            TileConfig(ci.id, ci.block_m, ci.block_n, ci.waves, bool(ci.causal),
                       bool(ci.split_kv), ci.lds_bytes, ci.name.decode(),
                       "bfloat16" if ci.dtype == FA_DTYPE_BF16 else "float16", ci.head_dim)
        )
    return out


def select_config(batch: int, heads: int, seq_len: int, causal: bool) -> int:
    return load_library().fa_select_config(batch, heads, seq_len, int(bool(causal)))


def kernel_attrs(config_id: int) -> dict:
    ka = _KernelAttrs()
    _check(load_library().fa_kernel_attrs(config_id, ctypes.byref(ka)))
    return {f: getattr(ka, f) for f, _ in _KernelAttrs._fields_}


_DTYPES_16 = ()  # (torch.float16, torch.bfloat16) once torch is imported (lazily)


def _stream_handle(stream, device=None) -> Optional[int]:
    """Raw hipStream_t of `stream` (None: torch's current stream on `device`)."""
    import torch

    if stream is None:
        stream = torch.cuda.current_stream(device)
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


def _check_qkvo(q, k, v, out):
    """Raise FlashAttentionError unless q, k, v, out are contiguous [B,H,S,D]
    device tensors of one 16-bit dtype, shape and device.  The common case is
    one short-circuit expression (a short launch's host cost is mostly this
    wrapper, tools/host_overhead.py); the per-tensor loop names the culprit."""
    global _DTYPES_16
    if not _DTYPES_16:
        import torch

        _DTYPES_16 = (torch.float16, torch.bfloat16)
    dt, sh, dv = q.dtype, q.shape, q.device
    if (q.is_cuda and len(sh) == 4 and dt in _DTYPES_16 and k.dtype is dt and v.dtype is dt
            and out.dtype is dt and k.shape == sh and v.shape == sh and out.shape == sh
            and k.device == dv and v.device == dv and out.device == dv and q.is_contiguous()
            and k.is_contiguous() and v.is_contiguous() and out.is_contiguous()):
        return
    _check_qkvo_each(q, k, v, out)


def _check_qkvo_each(q, k, v, out):
    import torch

    if q.dtype not in (torch.float16, torch.bfloat16):
        raise FlashAttentionError(FA_ERR_BAD_SHAPE, f"q must be float16 or bfloat16, got {q.dtype}")
    for name, t in (("q", q), ("k", k), ("v", v), ("out", out)):
        if t.dtype != q.dtype:
            raise FlashAttentionError(FA_ERR_BAD_SHAPE, f"{name} must be {q.dtype}, got {t.dtype}")
        if not t.is_cuda:
            raise FlashAttentionError(FA_ERR_NULL_POINTER, f"{name} must be a device tensor")
        if not t.is_contiguous():
            raise FlashAttentionError(FA_ERR_BAD_SHAPE, f"{name} must be contiguous (BHSD)")
        if t.dim() != 4 or t.shape != q.shape:
            raise FlashAttentionError(FA_ERR_BAD_SHAPE, f"{name} must be [B,H,S,D] like q")
        if t.device != q.device:
            raise FlashAttentionError(FA_ERR_BAD_SHAPE,
                                      f"{name} is on {t.device}, q on {q.device}: one device only")


_WS_NEED = {}  # (device, B, H, S, D, causal, piece_tiles) -> workspace bytes (fa_fwd_ws_bytes)
_WS_BUF = {}   # (device, stream) -> zero-filled uint8 workspace, kept for the process


def workspace_bytes(batch: int, heads: int, seq_len: int, head_dim: int, causal: bool,
                    device=None, piece_tiles: int = 0) -> int:
    """Workspace the split tier needs for this call on `device` (0: no split);
    piece_tiles as in :func:`flash_attention_fwd`."""
    import torch

    dev = torch.cuda.current_device() if device is None else torch.device(device).index
    key = (dev, batch, heads, seq_len, head_dim, bool(causal), int(piece_tiles))
    n = _WS_NEED.get(key)
    if n is None:
        with torch.cuda.device(dev):
            n = load_library().fa_fwd_ws_bytes(batch, heads, seq_len, head_dim, int(bool(causal)),
                                               int(piece_tiles))
        _WS_NEED[key] = n
    return n


def _workspace(nbytes: int, dev: int, st: int):
    """A zero-filled workspace of >= nbytes for launches on stream `st` of
    device `dev`, from torch's caching allocator, reused by every later launch
    on that stream (each launch leaves it reusable: fa_mi355x.h).  Under HIP
    graph capture a fresh one is captured with its zero fill instead."""
    import torch

    if torch.cuda.is_current_stream_capturing():
        return torch.zeros(nbytes, dtype=torch.uint8, device=dev)
    buf = _WS_BUF.get((dev, st))
    if buf is None or buf.numel() < nbytes:
        if buf is not None:
            torch.cuda.synchronize(dev)  # launches enqueued on the old one are done
        buf = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
        torch.cuda.current_stream(dev).synchronize()  # the fill lands before any stream uses it
        _WS_BUF[(dev, st)] = buf
    return buf


def flash_attention_fwd(q, k, v, causal: bool = False, out=None, config: Optional[int] = None,
                        stream=None, piece_tiles: int = 0):
    """O = softmax(Q K^T / sqrt(D) [+ causal mask]) V for fp16 or bf16 BHSD tensors.

    q, k, v: [batch, heads, seq_len, D] float16 (the reference's type) or
    bfloat16 contiguous device tensors, all of one dtype; D = 128 (the
    reference's head_dim) or 64.
    config: force a tile config id (see :func:`configs`); default = dispatcher,
    which for long causal launches short of the persistent tier splits query
    blocks' key ranges across workgroups through a workspace from torch's
    caching allocator (fa_fwd_*_ws; :func:`workspace_bytes`).
    piece_tiles > 0 (causal, head_dim 128, config None): force that split
    piece length in 64-key tiles.
    Enqueued on ``stream`` (default: torch's current stream); no sync.
    """
    import torch

    if out is None:
        out = torch.empty_like(q)
    _check_qkvo(q, k, v, out)
    b, h, s, d = q.shape
    lib = _lib or load_library()
    bf16 = q.dtype is torch.bfloat16
    dev = q.device.index
    if stream is None:
        st = torch._C._cuda_getCurrentRawStream(dev)
    else:
        st = stream if isinstance(stream, int) else stream.cuda_stream
    args = (q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), b, h, s, d, int(bool(causal)))
    if config is None:
        need = _WS_NEED.get((dev, b, h, s, d, bool(causal), piece_tiles))
        if need is None:
            need = workspace_bytes(b, h, s, d, causal, device=q.device, piece_tiles=piece_tiles)
        if need or piece_tiles:
            fn = lib.fa_fwd_bf16_ws if bf16 else lib.fa_fwd_f16_ws
            args += (int(piece_tiles), _workspace(need, dev, st).data_ptr() if need else None, need)
        else:
            fn = lib.fa_fwd_bf16 if bf16 else lib.fa_fwd_f16
    else:
        fn = lib.fa_fwd_bf16_config if bf16 else lib.fa_fwd_f16_config
        args += (int(config),)
    # the C side launches on (and sizes for) the current device: make it q's
    if dev == torch._C._cuda_getDevice():
        rc = fn(*args, st)
    else:
        with torch.cuda.device(dev):
            rc = fn(*args, st)
    _check(rc)
    return out


def splitkv_buffers(batch: int, heads: int, seq_len: int, num_splits: int, device="cuda"):
    """Allocate the reference-layout split-K buffers (O partials, (m,l))."""
    import torch

    rows = batch * heads * seq_len
    part_o = torch.empty(num_splits * rows * HEAD_DIM, dtype=torch.float32, device=device)
    part_ml = torch.empty(num_splits * rows * 2, dtype=torch.float32, device=device)
    return part_o, part_ml


def flash_attention_fwd_splitkv(q, k, v, causal: bool = False, num_splits: int = 0, out=None,
                                part_o=None, part_ml=None, stream=None):
    """Split-KV forward + log-sum-exp merge (ref split-K path, :169-180/:559-598)."""
    import torch

    # the split-KV entry is fp16-only (fa_fwd_f16_splitkv takes untyped
    # pointers, as the reference's half* split-K path does, :606-611): a bf16
    # tensor would be read as fp16 bits, so reject it before anything else
    if q.dtype != torch.float16:
        raise FlashAttentionError(FA_ERR_BAD_SHAPE,
                                  f"split-KV takes float16 tensors only, got {q.dtype}")
    if out is None:
        out = torch.empty_like(q)
    _check_qkvo(q, k, v, out)
    b, h, s, d = q.shape
    lib = load_library()
    if num_splits <= 0:
        num_splits = lib.fa_splitkv_num_splits(b, h, s, int(bool(causal)))
    if part_o is None or part_ml is None:
        part_o, part_ml = splitkv_buffers(b, h, s, num_splits, device=q.device)
    need_o = lib.fa_splitkv_o_bytes(b, h, s, d, num_splits)
    need_ml = lib.fa_splitkv_ml_bytes(b, h, s, d, num_splits)
    if part_o.numel() * 4 < need_o or part_ml.numel() * 4 < need_ml:
        raise FlashAttentionError(FA_ERR_WORKSPACE, "split-KV buffers too small")
    for name, t in (("part_o", part_o), ("part_ml", part_ml)):
        if t.device != q.device or t.dtype != torch.float32 or not t.is_contiguous():
            raise FlashAttentionError(FA_ERR_WORKSPACE,
                                      f"{name} must be contiguous float32 on {q.device}")
    with torch.cuda.device(q.device):
        st = ctypes.c_void_p(_stream_handle(stream, q.device))
        _check(lib.fa_fwd_f16_splitkv(
            ctypes.c_void_p(q.data_ptr()), ctypes.c_void_p(k.data_ptr()),
            ctypes.c_void_p(v.data_ptr()), ctypes.c_void_p(out.data_ptr()), b, h, s, d,
            int(bool(causal)), int(num_splits), ctypes.c_void_p(part_o.data_ptr()),
            ctypes.c_void_p(part_ml.data_ptr()), st))
    return out


def flash_attention_v9_dispatch(Q, K, V, Output, splitk_buf_O, splitk_buf_ml, batch_size: int,
                                num_heads: int, seq_len: int, head_dim: int, causal: bool,
                                stream=0):
    """Mirror of the reference host launch signature (flash_attention.cu:606-611).

    Q/K/V/Output are device tensors (or raw device pointers as ints) holding
    BHSD fp16 data on the current device.  splitk_buf_O/splitk_buf_ml are
    accepted and ignored, as the reference's dispatcher ignores them (it only
    launches split_k = 1; split-KV is :func:`flash_attention_fwd_splitkv`).
    Raises FlashAttentionError where the reference would exit(EXIT_FAILURE).
    """
    del splitk_buf_O, splitk_buf_ml

    # the reference's boundary is typed half* (:606-611): tensors must be
    # float16 (raw pointers cannot be checked and are taken as fp16 BHSD)
    for name, x in (("Q", Q), ("K", K), ("V", V), ("Output", Output)):
        if not isinstance(x, int):
            import torch

            if x.dtype != torch.float16:
                raise FlashAttentionError(FA_ERR_BAD_SHAPE, f"{name} must be float16, got {x.dtype}")

    def ptr(x):
        return x if isinstance(x, int) else x.data_ptr()

    lib = load_library()
    st = ctypes.c_void_p(_stream_handle(stream) if stream not in (0, None) else None)
    q, k, v, o = (ctypes.c_void_p(ptr(x)) for x in (Q, K, V, Output))
    _check(lib.fa_fwd_f16(q, k, v, o, batch_size, num_heads, seq_len, head_dim,
                          int(bool(causal)), st))


def attention_flops(batch: int, heads: int, seq_len: int, head_dim: int, causal: bool) -> float:
    """Reference FLOP convention: 4*B*H*S^2*D, halved when causal (:938-939)."""
    f = 4.0 * batch * heads * seq_len * seq_len * head_dim
    return f / 2 if causal else f


def kernel_symbol(config_name: str) -> str:
    """Substring of the kernel symbol rocprofv3 reports for a tile config."""
    if "_asm_persistent" in config_name:
        return "fa_fwd_f16_w4_kernel"
    if "persistent" in config_name:
        return "fa_fwd_f16_persistent_kernel"
    if "kvpair" in config_name or "kvquad" in config_name:
        return "fa_fwd_f16_kvpair_kernel"
    if "splitkv" in config_name:
        return "fa_fwd_f16_splitkv_kernel"
    return "fa_fwd_f16_kernel"
