"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper of libfa_oracle.so.

Restates the reference's cpu_attention (flash_attention.cu:668-697) and its
srand(42) input generator (:764-769).  Arrays are numpy uint16 holding IEEE
binary16 bit patterns, layout BHSD.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_LIB = os.path.join(_HERE, "libfa_oracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return ORACLE_LIB


def load() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_LIB):
            build()
        lib = ctypes.CDLL(ORACLE_LIB)
        vp, i = ctypes.c_void_p, ctypes.c_int
        lib.fa_oracle_gen_inputs.argtypes = [vp, vp, vp, ctypes.c_size_t, ctypes.c_uint]
        lib.fa_oracle_gen_inputs.restype = None
        lib.fa_oracle_attention.argtypes = [vp, vp, vp, vp, i, i, i, i, i, i]
        lib.fa_oracle_attention.restype = None
        lib.fa_oracle_attention_heads.argtypes = [vp, vp, vp, vp, i, i, i, i, i, i]
        lib.fa_oracle_attention_heads.restype = None
        lib.fa_oracle_attention_rows.argtypes = [vp, vp, vp, vp, i, i, i, vp, i, i]
        lib.fa_oracle_attention_rows.restype = None
        lib.fa_oracle_max_abs_diff.argtypes = [vp, vp, ctypes.c_size_t]
        lib.fa_oracle_max_abs_diff.restype = ctypes.c_float
        lib.fa_oracle_f32_to_f16.argtypes = [ctypes.c_float]
        lib.fa_oracle_f32_to_f16.restype = ctypes.c_uint16
        lib.fa_oracle_f16_to_f32.argtypes = [ctypes.c_uint16]
        lib.fa_oracle_f16_to_f32.restype = ctypes.c_float
        _lib = lib
    return _lib


def _p(a: np.ndarray) -> ctypes.c_void_p:
    assert a.flags["C_CONTIGUOUS"]
    return ctypes.c_void_p(a.ctypes.data)


def gen_inputs(batch: int, heads: int, seq_len: int, head_dim: int = 128, seed: int = 42):
    """Reference generator: srand(seed); per index draw Q, K, V (uint16 fp16 bits)."""
    n = batch * heads * seq_len * head_dim
    q = np.empty(n, np.uint16)
    k = np.empty(n, np.uint16)
    v = np.empty(n, np.uint16)
    load().fa_oracle_gen_inputs(_p(q), _p(k), _p(v), n, seed)
    shape = (batch, heads, seq_len, head_dim)
    return q.reshape(shape), k.reshape(shape), v.reshape(shape)


def attention(q, k, v, causal: bool, threads: int = 0) -> np.ndarray:
    """cpu_attention on full BHSD tensors; returns uint16 fp16 bits."""
    b, h, s, d = q.shape
    q, k, v = (np.ascontiguousarray(x, dtype=np.uint16) for x in (q, k, v))
    o = np.empty_like(q)
    threads = threads or max(1, min(os.cpu_count() or 1, 16))
    load().fa_oracle_attention(_p(q), _p(k), _p(v), _p(o), b, h, s, d, int(causal), threads)
    return o


def attention_heads(q, k, v, bh_begin: int, bh_end: int, causal: bool, threads: int = 0):
    """cpu_attention restricted to flat heads [bh_begin, bh_end); other heads of the
    returned array are zero."""
    b, h, s, d = q.shape
    q, k, v = (np.ascontiguousarray(x, dtype=np.uint16) for x in (q, k, v))
    o = np.zeros_like(q)
    threads = threads or max(1, min(os.cpu_count() or 1, 16))
    load().fa_oracle_attention_heads(_p(q), _p(k), _p(v), _p(o), bh_begin, bh_end, s, d,
                                     int(causal), threads)
    return o


def attention_rows(q, k, v, rows, causal: bool, threads: int = 0) -> np.ndarray:
    """cpu_attention for the query rows `rows` of ONE head (q, k, v: [S, D]
    uint16 fp16 bits); returns [len(rows), D].  Each row costs O(S * D), so
    heads far too long for a full pass can be checked by sampling."""
    s, d = q.shape
    q, k, v = (np.ascontiguousarray(x, dtype=np.uint16) for x in (q, k, v))
    r = np.ascontiguousarray(rows, dtype=np.int32)
    assert r.ndim == 1 and r.size > 0 and r.min() >= 0 and r.max() < s
    o = np.empty((r.size, d), np.uint16)
    threads = threads or max(1, min(os.cpu_count() or 1, 16))
    load().fa_oracle_attention_rows(_p(q), _p(k), _p(v), _p(o), s, d, int(causal), _p(r), r.size,
                                    threads)
    return o


def f16_bits_to_f32(a: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.uint16).view(np.float16).astype(np.float32)


def max_abs_diff(a: np.ndarray, b: np.ndarray) -> float:
    """Reference metric (:781-784) over fp16 bit arrays."""
    a = np.ascontiguousarray(a, dtype=np.uint16).ravel()
    b = np.ascontiguousarray(b, dtype=np.uint16).ravel()
    assert a.size == b.size
    return float(load().fa_oracle_max_abs_diff(_p(a), _p(b), a.size))
