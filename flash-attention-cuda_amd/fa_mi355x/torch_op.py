"""PyTorch custom operator for the MI355X forward kernel (SURVEY.md §8(f)
rank 3: the wrapper that puts the kernel beside PyTorch SDPA on one box).

    import fa_mi355x.torch_op  # registers torch.ops.fa_mi355x.fwd
    o = torch.ops.fa_mi355x.fwd(q, k, v, causal=True)

``q, k, v``: fp16 or bf16 ``[B, H, S, D]`` (D = 128 or 64) tensors on the GPU (BHSD, the
reference layout, flash_attention.cu:119-122); returns a new tensor of the same shape and dtype.  The op is registered with ``torch.library.custom_op`` so it is
opaque to ``torch.compile`` (a fake/meta implementation supplies the output
shape) and launches on the current HIP stream, so it can be captured in a
HIP graph.  It calls the same C ABI as every other entry point; there is no
CPU or eager fallback (a CPU tensor raises).
"""
from __future__ import annotations

import torch

from . import flash_attention_fwd

OP_NAME = "fa_mi355x::fwd"


@torch.library.custom_op(OP_NAME, mutates_args=())
def fwd(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = False) -> torch.Tensor:
    if not (q.is_cuda and k.is_cuda and v.is_cuda):
        raise ValueError("fa_mi355x::fwd needs GPU tensors (no CPU path)")
    return flash_attention_fwd(q.contiguous(), k.contiguous(), v.contiguous(), causal=causal)


@fwd.register_fake
def _fwd_fake(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = False) -> torch.Tensor:
    torch._check(q.dim() == 4 and q.shape[-1] in (64, 128), lambda: "expected [B, H, S, 64|128]")
    torch._check(q.dtype in (torch.float16, torch.bfloat16), lambda: "expected fp16 or bf16")
    return torch.empty_like(q, memory_format=torch.contiguous_format)
