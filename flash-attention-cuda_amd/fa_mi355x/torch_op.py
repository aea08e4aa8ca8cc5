"""PyTorch custom operator for the MI355X forward kernel (SURVEY.md §8(f)
rank 3: the wrapper that puts the kernel beside PyTorch SDPA on one box).

    import fa_mi355x.torch_op  # registers torch.ops.fa_mi355x.fwd
    o = torch.ops.fa_mi355x.fwd(q, k, v, causal=True)

``q, k, v``: fp16 or bf16 ``[B, H, S, D]`` (D = 128 or 64) tensors on the GPU (BHSD, the
reference layout, flash_attention.cu:119-122); returns a new tensor of the same shape and dtype.
The schema is defined with ``torch.library.Library`` and the kernel registered
for the CUDA dispatch key directly (``custom_op``'s extra dispatch layers cost
3.7 us more per call than this registration, 12.2 vs 8.5 us host time on a
short launch, tools/host_overhead.py); a fake (meta) implementation supplies
the output shape, so the op is opaque to ``torch.compile``, and it launches on
the current HIP stream, so it can be captured in a HIP graph.  It calls the
same C ABI as every other entry point; there is no CPU or eager fallback (a
CPU tensor raises ValueError).  Forward only: the Autograd key falls through
(no Python frame on the call path) and the GPU and fake kernels raise when a
gradient would be needed (q, k or v requiring grad with grad mode on)
instead of returning an output that backward would silently ignore.
"""
from __future__ import annotations

import torch

from . import flash_attention_fwd

OP_NAME = "fa_mi355x::fwd"

_LIB = torch.library.Library("fa_mi355x", "DEF")
_LIB.define("fwd(Tensor q, Tensor k, Tensor v, bool causal=False) -> Tensor")


def _no_grad_needed(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor) -> None:
    if torch.is_grad_enabled() and (q.requires_grad or k.requires_grad or v.requires_grad):
        raise RuntimeError("fa_mi355x::fwd is forward-only (no backward): call it under "
                           "torch.no_grad() / inference_mode or on tensors that do not require grad")


def _fwd_gpu(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = False) -> torch.Tensor:
    _no_grad_needed(q, k, v)
    return flash_attention_fwd(q.contiguous(), k.contiguous(), v.contiguous(), causal=causal)


def _fwd_cpu(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = False) -> torch.Tensor:
    raise ValueError("fa_mi355x::fwd needs GPU tensors (no CPU path)")


def _fwd_fake(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = False) -> torch.Tensor:
    _no_grad_needed(q, k, v)
    torch._check(q.dim() == 4 and q.shape[-1] in (64, 128), lambda: "expected [B, H, S, 64|128]")
    torch._check(q.dtype in (torch.float16, torch.bfloat16), lambda: "expected fp16 or bf16")
    return torch.empty_like(q, memory_format=torch.contiguous_format)


_LIB.impl("fwd", _fwd_gpu, "CUDA")
_LIB.impl("fwd", torch.library.fallthrough_kernel, "Autograd")
_LIB.impl("fwd", _fwd_cpu, "CPU")
torch.library.register_fake(OP_NAME, _fwd_fake, lib=_LIB)

fwd = torch.ops.fa_mi355x.fwd
