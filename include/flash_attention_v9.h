/*
 * flash_attention_v9.h -- the reference's host launch signature, kept verbatim
 * in meaning so reference callers recompile unchanged against the MI355X
 * library (C++ linkage, like the original).
 *
 * Reference: void flash_attention_v9_dispatch(const half* Q, const half* K,
 *   const half* V, half* Output, float* splitk_buf_O, float* splitk_buf_ml,
 *   int batch_size, int num_heads, int seq_len, int head_dim, bool causal,
 *   cudaStream_t stream = 0)   (/root/reference/flash_attention.cu:606-611)
 *
 * Semantics kept: device pointers owned by the caller, BHSD fp16, scale =
 * 1/sqrt(head_dim), asynchronous on `stream`, returns void, and on any error
 * prints "HIP error at <file>:<line>: <msg>" and exit(EXIT_FAILURE) exactly
 * as CUDA_CHECK(cudaGetLastError()) does (:22-30, :662).
 * splitk_buf_O / splitk_buf_ml: accepted and ignored, as in the reference
 * (its dispatcher never launches the split-K path; callers pass nullptr,
 * :777).  Split-KV is the explicit C entry fa_fwd_f16_splitkv (fa_mi355x.h),
 * which takes the split count and the buffers explicitly.
 * Tiers: the same as the workspace entries (fa_fwd_f16_ws): the wrapper keeps
 * one zero-filled device workspace per (device, stream) for the causal split
 * tier and the W4 tail pool, allocated on the first call that needs one and
 * grown outside graph capture only (a call captured before it exists runs
 * the workspace-free tiers of fa_fwd_f16).  The reference allocates nothing
 * here; this is the one host-side state besides the kernels' LDS attribute.
 */
#ifndef FLASH_ATTENTION_V9_H
#define FLASH_ATTENTION_V9_H

#include <hip/hip_fp16.h> /* `half` (the cuda_fp16.h type the reference uses) */
#include <hip/hip_runtime.h>

void flash_attention_v9_dispatch(const half* Q, const half* K, const half* V, half* Output,
                                 float* splitk_buf_O, float* splitk_buf_ml, int batch_size,
                                 int num_heads, int seq_len, int head_dim, bool causal,
                                 hipStream_t stream = 0);

#endif /* FLASH_ATTENTION_V9_H */
