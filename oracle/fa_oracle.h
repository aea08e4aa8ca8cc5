/*
 * fa_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's correctness oracle and input generator
 * (naveedprojects/flash-attention-cuda, flash_attention.cu).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library; the product path (flash-attention-cuda_amd/) never links it.
 *
 * Parity status: pinned against the known-answer values that SURVEY.md §8(c)
 * recorded from the reference's own cpu_attention (H=2, S=64, causal,
 * srand(42): q[0], o[0], sum(o)).  The reference itself is unbuildable here
 * (needs nvcc + cuda_runtime.h/cuda_fp16.h).
 *
 * fp16 values are passed as raw IEEE binary16 bit patterns (uint16_t).
 */
#ifndef FA_ORACLE_H
#define FA_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* IEEE fp32 -> binary16, round-to-nearest-even (== __float2half). */
uint16_t fa_oracle_f32_to_f16(float f);
/* binary16 -> fp32, exact (== __half2float). */
float fa_oracle_f16_to_f32(uint16_t h);

/*
 * Reference input generator (flash_attention.cu:764-769, repeated at
 * :796-801, :828-833, :860-865, :924-929): srand(seed); for every flat index
 * i draw Q[i], then K[i], then V[i], each (half)((float)rand()/RAND_MAX-0.5f).
 * Uses glibc rand(), exactly as the reference host code does.
 */
void fa_oracle_gen_inputs(uint16_t* q, uint16_t* k, uint16_t* v, size_t n,
                          unsigned seed);

/*
 * Restatement of cpu_attention (flash_attention.cu:668-697).
 * Layout BHSD ([batch*heads][seq][head_dim], contiguous).  fp32 dot with
 * sequential d accumulation, *scale, running fmaxf, expf, sum, divide,
 * fp32 P.V accumulation in j order, RNE to fp16.  causal: top-left aligned,
 * key j visible to query i iff j <= i (:679).
 * n_threads > 1 parallelises over (b,h) heads only; per-head arithmetic order
 * is unchanged, so the result is bit-identical for any n_threads.
 */
void fa_oracle_attention(const uint16_t* q, const uint16_t* k,
                         const uint16_t* v, uint16_t* o, int batch,
                         int num_heads, int seq_len, int head_dim, int causal,
                         int n_threads);

/* Same oracle restricted to heads [bh_begin, bh_end) of the flat B*H axis;
 * pointers address the full tensors.  Used for sampled checks at full size. */
void fa_oracle_attention_heads(const uint16_t* q, const uint16_t* k,
                               const uint16_t* v, uint16_t* o, int bh_begin,
                               int bh_end, int seq_len, int head_dim,
                               int causal, int n_threads);

/* Reference metric (flash_attention.cu:781-784): max over i of
 * |half2float(a[i]) - half2float(b[i])|. */
/* selected query rows of one head; o is nrows x head_dim */
void fa_oracle_attention_rows(const uint16_t* q, const uint16_t* k,
                              const uint16_t* v, uint16_t* o, int seq_len,
                              int head_dim, int causal, const int* rows,
                              int nrows, int n_threads);

float fa_oracle_max_abs_diff(const uint16_t* a, const uint16_t* b, size_t n);

#ifdef __cplusplus
}
#endif

#endif /* FA_ORACLE_H */
