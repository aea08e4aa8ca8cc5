/*
 * fa_oracle.c -- TEST INFRASTRUCTURE ONLY (see fa_oracle.h).
 *
 * A plain-C restatement of the reference's CPU oracle and input generator.
 * Citations are to /root/reference/flash_attention.cu.
 *
 * Build without -ffast-math / -march=native and with -ffp-contract=off, so the
 * fp32 arithmetic is the same sequence of IEEE operations the reference's
 * host build performs (SURVEY.md §8(c) last paragraph).
 */
#include "fa_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ---- binary16 conversions (cuda_fp16.h __float2half / __half2float) ---- */

uint16_t fa_oracle_f32_to_f16(float f) {
  uint32_t x;
  memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000u;
  const uint32_t absx = x & 0x7fffffffu;
  if (absx >= 0x7f800000u) { /* inf / nan */
    return (uint16_t)(sign | 0x7c00u | (absx > 0x7f800000u ? 0x200u : 0u));
  }
  if (absx >= 0x477ff000u) { /* rounds to >= 65520 -> inf */
    return (uint16_t)(sign | 0x7c00u);
  }
  if (absx < 0x38800000u) { /* result is subnormal or zero in fp16 */
    if (absx < 0x33000000u) return (uint16_t)sign; /* < 2^-25: rounds to 0 */
    const uint32_t e = absx >> 23;                  /* biased f32 exponent */
    const uint32_t mant = (absx & 0x7fffffu) | 0x800000u;
    const uint32_t shift = 126u - e; /* value = mant * 2^(e-150); ulp16 = 2^-24 */
    uint32_t q = mant >> shift;
    const uint32_t rem = mant & ((1u << shift) - 1u);
    const uint32_t half = 1u << (shift - 1u);
    if (rem > half || (rem == half && (q & 1u))) q++;
    return (uint16_t)(sign | q);
  }
  /* normal: rebias exponent, round 13 dropped bits to nearest even */
  uint32_t h = ((absx >> 13) - (112u << 10));
  const uint32_t rem = absx & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
  return (uint16_t)(sign | h);
}

float fa_oracle_f16_to_f32(uint16_t h) {
  const uint32_t sign = ((uint32_t)h & 0x8000u) << 16;
  const uint32_t e = ((uint32_t)h >> 10) & 0x1fu;
  uint32_t m = (uint32_t)h & 0x3ffu;
  uint32_t x;
  if (e == 0) {
    if (m == 0) {
      x = sign;
    } else { /* subnormal: normalise */
      uint32_t ee = 113u;
      while (!(m & 0x400u)) { m <<= 1; ee--; }
      x = sign | (ee << 23) | ((m & 0x3ffu) << 13);
    }
  } else if (e == 31) {
    x = sign | 0x7f800000u | (m << 13);
  } else {
    x = sign | ((e + 112u) << 23) | (m << 13);
  }
  float f;
  memcpy(&f, &x, 4);
  return f;
}

/* ---- input generator: flash_attention.cu:764-769 ---- */

void fa_oracle_gen_inputs(uint16_t* q, uint16_t* k, uint16_t* v, size_t n,
                          unsigned seed) {
  srand(seed);
  for (size_t i = 0; i < n; i++) {
    q[i] = fa_oracle_f32_to_f16((float)rand() / RAND_MAX - 0.5f);
    k[i] = fa_oracle_f32_to_f16((float)rand() / RAND_MAX - 0.5f);
    v[i] = fa_oracle_f32_to_f16((float)rand() / RAND_MAX - 0.5f);
  }
}

/* ---- cpu_attention: flash_attention.cu:668-697, one (b,h) head ---- */

/* rows [row_begin, row_end) of one head; rows are independent, so a head can
   be split over threads without changing any row's operation order.  Row i
   is written at o + (i - o_row0) * head_dim. */
static void attention_rows(const uint16_t* q, const uint16_t* k,
                           const uint16_t* v, uint16_t* o, int o_row0, int seq_len,
                           int head_dim, int causal, int row_begin, int row_end,
                           float* scores, float* qrow) {
  /* :670 scale = 1/sqrtf(head_dim) */
  const float scale = 1.0f / sqrtf((float)head_dim);
  for (int i = row_begin; i < row_end; i++) {
    /* __half2float(q[i*hd+d]) hoisted: same values, same order of use */
    for (int d = 0; d < head_dim; d++)
      qrow[d] = fa_oracle_f16_to_f32(q[(size_t)i * head_dim + d]);
    float max_val = -FLT_MAX;                       /* :678 */
    const int end_j = causal ? i + 1 : seq_len;     /* :679 */
    for (int j = 0; j < end_j; j++) {               /* :680-684 */
      const uint16_t* kj = k + (size_t)j * head_dim;
      float score = 0.0f;
      for (int d = 0; d < head_dim; d++)
        score += qrow[d] * fa_oracle_f16_to_f32(kj[d]);
      score *= scale;
      scores[j] = score;
      max_val = fmaxf(max_val, score);
    }
    float sum = 0.0f;                               /* :686-687 */
    for (int j = 0; j < end_j; j++) {
      scores[j] = expf(scores[j] - max_val);
      sum += scores[j];
    }
    for (int j = 0; j < end_j; j++) scores[j] /= sum; /* :688 */
    for (int d = 0; d < head_dim; d++) {            /* :689-693 */
      float val = 0.0f;
      for (int j = 0; j < end_j; j++)
        val += scores[j] * fa_oracle_f16_to_f32(v[(size_t)j * head_dim + d]);
      o[(size_t)(i - o_row0) * head_dim + d] = fa_oracle_f32_to_f16(val);
    }
  }
}

void fa_oracle_attention_heads(const uint16_t* q, const uint16_t* k,
                               const uint16_t* v, uint16_t* o, int bh_begin,
                               int bh_end, int seq_len, int head_dim,
                               int causal, int n_threads) {
  if (n_threads < 1) n_threads = 1;
  const size_t stride = (size_t)seq_len * head_dim;
  /* work item = (head, 64-row chunk): one head alone still uses every thread */
  const int chunk = 64;
  const int nchunk = (seq_len + chunk - 1) / chunk;
  const long long items = (long long)(bh_end - bh_begin) * nchunk;
#pragma omp parallel num_threads(n_threads)
  {
    float* scores = (float*)malloc((size_t)seq_len * sizeof(float));
    float* qrow = (float*)malloc((size_t)head_dim * sizeof(float));
#pragma omp for schedule(dynamic, 1)
    for (long long it = 0; it < items; it++) {
      /* causal: heaviest (last) chunks first for balance */
      const int bh = bh_begin + (int)(it / nchunk);
      const int c = nchunk - 1 - (int)(it % nchunk);
      const int r1 = (c + 1) * chunk < seq_len ? (c + 1) * chunk : seq_len;
      attention_rows(q + bh * stride, k + bh * stride, v + bh * stride,
                     o + bh * stride, 0, seq_len, head_dim, causal, c * chunk, r1,
                     scores, qrow);
    }
    free(qrow);
    free(scores);
  }
}

/* selected query rows of one head (q, k, v: seq_len x head_dim); o is
   nrows x head_dim, row r = query row rows[r].  For heads too long for a full
   pass (the maximum-size GPU tests): each row costs O(seq_len * head_dim). */
void fa_oracle_attention_rows(const uint16_t* q, const uint16_t* k,
                              const uint16_t* v, uint16_t* o, int seq_len,
                              int head_dim, int causal, const int* rows,
                              int nrows, int n_threads) {
  if (n_threads < 1) n_threads = 1;
#pragma omp parallel num_threads(n_threads)
  {
    float* scores = (float*)malloc((size_t)seq_len * sizeof(float));
    float* qrow = (float*)malloc((size_t)head_dim * sizeof(float));
#pragma omp for schedule(dynamic, 1)
    for (int r = 0; r < nrows; r++)
      attention_rows(q, k, v, o + (size_t)r * head_dim, rows[r], seq_len, head_dim,
                     causal, rows[r], rows[r] + 1, scores, qrow);
    free(qrow);
    free(scores);
  }
}

void fa_oracle_attention(const uint16_t* q, const uint16_t* k,
                         const uint16_t* v, uint16_t* o, int batch,
                         int num_heads, int seq_len, int head_dim, int causal,
                         int n_threads) {
  fa_oracle_attention_heads(q, k, v, o, 0, batch * num_heads, seq_len,
                            head_dim, causal, n_threads);
}

/* ---- metric: flash_attention.cu:781-784 ---- */

float fa_oracle_max_abs_diff(const uint16_t* a, const uint16_t* b, size_t n) {
  float maxdiff = 0.0f;
  for (size_t i = 0; i < n; i++)
    maxdiff = fmaxf(maxdiff, fabsf(fa_oracle_f16_to_f32(a[i]) -
                                   fa_oracle_f16_to_f32(b[i])));
  return maxdiff;
}
