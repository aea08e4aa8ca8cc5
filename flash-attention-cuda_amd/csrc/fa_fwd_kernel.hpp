// fa_fwd_kernel.hpp -- gfx950 (MI355X, CDNA4) fused attention forward tile loop.
//
// Re-designed for 64-lane waves and MFMA, not a translation of the reference's
// mma.sync/ldmatrix kernel (flash_attention.cu:67-554).  What it computes is
// the reference's contract: per (batch*head, query block) one workgroup runs
// QK^T -> online softmax -> PV over key/value tiles and writes O in fp16
// (:103-122 work mapping, :188-334 tile math, :497-553 epilogue).
//
// Structure (per wave = 32 query rows, per workgroup = WAVES*32 rows):
//  * Swapped first product  S^T = K . Q^T  on v_mfma_f32_32x32x16_f16:
//      A = K tile rows from LDS (ds_read_b128), B = Q held in 32 VGPRs.
//    The accumulator puts the query on the lane (q = lane&31) and 16 keys in
//    registers, so the row max / row sum are per-lane scalars plus ONE
//    cross-half exchange (v_permlane32_swap), no LDS, no shuffles.
//  * Second product  O^T = V^T . P^T : P^T is the first product's accumulator
//    converted to fp16 in place (B operand, no lane movement); V^T comes from
//    the row-major V tile in LDS through ds_read_b64_tr_b16 (hardware
//    transpose read) -- the MI355X replacement for ldmatrix.x2.trans (:305-310).
//  * One LDS image layout for K and V: 8-row x 32-column subtiles with a
//    16-byte-chunk XOR (bank-conflict-free for both the b128 row reads and
//    the tr_b16 column reads; see lds_off()).
//  * K/V tiles are register-staged and double-buffered in LDS: the global
//    loads of tile j+1 are issued before tile j's MFMAs and written to the
//    other LDS buffer after them, one barrier per tile (async-STAGE split).
//  * Online softmax in the exp2 domain with the scale folded into one FMA,
//    and a lazy rescale: O and l are rescaled only when some row max grew
//    by more than RESCALE_LOG2 (P is then bounded by 2^RESCALE_LOG2, exact
//    in fp16 range), wave-uniform branch.
//  * Causal: heaviest query blocks launch first (the reference does this
//    only for S < 2048, :103-112, :643-651; here for every length); waves
//    skip key tiles that are entirely above their diagonal.
//  * Non-causal: XCD-aware block remap so the query blocks of one head run
//    on one XCD and share its L2 copy of K/V.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fa {

typedef _Float16 f16;
typedef f16 f16x8 __attribute__((ext_vector_type(8)));
typedef f16 f16x4 __attribute__((ext_vector_type(4)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int HD = 128;           // head_dim (the reference hard-codes 128, :613)
constexpr int ROW_BYTES = HD * 2; // one K/V/Q row in bytes
constexpr float RESCALE_LOG2 = 8.0f;

struct FwdParams {
  const f16* q;
  const f16* k;
  const f16* v;
  f16* o;
  float* part_o;   // split-KV fp32 partial O  [split][bh][S][HD]  (nullptr if unused)
  float* part_ml;  // split-KV (m, l) per row  [split][bh][S][2]
  int seq_len;
  int bh;          // batch * heads
  int nqb;         // query blocks per head
  int num_splits;  // key splits (1 = no split)
  float c;         // scale * log2(e)
  float scale;     // 1/sqrt(head_dim)
};

// Byte offset of 16-byte chunk `ch` (0..15) of row `row` in one [rows][128]
// fp16 tile: 8-row x 32-column subtiles of 512 B, chunk XOR by (row>>2)&3.
__device__ __forceinline__ int lds_off(int row, int ch) {
  return 2048 * (row >> 3) + 512 * (ch >> 2) + 64 * (row & 7) +
         16 * ((ch & 3) ^ ((row >> 2) & 3));
}

__device__ __forceinline__ float max_with_partner(float x) {
  // lanes l and l^32 exchange; r[0] = {x[0..31], x[0..31]}, r[1] = {x[32..63], x[32..63]}
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float sum_with_partner(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

__device__ __forceinline__ f16x4 lds_read_tr(const char* base, int off) {
  typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
  i16x4 t = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + off));
  return __builtin_bit_cast(f16x4, t);
}

// Fill `out` (the key range [kv_lo, kv_hi) of one head) -- the hot loop.
//   WAVES  : 64-lane waves per workgroup (BM = 32*WAVES query rows)
//   BN     : keys per LDS tile (multiple of 32)
//   CAUSAL : top-left aligned causal mask (key j visible to query i iff j <= i)
//   SPLIT  : write unnormalised fp32 O + (m, l) instead of fp16 O
template <int WAVES, int BN, bool CAUSAL, bool SPLIT>
__device__ __forceinline__ void attention_tile_loop(const FwdParams& p, int bh, int qb,
                                                    int split, char* smem) {
  constexpr int NT = WAVES * 64;                 // threads per workgroup
  constexpr int BM = WAVES * 32;
  constexpr int TILE_BYTES = BN * ROW_BYTES;
  constexpr int NCH = (BN * 16) / NT;            // 16-B chunks per thread per tile
  static_assert((BN * 16) % NT == 0, "tile chunks must divide evenly");
  static_assert(BN % 32 == 0, "BN multiple of 32");

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31;
  const int h = lane >> 5;
  const int S = p.seq_len;

  const size_t head_off = (size_t)bh * (size_t)S * HD;
  const f16* __restrict__ Qh = p.q + head_off;
  const f16* __restrict__ Kh = p.k + head_off;
  const f16* __restrict__ Vh = p.v + head_off;

  const int q0 = qb * BM;
  const int qw = q0 + wave * 32;                 // first query row of this wave
  const int qrow = qw + r;                       // this lane's query row

  // key range of this workgroup
  int kv_lo = 0, kv_hi = CAUSAL ? min(q0 + BM, S) : S;
  if constexpr (SPLIT) {
    const int ntot = (kv_hi + BN - 1) / BN;
    const int per = (ntot + p.num_splits - 1) / p.num_splits;
    kv_lo = min(split * per, ntot) * BN;
    kv_hi = min(kv_hi, min((split + 1) * per, ntot) * BN);
  }
  const int ntiles = kv_hi > kv_lo ? (kv_hi - kv_lo + BN - 1) / BN : 0;

  // ---- Q fragments (B operand of S^T = K.Q^T): lane holds Q[qrow][16t+8h .. +7]
  f16x8 qf[8];
  {
    const f16x8* src = reinterpret_cast<const f16x8*>(Qh + (size_t)qrow * HD);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      f16x8 z = {};
      qf[t] = qrow < S ? src[2 * t + h] : z;
    }
  }

  // ---- staging map: chunk (row, ch) handled by this thread for slot i
  // one wave-instruction covers 4 rows x 256 B; lanes 0-7 hit 8 distinct
  // 16-B LDS slots (two rows of opposite parity) -> conflict-free ds_write_b128
  const int st_row0 = 4 * wave + 2 * ((lane >> 5) & 1) + ((lane >> 2) & 1);
  const int st_ch = 4 * ((lane >> 3) & 3) + (lane & 3);
  const int st_goff = st_row0 * HD + st_ch * 8;  // element offset inside a tile

  // ---- LDS read addresses (bytes, relative to a tile image)
  // K row read (A of S^T): row 32c+r, chunk 2t+h -> 8192c + 512(t>>1) + kaddr[t&1]
  const int kaddr0 = lds_off(r, h);
  const int kaddr1 = lds_off(r, 2 + h);
  // V transposed read (A of O^T): group G=lane>>4, i=lane&15=4qq+pp
  //   rows 32c+16s+8m+4h+qq, cols 32e+16(G&1)+4pp -> 8192c+4096s+512e + vaddr[m]
  int vaddr0, vaddr1;
  {
    const int G = lane >> 4, i = lane & 15, qq = i >> 2, pp = i & 3;
    const int base = 64 * (4 * h + qq) + 8 * (pp & 1);
    vaddr0 = base + 16 * ((2 * (G & 1) + (pp >> 1)) ^ (h));
    vaddr1 = 2048 + base + 16 * ((2 * (G & 1) + (pp >> 1)) ^ (2 + h));
  }

  f16x8 kst[NCH], vst[NCH];
  auto issue_loads = [&](int kv_base) {
    const f16* kt = Kh + (size_t)kv_base * HD;
    const f16* vt = Vh + (size_t)kv_base * HD;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int row = st_row0 + 4 * WAVES * i;
      const int off = st_goff + 4 * WAVES * i * HD;
      f16x8 z = {};
      const bool ok = kv_base + row < kv_hi;
      kst[i] = ok ? *reinterpret_cast<const f16x8*>(kt + off) : z;
      vst[i] = ok ? *reinterpret_cast<const f16x8*>(vt + off) : z;
    }
  };
  auto write_lds = [&](int buf) {
    char* kb = smem + buf * 2 * TILE_BYTES;
    char* vb = kb + TILE_BYTES;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int off = lds_off(st_row0 + 4 * WAVES * i, st_ch);
      *reinterpret_cast<f16x8*>(kb + off) = kst[i];
      *reinterpret_cast<f16x8*>(vb + off) = vst[i];
    }
  };

  f32x16 acc[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) acc[e] = f32x16{};
  float m_run = -__builtin_inff();
  float l_run = 0.f;
  const float c = p.c;

  if (ntiles > 0) {
    issue_loads(kv_lo);
    write_lds(0);
  }
  __syncthreads();

  for (int j = 0; j < ntiles; ++j) {
    const int kv0 = kv_lo + j * BN;
    const int buf = j & 1;
    const bool has_next = j + 1 < ntiles;
    if (has_next) issue_loads(kv0 + BN);

    // wave-uniform: does any key of this tile lie at/below some row of this wave?
    const bool active = !CAUSAL || (kv0 <= qw + 31);
    if (active) {
      const char* kb = smem + buf * 2 * TILE_BYTES;
      const char* vb = kb + TILE_BYTES;

      // ---- S^T = K . Q^T  (BN/32 accumulators of 32 keys x 32 queries)
      f32x16 s[BN / 32];
#pragma unroll
      for (int cb = 0; cb < BN / 32; ++cb) s[cb] = f32x16{};
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int ka = ((t & 1) ? kaddr1 : kaddr0) + 512 * (t >> 1);
#pragma unroll
        for (int cb = 0; cb < BN / 32; ++cb) {
          const f16x8 kf = *reinterpret_cast<const f16x8*>(kb + ka + 8192 * cb);
          s[cb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf, qf[t], s[cb], 0, 0, 0);
        }
      }

      // ---- mask (only tiles that cross the diagonal or the sequence end)
      const bool need_mask = (kv0 + BN > kv_hi) || (CAUSAL && kv0 + BN - 1 > qw);
      if (need_mask) {
#pragma unroll
        for (int cb = 0; cb < BN / 32; ++cb) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int kv = kv0 + 32 * cb + (i & 3) + 8 * (i >> 2) + 4 * h;
            const bool ok = kv < kv_hi && (!CAUSAL || kv <= qrow);
            s[cb][i] = ok ? s[cb][i] : -__builtin_inff();
          }
        }
      }

      // ---- online softmax (exp2 domain, lazy rescale)
      float mx = s[0][0];
#pragma unroll
      for (int cb = 0; cb < BN / 32; ++cb)
#pragma unroll
        for (int i = (cb == 0 ? 1 : 0); i < 16; ++i) mx = fmaxf(mx, s[cb][i]);
      mx = max_with_partner(mx);
      const float m_new = fmaxf(m_run, mx);
      if (__any((m_new - m_run) * c > RESCALE_LOG2)) {
        const float alpha = __builtin_amdgcn_exp2f((m_run - m_new) * c);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] *= alpha;
        l_run *= alpha;
        m_run = m_new;
      }
      // m_run stays -inf only for a row with no visible key yet: keep P = 0, not NaN
      const float mc = m_run == -__builtin_inff() ? 0.f : m_run * c;

      f16x8 pf[BN / 16];
      float lsum = 0.f;
#pragma unroll
      for (int cb = 0; cb < BN / 32; ++cb) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(s[cb][i], c, -mc));
          lsum += pv;
          pf[2 * cb + (i >> 3)][i & 7] = (f16)pv;
        }
      }
      l_run += lsum;

      // ---- O^T += V^T . P^T
#pragma unroll
      for (int u = 0; u < BN / 16; ++u) {
        const int cb = u >> 1, sb = u & 1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int imm = 8192 * cb + 4096 * sb + 512 * e;
          const f16x4 lo = lds_read_tr(vb, vaddr0 + imm);
          const f16x4 hi = lds_read_tr(vb, vaddr1 + imm);
          const f16x8 vf = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
          acc[e] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf, pf[u], acc[e], 0, 0, 0);
        }
      }
    }

    if (has_next) write_lds(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: lane holds O^T[d = 32e + (i&3) + 8(i>>2) + 4h][q = qrow]
  if constexpr (!SPLIT) {
    const float lt = sum_with_partner(l_run);
    const float inv = lt > 0.f ? 1.0f / lt : 0.f;
    if (qrow < S) {
      f16* orow = p.o + head_off + (size_t)qrow * HD;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          f16x4 w;
#pragma unroll
          for (int x = 0; x < 4; ++x) w[x] = (f16)(acc[e][4 * g + x] * inv);
          *reinterpret_cast<f16x4*>(orow + 32 * e + 8 * g + 4 * h) = w;
        }
      }
    }
  } else {
    const float lt = sum_with_partner(l_run);
    if (qrow < S) {
      const size_t prow = ((size_t)split * p.bh + bh) * (size_t)S + qrow;
      float* po = p.part_o + prow * HD;
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float4 w = make_float4(acc[e][4 * g + 0], acc[e][4 * g + 1], acc[e][4 * g + 2],
                                 acc[e][4 * g + 3]);
          *reinterpret_cast<float4*>(po + 32 * e + 8 * g + 4 * h) = w;
        }
      if (h == 0) {
        // m in the reference's units (scaled score = m_run*scale, ref m_i);
        // an empty split writes (-inf, 0)
        float2 ml = make_float2(lt > 0.f ? m_run * p.scale : -__builtin_inff(), lt);
        *reinterpret_cast<float2*>(p.part_ml + prow * 2) = ml;
      }
    }
  }
}

}  // namespace fa
