// fa_fwd.hip -- kernels, tile-config table, dispatcher and C ABI
// (include/fa_mi355x.h) of the MI355X flash-attention forward path.
//
// Replaces the reference's host dispatcher flash_attention_v9_dispatch and
// its four template instantiations (flash_attention.cu:606-663), plus the
// never-launched split-K path (:169-180, :460-496) and its merge kernel
// flash_attention_splitk_merge (:559-598).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <map>
#include <mutex>

#include "fa_fwd_kernel.hpp"
#include "fa_mi355x.h"

namespace fa {

// ---------------------------------------------------------------------------
// workgroup -> (query block, batch*head)
// ---------------------------------------------------------------------------
// Causal (B*H % 8 == 0): XCD-aware, heaviest-first in "rank bands".  Blocks
// b, b+8, b+16 ... share an XCD (its own L2); XCD x owns heads x, x+8, ...
// and walks them heaviest rank band first, the `band` query blocks of one
// head consecutive inside a band, so co-running blocks on one XCD stream the
// same K/V tiles through its L2 while load balance stays LPT-like.  (The
// reference reverses query blocks for S < 2048 only, :103-112.)
// Otherwise heads are interleaved inside a rank (plain heaviest-first).
// Non-causal: bijective XCD remap -- each XCD gets a contiguous run of
// (head, query block) items, so the query blocks of one head share K/V in L2.
__device__ __forceinline__ void map_block(int id, int nblk, int nqb, int bh_count, int band,
                                          bool causal, int& qb, int& bh) {
  if (causal) {
    if ((bh_count & 7) == 0 && nblk == bh_count * nqb && band > 1) {
      const int x = id & 7, j = id >> 3, hx = bh_count >> 3;
      const int r = min(nqb, band);
      const int full = nqb / r, rl = nqb - full * r;
      int rank, lh;
      if (j < full * hx * r) {
        const int bnd = j / (hx * r), k = j - bnd * hx * r;
        lh = k / r;
        rank = bnd * r + (k - lh * r);
      } else {
        const int k = j - full * hx * r;
        lh = k / rl;
        rank = full * r + (k - lh * rl);
      }
      bh = x + 8 * lh;
      qb = nqb - 1 - rank;
      return;
    }
    const int rank = id / bh_count;
    bh = id - rank * bh_count;
    qb = nqb - 1 - rank;
  } else {
    const int xcd = id & 7, slot = id >> 3;
    const int q8 = nblk >> 3, r8 = nblk & 7;
    const int w = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
    bh = w / nqb;
    qb = w - bh * nqb;
  }
}

// SCHED: 0 = one-barrier-per-tile loop (any wave count), 1 = 8-wave ping-pong
// (MFMA phase at s_setprio 1), 3 = ping-pong with LDS-DMA tile loads into
// three rotating buffers
// BF16: Q/K/V/O and the MFMA operands are bf16
// HDIM: head_dim (128 or 64)
template <int WAVES, int BN, bool CAUSAL, bool SPLIT, int SCHED, bool BF16 = false, int HDIM = 128>
__device__ __forceinline__ void run_tile_loop(const FwdParams& p, int bh, int qb, int split,
                                              char* smem) {
  using Pol = M16<BN, typename std::conditional<BF16, __bf16, f16>::type, HDIM>;
  if constexpr (SCHED == 1 || SCHED == 3) {
    static_assert(WAVES == 8, "ping-pong needs two groups of four waves");
    attention_pingpong<Pol, CAUSAL, SPLIT, true, SCHED == 3>(p, bh, qb, split, smem);
  } else {
    attention_tile_loop<Pol, WAVES, CAUSAL, SPLIT>(p, bh, qb, split, smem);
  }
}

template <int WAVES, int BN, bool CAUSAL, int SCHED, bool BF16 = false, int HDIM = 128>
__global__ __launch_bounds__(WAVES * 64, BN == 128 ? 1 : 2) void fa_fwd_f16_kernel(FwdParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
#ifdef FA_STAMPS
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  const unsigned long long c_start = __builtin_amdgcn_s_memtime();
#endif
  int qb, bh;
  map_block(blockIdx.x, gridDim.x, p.nqb, p.bh, p.band, CAUSAL, qb, bh);
  run_tile_loop<WAVES, BN, CAUSAL, false, SCHED, BF16, HDIM>(p, bh, qb, 0, smem);
#ifdef FA_STAMPS
  if (threadIdx.x == 0 && blockIdx.x < FA_MAX_TIMELINE) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    g_fa_timeline[blockIdx.x][0] = t_start;
    g_fa_timeline[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
    g_fa_timeline[blockIdx.x][3] = __builtin_amdgcn_s_memtime() - c_start;
    g_fa_timeline[blockIdx.x][2] =
        (unsigned long long)hw | ((unsigned long long)xcc << 32) | ((unsigned long long)(qb & 0xFFFF) << 40) |
        ((unsigned long long)(bh & 0xFF) << 56);
  }
#endif
}

// Persistent variant: gridDim = 8 x C workgroups, one per CU.
// Workgroups b, b+8, ... share an XCD; XCD x owns heads x, x+8, ... and walks
// its item list (causal: rank bands of `band` query blocks of one head,
// heaviest band first; non-causal: head-major) in rounds of C items, the
// C workgroups taking a round in snake order (forward on even rounds,
// reversed on odd ones).  Within a band the item costs fall linearly, so the
// snake makes every CU's cost equal over each pair of rounds -- LPT balance
// by construction, with no atomics or per-launch state -- while the items of
// one round (one or two heads' query blocks) co-run on the XCD and share K/V
// through its L2.
__device__ __forceinline__ void xcd_item(int j, int hx, int nqb, int band, bool causal, int& lh,
                                         int& rank) {
  if (!causal) {
    lh = j / nqb;
    rank = j - lh * nqb;
    return;
  }
  const int r = min(nqb, max(band, 1));
  const int full = nqb / r, rl = nqb - full * r;
  if (j < full * hx * r) {
    const int bnd = j / (hx * r), k = j - bnd * hx * r;
    lh = k / r;
    rank = bnd * r + (k - lh * r);
  } else {
    const int k = j - full * hx * r;
    lh = k / rl;
    rank = full * r + (k - lh * rl);
  }
}

// The item list of XCD x (blockIdx & 7) for the persistent kernels.
// Head-affine XCD split when B*H % 8 == 0; otherwise heads do not divide
// over the 8 XCDs (B=1 H=2 would leave 6 of them idle: 343 vs 1000+
// TFLOP/s at S=32768), so XCD x takes every 8th item of the global list
// (causal: rank-major, heaviest first -- a balanced mix) or a contiguous
// 1/8 of it (non-causal: head-major, so runs of one head's query blocks).
template <bool CAUSAL>
struct XcdItems {
  int x, hx, start8, L;
  bool affine;
  __device__ __forceinline__ XcdItems(const FwdParams& p, int x_) : x(x_) {
    affine = (p.bh & 7) == 0;
    const int Lall = p.bh * p.nqb;
    hx = (p.bh - x + 7) >> 3;  // heads h < bh with h % 8 == x
    const int per8 = Lall >> 3, rem8 = Lall & 7;
    L = affine ? hx * p.nqb : (CAUSAL ? (Lall - x + 7) >> 3 : per8 + (x < rem8 ? 1 : 0));
    start8 = x * per8 + min(x, rem8);
  }
  __device__ __forceinline__ void item(const FwdParams& p, int pos, int& bh, int& qb) const {
    if (affine) {
      int lh, rank;
      xcd_item(pos, hx, p.nqb, p.band, CAUSAL, lh, rank);
      bh = x + 8 * lh;
      qb = CAUSAL ? p.nqb - 1 - rank : rank;
    } else if (CAUSAL) {
      const int g = x + 8 * pos, rank = g / p.bh;
      bh = g - rank * p.bh;
      qb = p.nqb - 1 - rank;
    } else {
      const int g = start8 + pos;
      bh = g / p.nqb;
      qb = g - bh * p.nqb;
    }
  }
};

template <int WAVES, int BN, bool CAUSAL, int SCHED, bool BF16 = false, int HDIM = 128>
__global__ __launch_bounds__(WAVES * 64, 2) void fa_fwd_f16_persistent_kernel(
    FwdParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int x = blockIdx.x & 7, lcu = blockIdx.x >> 3, C = gridDim.x >> 3;
  const XcdItems<CAUSAL> items(p, x);
  const int L = items.L;
  auto item_of = [&](int pos, int& bh, int& qb) { items.item(p, pos, bh, qb); };
  // Non-causal tail: items cost the same, so a last round of `tail` <= C/2
  // items would leave C - tail CUs idle (1.5 items per CU: 75 %).  Those
  // items run instead as 2*tail 128-row KV-pair halves on 2*tail CUs.
  constexpr bool kTailSplit = !CAUSAL && SCHED == 1;
  const int full = L / C, tail = L - full * C;
  const bool split_tail = kTailSplit && tail > 0 && 2 * tail <= C;
  // Causal pair order: CU lcu runs the two query blocks (nqb-1-p, p) of one
  // head back to back -- the heavy one in round 2R, the light one in round
  // 2R+1 -- so every CU costs exactly nqb+1 key tiles per pair of rounds and
  // the pairs' heavy items co-start: the XCD's CUs walk one or two heads'
  // K/V tiles in lockstep (heavy items) or as a one-tile-apart staircase
  // (light items), which the 4 MB L2 holds.  The snake over rank bands
  // below balances the same way but mixes heads and ranks in a round, and
  // after the first round its items start staggered (2.2-3.5x the
  // algorithmic HBM bytes at B=1 S=8192-16384, profiles/r01_tier_pmc.txt).
  // Pairs cut that to 1.38-1.39x at equal speed; with many heads per XCD the
  // band-16 snake co-starts whole heads and fetches less (B=64 S=4096: 1.07x
  // vs 1.41x), so pairs replace only the plain heaviest-first order (band 1,
  // <= 64 heads; profiles/r02_causal_pairs_{ab,traffic}.jsonl).
  const bool pairs = CAUSAL && items.affine && (p.nqb & 1) == 0 && p.band == 1;
  // Which block of a pair runs first.  Light first (p, then nqb-1-p): CU p
  // starts its heavy block at key tile 0 when its light one ends, so the
  // XCD's CUs read K/V inside a window of ~4*32 key tiles that L2 holds if
  // it fits (nqb <= 32, S <= 8192: 64 tiles x 32 KB = 2 MB at S=8192, HBM
  // traffic 1.33 -> 1.26x); heavy first otherwise (S=16384: 1.32x vs 1.49x
  // light first; profiles/r02_pair_light_first.jsonl).
  const int light_first = p.nqb <= 32 ? 1 : 0;
  const int npairs = items.hx * (p.nqb >> 1);
  const int rounds = pairs ? 2 * ((npairs + C - 1) / C) : split_tail ? full : (L + C - 1) / C;
  for (int r = 0; r < rounds; ++r) {
    const int pos = pairs ? (r >> 1) * C + lcu : r * C + ((r & 1) ? (C - 1 - lcu) : lcu);
    if (pos < (pairs ? npairs : L)) {
      int bh, qb;
      if (pairs) {
        const int half = p.nqb >> 1, lh = pos / half, pp = pos - lh * half;
        bh = x + 8 * lh;
        qb = ((r & 1) != light_first) ? pp : p.nqb - 1 - pp;
      } else {
        item_of(pos, bh, qb);
      }
#ifdef FA_STAMPS
      const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
      const unsigned long long c_start = __builtin_amdgcn_s_memtime();
#endif
      run_tile_loop<WAVES, BN, CAUSAL, false, SCHED, BF16, HDIM>(p, bh, qb, 0, smem);
#ifdef FA_STAMPS
      const int rec = bh * p.nqb + qb;
      if (threadIdx.x == 0 && rec < FA_MAX_TIMELINE) {
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        g_fa_timeline[rec][0] = t_start;
        g_fa_timeline[rec][1] = __builtin_amdgcn_s_memrealtime();
        g_fa_timeline[rec][3] = __builtin_amdgcn_s_memtime() - c_start;
        g_fa_timeline[rec][2] =
            (unsigned long long)hw | ((unsigned long long)xcc << 32) | ((unsigned long long)(qb & 0xFFFF) << 40) |
        ((unsigned long long)(bh & 0xFF) << 56);
      }
#endif
    }
    __syncthreads();  // LDS images are reused by the next item
  }
  if constexpr (kTailSplit) {
    if (split_tail && lcu < 2 * tail) {
      using Pol = M16<BN, typename std::conditional<BF16, __bf16, f16>::type, HDIM>;
      int bh, qb;
      item_of(full * C + (lcu >> 1), bh, qb);
      attention_kvpair<Pol, CAUSAL>(p, bh, 2 * qb + (lcu & 1), smem);  // 128-row half
    }
  }
}

}  // namespace fa

// one wave per SIMD, 64 query rows per wave, asm-owned register file
#include "fa_w4_kernel.hpp"
// one wave per SIMD, 16 rows of each of two query blocks per wave (short sequences)
#include "fa_w4p_kernel.hpp"

namespace fa {

// KV-pair (short sequences): 128 query rows per workgroup, the two waves of a
// SIMD split the key range (attention_kvpair); one workgroup per item, items
// ordered as map_block.
// SUB = 2: KV-quad (64 query rows, four-way key split).
template <int BN, bool CAUSAL, bool BF16 = false, int HDIM = 128, int SUB = 1>
__global__ __launch_bounds__(512, 2) void fa_fwd_f16_kvpair_kernel(FwdParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  using Pol = M16<BN, typename std::conditional<BF16, __bf16, f16>::type, HDIM>;
#ifdef FA_STAMPS
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  const unsigned long long c_start = __builtin_amdgcn_s_memtime();
#endif
  int qb, bh;
  map_block(blockIdx.x, gridDim.x, p.nqb, p.bh, p.band, CAUSAL, qb, bh);
  attention_kvpair<Pol, CAUSAL, SUB>(p, bh, qb, smem);
#ifdef FA_STAMPS
  if (threadIdx.x == 0 && blockIdx.x < FA_MAX_TIMELINE) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    g_fa_timeline[blockIdx.x][0] = t_start;
    g_fa_timeline[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
    g_fa_timeline[blockIdx.x][3] = __builtin_amdgcn_s_memtime() - c_start;
    g_fa_timeline[blockIdx.x][2] =
        (unsigned long long)hw | ((unsigned long long)xcc << 32) | ((unsigned long long)(qb & 0xFFFF) << 40) |
        ((unsigned long long)(bh & 0xFF) << 56);
  }
#endif
}

// Split-KV: workgroup id -> (split, item); items ordered as map_block.
template <int WAVES, int BN, bool CAUSAL, int SCHED>
__global__ __launch_bounds__(WAVES * 64, 2) void fa_fwd_f16_splitkv_kernel(FwdParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int split = blockIdx.x % p.num_splits;
  const int item = blockIdx.x / p.num_splits;
  int qb, bh;
  map_block(item, gridDim.x / p.num_splits, p.nqb, p.bh, 0, CAUSAL, qb, bh);
  run_tile_loop<WAVES, BN, CAUSAL, true, SCHED>(p, bh, qb, split, smem);
}

// Log-sum-exp merge of split partials (ref flash_attention_splitk_merge,
// :559-598): one wave per query row, 2 head-dim columns per lane.
//   M = max_s m_s ; L = sum_s l_s e^(m_s-M) ; O = sum_s O_s e^(m_s-M) / L
__global__ __launch_bounds__(256) void fa_splitkv_merge_kernel(const float* __restrict__ part_o,
                                                               const float* __restrict__ part_ml,
                                                               f16* __restrict__ o, int rows,
                                                               int num_splits) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  float M = -__builtin_inff();
  for (int s = 0; s < num_splits; ++s) M = fmaxf(M, part_ml[((size_t)s * rows + row) * 2]);
  float L = 0.f, o0 = 0.f, o1 = 0.f;
  for (int s = 0; s < num_splits; ++s) {
    const float2 ml = *reinterpret_cast<const float2*>(part_ml + ((size_t)s * rows + row) * 2);
    if (ml.y > 0.f) {
      const float w = __builtin_amdgcn_exp2f((ml.x - M) * 1.4426950408889634f);
      const float2 po =
          *reinterpret_cast<const float2*>(part_o + ((size_t)s * rows + row) * HD + 2 * lane);
      L += ml.y * w;
      o0 += po.x * w;
      o1 += po.y * w;
    }
  }
  const float inv = L > 0.f ? 1.0f / L : 0.f;
  typedef f16 f16x2 __attribute__((ext_vector_type(2)));
  f16x2 out = {(f16)(o0 * inv), (f16)(o1 * inv)};
  *reinterpret_cast<f16x2*>(o + (size_t)row * HD + 2 * lane) = out;
}

// ---------------------------------------------------------------------------
// config table
// ---------------------------------------------------------------------------
typedef void (*kernel_fn)(FwdParams);

struct Config {
  fa_config_info_t info;
  int sched;  // 0 = one barrier per tile, 1 = 8-wave ping-pong, 3 = ping-pong + LDS-DMA tiles
  int kind;   // 0 = one workgroup per item, 1 = split-KV, 2 = persistent, 3 = KV-pair,
              // 4 = KV-quad, 5 = persistent, one wave per SIMD (W4, asm item program),
              // 6 = paired 64-row query blocks, one wave per SIMD (W4P, asm item program),
              // 7 = two pairs per workgroup (the same program), 8 = one 64-row
              // block per workgroup (the same program), 9 = causal singles
              // and pairs mixed to fill the CUs (the same program), 10 =
              // causal groups of one to four blocks planned on the host
              // (w4p_plan: the two- or the four-block program per group)
  kernel_fn fn;
};

template <int W, int BN_, int C, int KIND, int SCHED, int DT, int HDIM>
constexpr kernel_fn pick_kernel() {
  if constexpr (KIND == 5)
    return fa_fwd_f16_w4_kernel<(C != 0), DT == 1, HDIM>;
  else if constexpr (KIND == 6)
    return fa_fwd_w4p_kernel<(C != 0), DT == 1, 1, HDIM>;
  else if constexpr (KIND == 7)
    return fa_fwd_w4p_kernel<(C != 0), DT == 1, 2, HDIM>;
  else if constexpr (KIND == 8)
    return fa_fwd_w4p_kernel<(C != 0), DT == 1, 0, HDIM>;
  else if constexpr (KIND == 9)
    return fa_fwd_w4p_kernel<(C != 0), DT == 1, 3, HDIM>;
  else if constexpr (KIND == 10)
    return fa_fwd_w4p_kernel<(C != 0), DT == 1, 4, HDIM>;

  else if constexpr (KIND == 3)
    return fa_fwd_f16_kvpair_kernel<BN_, (C != 0), DT == 1, HDIM>;
  else if constexpr (KIND == 4)
    return fa_fwd_f16_kvpair_kernel<BN_, (C != 0), DT == 1, HDIM, 2>;
  else if constexpr (KIND == 1)
    return fa_fwd_f16_splitkv_kernel<W, BN_, (C != 0), SCHED>;
  else if constexpr (KIND == 2)
    return fa_fwd_f16_persistent_kernel<W, BN_, (C != 0), SCHED, DT == 1, HDIM>;
  else
    return fa_fwd_f16_kernel<W, BN_, (C != 0), SCHED, DT == 1, HDIM>;
}

// KIND: 0 = one workgroup per (head, query block), 1 = split-KV, 2 = persistent
// DT: 0 = fp16, 1 = bf16 (FA_DTYPE_*)
// LDS images keep 256-B row slots at head_dim 64 too (fa_fwd_kernel.hpp M16)
#define FA_CFG_TD(ID, W, BN_, C, KIND, SCHED, DT, HDIM, NAME)                              \
  {{ID, 32 * (W), BN_, W, C, (KIND) == 1,                                                    \
    ((SCHED) == 3 ? 6 * (BN_) * ROW_BYTES                                                   \
     : ((KIND) == 2 && !(C)) ? std::max(4 * (BN_) * ROW_BYTES, kKvpairLdsBytes) /* tail */ \
                   : 4 * (BN_) * ROW_BYTES),                                                \
    NAME, DT, HDIM}, SCHED,                                                                 \
   KIND, pick_kernel<W, BN_, C, KIND, SCHED, DT, HDIM>()}
#define FA_CFG_T(ID, W, BN_, C, KIND, SCHED, DT, NAME) \
  FA_CFG_TD(ID, W, BN_, C, KIND, SCHED, DT, 128, NAME)
#define FA_CFG(ID, W, BN_, C, KIND, SCHED, NAME) FA_CFG_T(ID, W, BN_, C, KIND, SCHED, 0, NAME)
// KV-pair: 8 waves on 128 query rows (two waves per row block, key range split)
#define FA_CFG_KVPAIR(ID, C, DT, HDIM, NAME)                                           \
  {{ID, 128, 64, 8, C, 0, kKvpairLdsBytes, NAME, DT, HDIM}, 1, 3,                       \
   pick_kernel<8, 64, C, 3, 1, DT, HDIM>()}
// KV-quad: 8 waves on 64 query rows (four waves per row block, key range split four ways)
#define FA_CFG_KVQUAD(ID, C, DT, HDIM, NAME)                                           \
  {{ID, 64, 64, 8, C, 0, kKvquadLdsBytes, NAME, DT, HDIM}, 1, 4,                        \
   pick_kernel<8, 64, C, 4, 1, DT, HDIM>()}

// W4: 4 waves x 64 query rows (one wave per SIMD), K/V double-buffered (64 KB)
#define FA_CFG_W4D(ID, C, DT, HDIM, NAME)                                              \
  {{ID, 256, 64, 4, C, 0, w4_lds_bytes<HDIM>(), NAME, DT, HDIM}, 0, 5,                   \
   pick_kernel<4, 64, C, 5, 0, DT, HDIM>()}
#define FA_CFG_W4(ID, C, DT, NAME) FA_CFG_W4D(ID, C, DT, 128, NAME)
// W4P: 4 waves x 16 query rows of each of two (G = 1) or four (G = 2) 64-row
// blocks, K/V double-buffered (64 KB)
#define FA_CFG_W4PD(ID, G, C, DT, HDIM, NAME)                                          \
  {{ID, 128 * (G), 64, 4, C, 0, w4p_lds_bytes<G, HDIM>(), NAME, DT, HDIM}, 0, 5 + (G),    \
   pick_kernel<4, 64, C, 5 + (G), 0, DT, HDIM>()}
#define FA_CFG_W4P(ID, G, C, DT, NAME) FA_CFG_W4PD(ID, G, C, DT, 128, NAME)
// W4P singles: 4 waves x 16 query rows of one 64-row block (KIND 8), or of
// one or two (KIND 9: the heaviest blocks alone, the rest paired)
#define FA_CFG_W4PS(ID, C, DT, HDIM, NAME, KIND)                                       \
  {{ID, 64, 64, 4, C, 0, w4p_lds_bytes<(KIND) == 10 ? 4 : (KIND) == 9 ? 3 : 0, HDIM>(), NAME, DT, \
    HDIM}, 0, KIND, pick_kernel<4, 64, C, KIND, 0, DT, HDIM>()}

// Only tiers the dispatcher picks, explicit entry points (split-KV) and the
// baselines a test compares against (the per-item ping-pong 2/3: the
// persistent kernel must reproduce it bit for bit; LDS-DMA 20/21) ship.
static const Config kConfigs[] = {
    FA_CFG(0, 4, 64, 0, 0, 0, "bm128_bn64_w4_m16_noncausal"),
    FA_CFG(1, 4, 64, 1, 0, 0, "bm128_bn64_w4_m16_causal"),
    FA_CFG(2, 8, 64, 0, 0, 1, "bm256_bn64_w8_m16_pingpong_noncausal"),
    FA_CFG(3, 8, 64, 1, 0, 1, "bm256_bn64_w8_m16_pingpong_causal"),
    FA_CFG(4, 4, 64, 0, 1, 0, "bm128_bn64_w4_m16_noncausal_splitkv"),
    FA_CFG(5, 4, 64, 1, 1, 0, "bm128_bn64_w4_m16_causal_splitkv"),
    FA_CFG(6, 8, 64, 0, 2, 1, "bm256_bn64_w8_m16_pingpong_persistent_noncausal"),
    FA_CFG(7, 8, 64, 1, 2, 1, "bm256_bn64_w8_m16_pingpong_persistent_causal"),
    // bf16 twins of the dispatched fp16 tiers
    FA_CFG_T(8, 4, 64, 0, 0, 0, 1, "bf16_bm128_bn64_w4_m16_noncausal"),
    FA_CFG_T(9, 4, 64, 1, 0, 0, 1, "bf16_bm128_bn64_w4_m16_causal"),
    FA_CFG_T(10, 8, 64, 0, 2, 1, 1, "bf16_bm256_bn64_w8_m16_pingpong_persistent_noncausal"),
    FA_CFG_T(11, 8, 64, 1, 2, 1, 1, "bf16_bm256_bn64_w8_m16_pingpong_persistent_causal"),
    // head_dim 64 twins (fp16, bf16)
    FA_CFG_TD(12, 4, 64, 0, 0, 0, 0, 64, "d64_bm128_bn64_w4_m16_noncausal"),
    FA_CFG_TD(13, 4, 64, 1, 0, 0, 0, 64, "d64_bm128_bn64_w4_m16_causal"),
    FA_CFG_TD(14, 8, 64, 0, 2, 1, 0, 64, "d64_bm256_bn64_w8_m16_pingpong_persistent_noncausal"),
    FA_CFG_TD(15, 8, 64, 1, 2, 1, 0, 64, "d64_bm256_bn64_w8_m16_pingpong_persistent_causal"),
    FA_CFG_TD(16, 4, 64, 0, 0, 0, 1, 64, "bf16_d64_bm128_bn64_w4_m16_noncausal"),
    FA_CFG_TD(17, 4, 64, 1, 0, 0, 1, 64, "bf16_d64_bm128_bn64_w4_m16_causal"),
    FA_CFG_TD(18, 8, 64, 0, 2, 1, 1, 64, "bf16_d64_bm256_bn64_w8_m16_pingpong_persistent_noncausal"),
    FA_CFG_TD(19, 8, 64, 1, 2, 1, 1, 64, "bf16_d64_bm256_bn64_w8_m16_pingpong_persistent_causal"),
    // K/V by LDS-DMA into three rotating LDS buffers
    FA_CFG(20, 8, 64, 0, 2, 3, "bm256_bn64_w8_m16_pingpong_persistent_dma_noncausal"),
    FA_CFG(21, 8, 64, 1, 2, 3, "bm256_bn64_w8_m16_pingpong_persistent_dma_causal"),
    // KV-pair (short sequences): the two waves of a SIMD split the keys of 32 query rows
    FA_CFG_KVPAIR(22, 0, 0, 128, "bm128_bn64_w8_m16_kvpair_noncausal"),
    FA_CFG_KVPAIR(23, 1, 0, 128, "bm128_bn64_w8_m16_kvpair_causal"),
    FA_CFG_KVPAIR(24, 0, 1, 128, "bf16_bm128_bn64_w8_m16_kvpair_noncausal"),
    FA_CFG_KVPAIR(25, 1, 1, 128, "bf16_bm128_bn64_w8_m16_kvpair_causal"),
    FA_CFG_KVPAIR(26, 0, 0, 64, "d64_bm128_bn64_w8_m16_kvpair_noncausal"),
    FA_CFG_KVPAIR(27, 1, 0, 64, "d64_bm128_bn64_w8_m16_kvpair_causal"),
    FA_CFG_KVPAIR(28, 0, 1, 64, "bf16_d64_bm128_bn64_w8_m16_kvpair_noncausal"),
    FA_CFG_KVPAIR(29, 1, 1, 64, "bf16_d64_bm128_bn64_w8_m16_kvpair_causal"),
    // KV-quad (shortest sequences): four waves split the keys of 32 query rows
    FA_CFG_KVQUAD(30, 0, 0, 128, "bm64_bn64_w8_m16_kvquad_noncausal"),
    FA_CFG_KVQUAD(31, 1, 0, 128, "bm64_bn64_w8_m16_kvquad_causal"),
    FA_CFG_KVQUAD(32, 0, 1, 128, "bf16_bm64_bn64_w8_m16_kvquad_noncausal"),
    FA_CFG_KVQUAD(33, 1, 1, 128, "bf16_bm64_bn64_w8_m16_kvquad_causal"),
    FA_CFG_KVQUAD(34, 0, 0, 64, "d64_bm64_bn64_w8_m16_kvquad_noncausal"),
    FA_CFG_KVQUAD(35, 1, 0, 64, "d64_bm64_bn64_w8_m16_kvquad_causal"),
    FA_CFG_KVQUAD(36, 0, 1, 64, "bf16_d64_bm64_bn64_w8_m16_kvquad_noncausal"),
    FA_CFG_KVQUAD(37, 1, 1, 64, "bf16_d64_bm64_bn64_w8_m16_kvquad_causal"),
    // 4 waves x 64 query rows, persistent, asm item program (fa_w4_kernel.hpp)
    FA_CFG_W4(38, 0, 0, "bm256_bn64_w4x64_m16_asm_persistent_noncausal"),
    FA_CFG_W4(39, 1, 0, "bm256_bn64_w4x64_m16_asm_persistent_causal"),
    FA_CFG_W4(40, 0, 1, "bf16_bm256_bn64_w4x64_m16_asm_persistent_noncausal"),
    FA_CFG_W4(41, 1, 1, "bf16_bm256_bn64_w4x64_m16_asm_persistent_causal"),
    FA_CFG(42, 4, 128, 0, 0, 0, "bm128_bn128_w4_m16_noncausal"),
    FA_CFG(43, 4, 128, 1, 0, 0, "bm128_bn128_w4_m16_causal"),
    // head_dim 64 twins of the W4 tier (register-staged K/V)
    FA_CFG_W4D(44, 0, 0, 64, "d64_bm256_bn64_w4x64_m16_asm_persistent_noncausal"),
    FA_CFG_W4D(45, 1, 0, 64, "d64_bm256_bn64_w4x64_m16_asm_persistent_causal"),
    FA_CFG_W4D(46, 0, 1, 64, "bf16_d64_bm256_bn64_w4x64_m16_asm_persistent_noncausal"),
    FA_CFG_W4D(47, 1, 1, 64, "bf16_d64_bm256_bn64_w4x64_m16_asm_persistent_causal"),
    // paired 64-row query blocks, one wave per SIMD, asm item program (fa_w4p_kernel.hpp)
    FA_CFG_W4P(48, 1, 0, 0, "bm128_bn64_w4x32_m16_asm_pair_noncausal"),
    FA_CFG_W4P(49, 1, 1, 0, "bm128_bn64_w4x32_m16_asm_pair_causal"),
    FA_CFG_W4P(50, 1, 0, 1, "bf16_bm128_bn64_w4x32_m16_asm_pair_noncausal"),
    FA_CFG_W4P(51, 1, 1, 1, "bf16_bm128_bn64_w4x32_m16_asm_pair_causal"),
    // two pairs per workgroup: four 64-row blocks, 16 rows of each per wave
    FA_CFG_W4P(52, 2, 0, 0, "bm256_bn64_w4x64_m16_asm_quad_noncausal"),
    FA_CFG_W4P(53, 2, 1, 0, "bm256_bn64_w4x64_m16_asm_quad_causal"),
    FA_CFG_W4P(54, 2, 0, 1, "bf16_bm256_bn64_w4x64_m16_asm_quad_noncausal"),
    FA_CFG_W4P(55, 2, 1, 1, "bf16_bm256_bn64_w4x64_m16_asm_quad_causal"),
    // their head_dim-64 twins (round 5: the generator's set_hd, W4's packed
    // 128-B-row images)
    FA_CFG_W4PD(56, 1, 0, 0, 64, "d64_bm128_bn64_w4x32_m16_asm_pair_noncausal"),
    FA_CFG_W4PD(57, 1, 1, 0, 64, "d64_bm128_bn64_w4x32_m16_asm_pair_causal"),
    FA_CFG_W4PD(58, 1, 0, 1, 64, "bf16_d64_bm128_bn64_w4x32_m16_asm_pair_noncausal"),
    FA_CFG_W4PD(59, 1, 1, 1, 64, "bf16_d64_bm128_bn64_w4x32_m16_asm_pair_causal"),
    FA_CFG_W4PD(60, 2, 0, 0, 64, "d64_bm256_bn64_w4x64_m16_asm_quad_noncausal"),
    FA_CFG_W4PD(61, 2, 1, 0, 64, "d64_bm256_bn64_w4x64_m16_asm_quad_causal"),
    FA_CFG_W4PD(62, 2, 0, 1, 64, "bf16_d64_bm256_bn64_w4x64_m16_asm_quad_noncausal"),
    FA_CFG_W4PD(63, 2, 1, 1, 64, "bf16_d64_bm256_bn64_w4x64_m16_asm_quad_causal"),
    // one 64-row block per workgroup on the pair program (launches of at most
    // one block per CU)
    FA_CFG_W4PS(64, 0, 0, 128, "bm64_bn64_w4x16_m16_asm_single_noncausal", 8),
    FA_CFG_W4PS(65, 1, 0, 128, "bm64_bn64_w4x16_m16_asm_single_causal", 8),
    FA_CFG_W4PS(66, 0, 1, 128, "bf16_bm64_bn64_w4x16_m16_asm_single_noncausal", 8),
    FA_CFG_W4PS(67, 1, 1, 128, "bf16_bm64_bn64_w4x16_m16_asm_single_causal", 8),
    FA_CFG_W4PS(68, 0, 0, 64, "d64_bm64_bn64_w4x16_m16_asm_single_noncausal", 8),
    FA_CFG_W4PS(69, 1, 0, 64, "d64_bm64_bn64_w4x16_m16_asm_single_causal", 8),
    FA_CFG_W4PS(70, 0, 1, 64, "bf16_d64_bm64_bn64_w4x16_m16_asm_single_noncausal", 8),
    FA_CFG_W4PS(71, 1, 1, 64, "bf16_d64_bm64_bn64_w4x16_m16_asm_single_causal", 8),
    // causal launches between one and two 64-row blocks per CU: the heaviest
    // blocks alone, the rest in pairs, one workgroup per CU
    FA_CFG_W4PS(72, 1, 0, 128, "bm64_bn64_w4x16_m16_asm_mixed_causal", 9),
    FA_CFG_W4PS(73, 1, 1, 128, "bf16_bm64_bn64_w4x16_m16_asm_mixed_causal", 9),
    FA_CFG_W4PS(74, 1, 0, 64, "d64_bm64_bn64_w4x16_m16_asm_mixed_causal", 9),
    FA_CFG_W4PS(75, 1, 1, 64, "bf16_d64_bm64_bn64_w4x16_m16_asm_mixed_causal", 9),
    // causal launches of two to four blocks per CU short of whole quads:
    // groups of one to four blocks planned on the host, one workgroup per CU
    FA_CFG_W4PS(76, 1, 0, 128, "bm64_bn64_w4x16_m16_asm_planned_causal", 10),
    FA_CFG_W4PS(77, 1, 1, 128, "bf16_bm64_bn64_w4x16_m16_asm_planned_causal", 10),
    FA_CFG_W4PS(78, 1, 0, 64, "d64_bm64_bn64_w4x16_m16_asm_planned_causal", 10),
    FA_CFG_W4PS(79, 1, 1, 64, "bf16_d64_bm64_bn64_w4x16_m16_asm_planned_causal", 10),
};
static constexpr int kNumConfigs = sizeof(kConfigs) / sizeof(kConfigs[0]);

static int prepare(int id) {
  // raise the dynamic-LDS limit once per (device, config) -- the reference
  // re-does this inside every dispatch (:633/641/650/659).  Per device, so a
  // process driving several GPUs (one host thread each) sets it on every one.
  constexpr int kMaxDev = 64;
  static std::once_flag flags[kMaxDev][kNumConfigs];
  static hipError_t errs[kMaxDev][kNumConfigs];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return FA_ERR_HIP;
  std::call_once(flags[dev][id], [dev, id] {
    errs[dev][id] = hipFuncSetAttribute((const void*)kConfigs[id].fn,
                                        hipFuncAttributeMaxDynamicSharedMemorySize,
                                        kConfigs[id].info.lds_bytes);
  });
  return errs[dev][id] == hipSuccess ? FA_OK : FA_ERR_HIP;
}


// CUs of the current device (cached per device id)
static int num_cus() {
  static int cache[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cache[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}

// ---------------------------------------------------------------------------
// W4P planned groups (kind 10): a head's nq causal 64-row blocks (block b has
// b + 1 key tiles) in W workgroups of one to four blocks, minimising the
// heaviest workgroup under a cycle model from the stamps
// (profiles/r06_final_w4p_stamps.jsonl, r05_w4q2_stamps.jsonl): an
// iteration with L live blocks costs 1092 / 1617 cycles in the two-block
// program and 1550 / 1620 / 2875 / 2789 in the four-block one, plus a
// per-group prologue + epilogue of 7.0k / 8.8k / 13.5k / 16.0k cycles.
// Greedy placement (the W heaviest blocks one per group, the rest each to
// the group it costs least), then a deterministic local search of moves and
// swaps that never raise the pair of groups' larger cost.  Cached per
// (nq, W); the quads' cost under the same model decides whether to use it.
// ---------------------------------------------------------------------------
struct W4PPlan {
  long long cost = 0, quads_cost = 0;
  unsigned char g[256];
};

static long long w4p_group_cost(const int* blocks, int n) {
  static const int c2[3] = {0, 1092, 1617}, c4[5] = {0, 1550, 1620, 2875, 2789};
  static const int fix[5] = {0, 7000, 8800, 13500, 16000};
  if (n == 0) return 0;
  int t[4];
  for (int i = 0; i < n; ++i) t[i] = blocks[i] + 1;
  std::sort(t, t + n, [](int a, int b) { return a > b; });
  long long tot = fix[n];
  for (int i = 0; i < n; ++i) {
    const int next = i + 1 < n ? t[i + 1] : 0;
    tot += (long long)(t[i] - next) * (n <= 2 ? c2[i + 1] : c4[i + 1]);
  }
  return tot;
}

static W4PPlan w4p_plan(int nq, int W) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, W4PPlan> cache;
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find({nq, W});
  if (it != cache.end()) return it->second;
  W4PPlan pl;
  std::fill(pl.g, pl.g + 256, (unsigned char)0xff);
  if (nq < 1 || nq > 64 || W < (nq + 3) / 4 || W > nq || W > 64) {
    pl.cost = pl.quads_cost = 0;
    return cache[{nq, W}] = pl;
  }
  int grp[64][4], cnt[64] = {};
  long long cost[64] = {};
  for (int i = 0; i < W; ++i) {
    grp[i][0] = nq - 1 - i;
    cnt[i] = 1;
    cost[i] = w4p_group_cost(grp[i], 1);
  }
  for (int b = nq - 1 - W; b >= 0; --b) {
    int best = -1;
    long long bc = 0;
    for (int i = 0; i < W; ++i) {
      if (cnt[i] == 4) continue;
      grp[i][cnt[i]] = b;
      const long long c = w4p_group_cost(grp[i], cnt[i] + 1);
      if (best < 0 || c < bc) best = i, bc = c;
    }
    grp[best][cnt[best]++] = b;
    cost[best] = bc;
  }
  unsigned seed = 12345;
  auto rnd = [&seed](int n) {
    seed = seed * 1103515245u + 12345u;
    return (int)(((seed & 0x7fffffffu) >> 8) % (unsigned)n);
  };
  for (int it2 = 0; it2 < 20000; ++it2) {
    const int a = rnd(W), b = rnd(W);
    if (a == b) continue;
    int na[4], nb[4], ca = cnt[a], cbn = cnt[b];
    std::copy(grp[a], grp[a] + 4, na);
    std::copy(grp[b], grp[b] + 4, nb);
    if (rnd(2) == 0 && cnt[b] < 4 && cnt[a] > 1) {  // move one block a -> b
      const int x = rnd(cnt[a]);
      nb[cbn++] = na[x];
      na[x] = na[--ca];
    } else {  // swap one block of a with one of b
      const int x = rnd(cnt[a]), y = rnd(cnt[b]);
      std::swap(na[x], nb[y]);
    }
    const long long xa = w4p_group_cost(na, ca), xb = w4p_group_cost(nb, cbn);
    if (std::max(xa, xb) <= std::max(cost[a], cost[b])) {
      std::copy(na, na + 4, grp[a]);
      std::copy(nb, nb + 4, grp[b]);
      cnt[a] = ca, cnt[b] = cbn, cost[a] = xa, cost[b] = xb;
    }
  }
  // ranks heaviest first (the first-dispatched workgroups)
  int order[64];
  for (int i = 0; i < W; ++i) order[i] = i;
  std::sort(order, order + W, [&](int x, int y) { return cost[x] > cost[y] || (cost[x] == cost[y] && x < y); });
  for (int r = 0; r < W; ++r) {
    const int i = order[r];
    for (int k = 0; k < cnt[i]; ++k) pl.g[4 * r + k] = (unsigned char)grp[i][k];
    pl.cost = std::max(pl.cost, cost[i]);
  }
  // the quads (G = 2): item i = pairs 2i, 2i+1, pair r = (nq-1-r, r)
  const int np = (nq + 1) / 2;
  for (int i = 0; 2 * i < np; ++i) {
    int q[4], n = 0;
    for (int r = 2 * i; r < 2 * i + 2 && r < np; ++r) {
      q[n++] = nq - 1 - r;
      if (r < nq - 1 - r) q[n++] = r;
    }
    pl.quads_cost = std::max(pl.quads_cost, w4p_group_cost(q, n));
  }
  return cache[{nq, W}] = pl;
}

static int check_args(const void* q, const void* k, const void* v, const void* o, int batch,
                      int heads, int seq_len, int head_dim) {
  if (batch < 0 || heads < 0 || seq_len < 0 || head_dim < 0) return FA_ERR_BAD_SHAPE;
  if (head_dim != 128 && head_dim != 64) return FA_ERR_UNSUPPORTED_HEAD_DIM;
  if ((long long)batch * heads > 0x7fffffffLL) return FA_ERR_BAD_SHAPE;
  // a head's rows are addressed through one buffer resource whose byte range
  // (S * 2 * head_dim) is a 32-bit int: S <= 8388607 at head_dim 128
  if ((long long)seq_len * 2 * head_dim > 0x7fffffffLL) return FA_ERR_BAD_SHAPE;
  if (batch == 0 || heads == 0 || seq_len == 0) return FA_OK;
  if (!q || !k || !v || !o) return FA_ERR_NULL_POINTER;
  return FA_OK;
}

// W4 launches with a cross-XCD tail pool (fa_w4_kernel.hpp): the snake order
// (not the causal pairs of <= 64 heads) with >= 64 rounds per XCD list
// (w4_pool_rounds)
static bool w4_pool_on(const Config& cfg, long long bh, int nqb, long long blocks) {
  if (cfg.kind != 5 || blocks < 8) return false;
  if (cfg.info.causal && bh <= 64 && bh % 8 == 0 && nqb % 2 == 0) return false;  // pairs
  const long long per_xcd = (bh * nqb + 7) / 8, c = blocks / 8;
  return w4_pool_rounds((int)std::min<long long>((per_xcd + c - 1) / c, 1 << 30)) > 0;
}

static long long persistent_blocks(const Config& cfg, long long bh, int nqb) {
  // one workgroup per CU, 8 per XCD group; never more than the items per XCD
  const long long per_xcd = (bh & 7) == 0 ? (bh / 8) * nqb : (bh * nqb + 7) / 8;
  const long long c = std::min<long long>(std::max(1, num_cus() / 8), per_xcd);
  return 8 * c;
}

// band of the causal item order at <= 64 heads: 1 = the causal pairs (A/B
// knob for traffic studies: -DFA_BAND_FEW_HEADS=16 runs the band snake)
#ifndef FA_BAND_FEW_HEADS
#define FA_BAND_FEW_HEADS 1
#endif

static int launch(int id, const void* q, const void* k, const void* v, void* o, int bh,
                  int seq_len, int num_splits, float* part_o, float* part_ml,
                  hipStream_t stream, unsigned* pool_ctr = nullptr) {
  const Config& cfg = kConfigs[id];
  int rc = prepare(id);
  if (rc != FA_OK) return rc;
  FwdParams p = {};
  p.q = static_cast<const f16*>(q);
  p.k = static_cast<const f16*>(k);
  p.v = static_cast<const f16*>(v);
  p.o = static_cast<f16*>(o);
  p.part_o = part_o;
  p.part_ml = part_ml;
  p.seq_len = seq_len;
  p.bh = bh;
  p.nqb = (seq_len + cfg.info.block_m - 1) / cfg.info.block_m;
  p.num_splits = num_splits;
  p.scale = 1.0f / sqrtf((float)cfg.info.head_dim);  // ref :612
  p.c = p.scale * 1.4426950408889634f;        // LOG2E, ref :239
  // few heads per XCD: plain heaviest-first balances better; many: keep the
  // query blocks of a head together for L2 reuse (profiles/r01_band_ab.txt)
  p.band = bh <= 64 ? FA_BAND_FEW_HEADS : 16;
  if (cfg.kind == 9) {
    // workgroups per head: the CUs' share, between ceil(nqb64 / 2) (pairs)
    // and nqb64 (singles)
    const int nq = (seq_len + 63) / 64;
    p.nqb = std::max((nq + 1) / 2, std::min(nq, num_cus() / std::max(bh, 1)));
  }
  if (cfg.kind == 10) {
    // workgroups per head: the CUs' share, between ceil(nqb64 / 4) and nqb64
    const int nq = (seq_len + 63) / 64;
    if (nq > 64) return FA_ERR_BAD_CONFIG;
    p.nqb = std::max((nq + 3) / 4, std::min(nq, num_cus() / std::max(bh, 1)));
    const W4PPlan pl = w4p_plan(nq, p.nqb);
    std::copy(pl.g, pl.g + 256, p.plan);
  }
  long long blocks = (long long)p.nqb * bh * num_splits;
  if (blocks > 0x7fffffffLL) return FA_ERR_BAD_SHAPE;
  if (cfg.kind == 2 || cfg.kind == 5) blocks = persistent_blocks(cfg, bh, p.nqb);
  if (pool_ctr && w4_pool_on(cfg, bh, p.nqb, blocks)) p.ws_ctr = pool_ctr;

  hipLaunchKernelGGL(cfg.fn, dim3((unsigned)blocks), dim3(cfg.info.waves * 64),
                     cfg.info.lds_bytes, stream, p);
  return hipGetLastError() == hipSuccess ? FA_OK : FA_ERR_LAUNCH;
}

// the fp16 head_dim-128 config of a tier: (block_m, waves, block_n, mask,
// schedule, kind) -- every field that tells two tiers apart
static int cfg_for(int block_m, int waves, int bn, int causal, int sched, int kind) {
  for (int i = 0; i < kNumConfigs; ++i) {
    const Config& c = kConfigs[i];
    if (c.info.block_m == block_m && c.info.waves == waves && c.info.block_n == bn &&
        c.info.causal == causal && c.kind == kind && c.sched == sched &&
        c.info.dtype == FA_DTYPE_F16 && c.info.head_dim == 128)
      return i;
  }
  return -1;
}

// the twin of a config for another element type / head_dim (same tile
// shape, schedule and kind), or -1
static int twin(int id, int dtype, int head_dim) {
  if (id < 0) return -1;
  const Config& c = kConfigs[id];
  for (int i = 0; i < kNumConfigs; ++i) {
    const Config& t = kConfigs[i];
    if (t.info.dtype == dtype && t.info.head_dim == head_dim && t.info.block_m == c.info.block_m &&
        t.info.waves == c.info.waves && t.info.block_n == c.info.block_n &&
        t.info.causal == c.info.causal && t.info.split_kv == c.info.split_kv &&
        t.sched == c.sched && t.kind == c.kind)
      return i;
  }
  return -1;
}

// one forced config: its mask, dtype and head_dim must match the call
static int launch_config(int config_id, int dtype, const void* q, const void* k, const void* v,
                         void* o, int batch, int heads, int seq_len, int head_dim, int causal,
                         void* hip_stream) {
  int rc = check_args(q, k, v, o, batch, heads, seq_len, head_dim);
  if (rc != FA_OK) return rc;
  if (config_id < 0 || config_id >= kNumConfigs) return FA_ERR_BAD_CONFIG;
  const Config& cfg = kConfigs[config_id];
  if (cfg.info.causal != (causal ? 1 : 0) || cfg.info.split_kv || cfg.info.dtype != dtype)
    return FA_ERR_BAD_CONFIG;
  if (cfg.info.head_dim != head_dim) return FA_ERR_UNSUPPORTED_HEAD_DIM;
  if (batch == 0 || heads == 0 || seq_len == 0) return FA_OK;
  return launch(config_id, q, k, v, o, batch * heads, seq_len, 1, nullptr, nullptr,
                (hipStream_t)hip_stream);
}

// dispatcher tier, as the twin for this dtype / head_dim
static int launch_auto(int dtype, const void* q, const void* k, const void* v, void* o,
                       int batch, int heads, int seq_len, int head_dim, int causal,
                       void* hip_stream, unsigned* pool_ctr = nullptr);

}  // namespace fa

using namespace fa;

// the tier table; pair = false skips the paired tier (it has no head_dim-64 twin)
static int select_tier(int batch, int heads, int seq_len, int causal, bool pair);

extern "C" int fa_select_config(int batch, int heads, int seq_len, int causal) {
  return select_tier(batch, heads, seq_len, causal, true);
}

static int select_tier(int batch, int heads, int seq_len, int causal, bool pair) {
  // Tier table re-derived for 256 CUs (ref :620-661 picks by seq >= 2048 on
  // 58 SMs), from tools/small_s.py and tools/sweep.py on the box:
  //  * 8-wave persistent ping-pong (256 rows / workgroup) once there are
  //    1.5 256-row items per CU, or 0.6 per CU without a mask (S=2048 B=1
  //    H=32 non-causal: 1015 vs 873 TFLOP/s), or one per CU of short items
  //    (profiles/r01_tier_study.jsonl, r01_tier_study_heads.jsonl);
  //  * S <= 128: the 4-wave 128-row loop (a 256-row item would be half
  //    padding: B=64 H=32 S=128 364 vs 229 TFLOP/s non-causal);
  //  * under-filled launches (<= 512 128-row blocks): the KV-pair kernel
  //    (128 rows per workgroup, the two waves of a SIMD splitting the keys):
  //    twice the workgroups of the 256-row tier and half the heaviest causal
  //    key loop; 1.0-1.2x the 4-wave loop at B=1 H=32, S=512-2048
  //    (profiles/r01_short_s_ab.jsonl);
  //  * launches of <= 256 64-row blocks (one workgroup per CU): the KV-quad
  //    (64 rows, four-way key split): B=1 H=8 S=2048 633 vs KV-pair 511,
  //    H=4 S=4096 causal 396 vs 285; at 512 blocks it loses (H=16 S=2048
  //    637 vs 907) (profiles/r01_kvquad_study.jsonl);
  //  * S <= 256 short of the persistent tier: the 4-wave loop (B=1 H=32
  //    S=256 109 vs KV-pair 100, B=4 387 vs 352, same study);
  //  * otherwise the 4-wave loop (with many blocks the KV-pair's doubled LDS
  //    traffic per FLOP costs more than its balance gains: B=16 S=512
  //    causal 4-wave 398 vs KV-pair 294, profiles/r01_tier_study.jsonl).
  const long long bh = (long long)batch * heads;
  const long long wg256 = bh * ((seq_len + 255) / 256);
  const long long wg128 = bh * ((seq_len + 127) / 128);
  const long long wg64 = bh * ((seq_len + 63) / 64);
  const long long nqb256 = (seq_len + 255) / 256;
  const int c = causal ? 1 : 0;
  // at most one 64-row query block per CU (heads of <= 64 blocks): one block
  // per workgroup on the W4P pair program (singles) -- a pair's second block
  // adds its prologue Q rows, its iterations and its epilogue to the
  // workgroup with CUs to spare.  Same process against the tier it replaced
  // (profiles/r06_ab_w4p_single.jsonl): B=1 H=32 S=512 causal 248 vs pairs
  // 219, non-causal 474 vs KV-quad 369; S=256 causal 83 vs the 4-wave loop 53,
  // non-causal 164 vs 114; S=128 22 vs 18 / 44 vs 39, B=4 87 vs 69 / 177 vs
  // 151; H=16 S=1024 causal 339 vs 312, non-causal 640 vs 535; H=8 S=2048 422
  // vs 401 / 770 vs 677; H=4 S=4096 487 vs 471 / 751 vs 748; past one block
  // per CU it loses (H=32 S=768 causal 361 vs 379).  Head_dim 64 non-causal
  // (pair = false) up to 16 blocks per head: S=512 308 vs KV-quad 276, H=16
  // S=1024 417 vs 406; H=8 S=2048 507 vs 525, H=4 S=4096 485 vs 607
  if (wg64 <= num_cus() && (seq_len + 63) / 64 <= (pair ? 64 : 16)) return cfg_for(64, 4, 64, c, 0, 8);
  // causal with about one 256-row item per CU: the snake cannot balance item
  // costs 1..nqb256, so the KV-pair's halved heaviest key loop wins from
  // nqb256 = 4 on (B=2 S=1024: 503 vs 461; B=4 S=512: 264 vs 364)
  // non-causal: from 160 items (B=1 H=24 S=2048: 829 vs KV-pair 668; H=6
  // S=8192: 1039 vs 854; at 128 items the KV-pair still wins, 732 vs 532)
  const bool persist =
      seq_len > 128 && (causal ? (wg256 >= 384 || (wg256 >= 256 && nqb256 <= 2)) : wg256 >= 160);
  if (persist) {
    // the one-wave-per-SIMD asm kernel (W4, same items and order), except a
    // non-causal launch whose last round is short: the ping-pong runs that
    // tail as KV-pair halves on twice the CUs, W4 has no tail split
    // (CUs per XCD as launch() sizes the persistent grid)
    const long long per_xcd = (wg256 + 7) / 8,
                    cus = std::min<long long>(std::max(1, num_cus() / 8), per_xcd);
    const long long tail = per_xcd % cus;
    if (!causal && tail > 0 && 2 * tail <= cus) return cfg_for(256, 8, 64, c, 1, 2);
    return cfg_for(256, 4, 64, c, 0, 5);
  }
  // paired 64-row query blocks (W4P, fa_w4p_kernel.hpp), same-process A/Bs
  // against the KV-pair / KV-quad / split tiers (profiles/r05_w4p_*ab*.jsonl):
  //  * causal, S <= 4096, one round of pairs on the CUs (every pair costs
  //    nqb64+1 key tiles): B=1 H=32 S=1024 530 vs 388, B=2 H=8 S=2048 673 vs
  //    507, H=24 S=1024 429 vs 315, H=8 S=4096 755 vs KV-quad 667 and split
  //    714; longer heads stay on the split tier / KV-quad (H=4 S=8192 742 vs
  //    884 / 785);
  //  * non-causal from 3/4 of a round of pairs (below, the KV-quad: H=16
  //    S=1024 470 vs 514) up to the persistent tier: H=4 S=8192 1182 vs 1090,
  //    H=16 S=2048 1004 vs 899, H=48 S=512 557 vs 468
  //  * causal launches of one to two rounds of pairs run them two per
  //    workgroup (quads: four blocks per wave while the light blocks last,
  //    two after): B=1 H=32 S=2048 816 vs pairs 663, B=2 H=32 S=1024 662 vs
  //    532, H=16 S=4096 942 vs KV-pair 862; past that the persistent tier
  //    (B=4 H=32 S=1024 802 vs 701)
  //  * S <= 256 (round 6): one round of pairs (or the mixed grouping) beats
  //    the 4-wave loop there too (H=96 S=256 causal 193 vs 147, H=65 S=256
  //    mixed 152 vs 105, B=2 H=64 S=256 257 vs 195, H=200 S=128 120 vs 105;
  //    non-causal H=96 S=256 357 vs 324, H=200 S=128 233 vs 228;
  //    profiles/r06_ab_w4p_short.jsonl); quads stay above S=256 (unmeasured
  //    below)
  if (pair) {
    const long long nq64 = (seq_len + 63) / 64, pairs = bh * ((nq64 + 1) / 2), cus = num_cus();
    // causal, between one and two blocks per CU: the heaviest blocks alone,
    // the rest paired, one workgroup per CU (a pair's two-block iterations
    // cost less than two singles', so the heaviest block sets the launch);
    // bit-identical to the pairs, same process (profiles/r06_ab_w4p_mixed.jsonl):
    // H=32 S=768 417 vs pairs 375, S=640 335 vs 303, S=896 506 vs 474, H=24
    // S=1024 483 vs 445, H=20 S=1024 415 vs 384, B=3 H=8 S=1024 486 vs 447,
    // H=10 S=2048 444 vs 432, H=12 S=2048 553 vs 556, H=6 S=4096 607 vs 599;
    // d64 S=768 287 vs 259.  Where no block can go alone (B=1 H=32 S=1024:
    // 8 CUs for 16 blocks per head) it is the pair grouping itself.
    if (causal && nq64 <= 64 && pairs <= cus) {
      const bool mixed = cus / bh > (nq64 + 1) / 2;
      return mixed ? cfg_for(64, 4, 64, c, 0, 9) : cfg_for(128, 4, 64, c, 0, 6);
    }
    if (causal && nq64 <= 64 && pairs <= 2 * cus && seq_len > 256) {
      // groups planned on the host where the quads leave CUs idle and the
      // plan's modelled heaviest workgroup is >= 5 % lighter than theirs;
      // bit-identical to the pairs, same process (profiles/r06_ab_w4p_planned.jsonl):
      // H=32 S=1280 655 vs quads 533, S=1536 701 vs 675, S=1792 802 vs 764,
      // H=25 S=2048 731 vs 704, H=16 S=2560 807 vs 641, S=3072 896 vs 792,
      // d64 S=1536 507 vs 462; where whole quads fill the CUs the model keeps
      // them (S=2048 862 vs planned 858, B=2 S=1024 684 vs 673)
      const int W = (int)std::min<long long>(nq64, cus / bh);
      const W4PPlan pl = w4p_plan((int)nq64, W);
      if (pl.cost > 0 && 100 * pl.cost <= 95 * pl.quads_cost) return cfg_for(64, 4, 64, c, 0, 10);
      return cfg_for(256, 4, 64, c, 0, 7);
    }
    // non-causal below 3/4 of a round too, past the singles (heads of <= 64
    // blocks; r06_ab_w4p_short.jsonl: H=20 S=1024 570 vs KV-pair 520, H=18
    // 520 vs 478, H=10 S=2048 704 vs 629)
    if (!causal && (4 * pairs >= 3 * cus ? (seq_len > 256 || pairs <= cus) : nq64 <= 64))
      return cfg_for(128, 4, 64, c, 0, 6);
  }
  if (seq_len <= 256) return cfg_for(128, 4, 64, c, 0, 0);
  // causal, two rounds of 64-row blocks over long heads (>= 32 blocks per
  // head): the KV-quad's four-way key split halves the heaviest block's key
  // loop against the KV-pair (B=1 H=4 S=8192 765 vs 599, H=2 S=16384 808 vs
  // 623, H=8 S=4096 694 vs 562, H=16 S=2048 544 vs 513; at S=1024 or past
  // 512 blocks the KV-pair still wins: profiles/r02_pair_vs_quad.jsonl)
  const long long nqb64 = (seq_len + 63) / 64;
  if (wg64 <= 256 || (causal && wg64 <= 512 && nqb64 >= 32))
    return cfg_for(64, 8, 64, c, 1, 4);
  if (wg128 <= 512) return cfg_for(128, 8, 64, c, 1, 3);
  return cfg_for(128, 4, 64, c, 0, 0);
}

namespace fa {
// the paired tier (W4P) at head_dim 64 only for causal launches: non-causal
// its d64 twin trails the KV-pair / W4 d64 (B=1 H=4 S=8192 851 vs 886, H=16
// S=2048 722 vs 744); causal it leads (H=32 S=1024 374 vs 301, S=2048 quad
// 653 vs 582, B=2 S=1024 502 vs 410; profiles/r05_ab_w4p_d64.jsonl).  One
// rule for the launch and for fa_fwd_ws_bytes / the pool decision.
static bool pair_tier_ok(int head_dim, int causal) { return head_dim == HD || causal; }

static int launch_auto(int dtype, const void* q, const void* k, const void* v, void* o,
                           int batch, int heads, int seq_len, int head_dim, int causal,
                           void* hip_stream, unsigned* pool_ctr) {
  int rc = check_args(q, k, v, o, batch, heads, seq_len, head_dim);
  if (rc != FA_OK) return rc;
  if (batch == 0 || heads == 0 || seq_len == 0) return FA_OK;
  const int sel = select_tier(batch, heads, seq_len, causal, pair_tier_ok(head_dim, causal));
  // (head_dim 64 of the W4 tier is the same item program with 2-step QK^T
  // chains and 8-KiB packed tiles: +4-9 % over the 8-wave ping-pong at
  // head_dim 64, profiles/r04_ab_w4_d64.jsonl, r05_ab_d64dma.jsonl)
  const int id = twin(sel, dtype, head_dim);
  if (id < 0) return FA_ERR_BAD_CONFIG;
  return launch(id, q, k, v, o, batch * heads, seq_len, 1, nullptr, nullptr,
                (hipStream_t)hip_stream, pool_ctr);
}

// the default dispatch of a workspace call runs the W4 tier with a cross-XCD
// tail pool (its counters live in the workspace's counter region)
static bool auto_pool(int batch, int heads, int seq_len, int head_dim, int causal) {
  if (batch <= 0 || heads <= 0 || seq_len <= 0 || (head_dim != HD && head_dim != 64)) return false;
  const int id = twin(select_tier(batch, heads, seq_len, causal, pair_tier_ok(head_dim, causal)),
                      FA_DTYPE_F16, head_dim);
  if (id < 0 || kConfigs[id].kind != 5) return false;
  const long long bh = (long long)batch * heads;
  const int nqb = (seq_len + kConfigs[id].info.block_m - 1) / kConfigs[id].info.block_m;
  return w4_pool_on(kConfigs[id], bh, nqb, persistent_blocks(kConfigs[id], bh, nqb));
}
}  // namespace fa

extern "C" int fa_fwd_f16_config(const void* q, const void* k, const void* v, void* o,
                                 int batch, int heads, int seq_len, int head_dim, int causal,
                                 int config_id, void* hip_stream) {
  return launch_config(config_id, FA_DTYPE_F16, q, k, v, o, batch, heads, seq_len, head_dim,
                       causal, hip_stream);
}

extern "C" int fa_fwd_bf16_config(const void* q, const void* k, const void* v, void* o,
                                  int batch, int heads, int seq_len, int head_dim, int causal,
                                  int config_id, void* hip_stream) {
  return launch_config(config_id, FA_DTYPE_BF16, q, k, v, o, batch, heads, seq_len, head_dim,
                       causal, hip_stream);
}

extern "C" int fa_fwd_bf16(const void* q, const void* k, const void* v, void* o, int batch,
                           int heads, int seq_len, int head_dim, int causal, void* hip_stream) {
  return launch_auto(FA_DTYPE_BF16, q, k, v, o, batch, heads, seq_len, head_dim, causal,
                     hip_stream);
}

extern "C" int fa_fwd_f16(const void* q, const void* k, const void* v, void* o, int batch,
                          int heads, int seq_len, int head_dim, int causal, void* hip_stream) {
  return launch_auto(FA_DTYPE_F16, q, k, v, o, batch, heads, seq_len, head_dim, causal,
                     hip_stream);
}

// ---- causal split tier (workspace entries) -----------------------------------
// Short causal launches (fewer 256-row items than the persistent tier needs):
// fa_fwd_f16_w4s_kernel cuts each query block's key range into pieces of T
// 64-key tiles, one workgroup each, merged in-launch through the workspace.
// T = the shortest piece (>= 4 tiles: the diagonal piece keeps every wave
// busy) whose pieces all fit one round on the device's CUs, at most 8 pieces
// per query block.
struct SplitPlan {
  int T = 0, pmax = 0, nqb = 0;
  long long items = 0;
  unsigned long long ctr_bytes = 0, lse_bytes = 0, o_bytes = 0;
  unsigned long long bytes() const { return ctr_bytes + lse_bytes + o_bytes; }
};

// Workspace layout: arrival counters in a FIXED first 64 KB (one per query
// block, at most 16384 blocks), then the per-row log2-sum-exp, then the
// partial O slabs.  The counter region never overlaps another shape's data
// regions, so one zero-filled buffer stays valid across shapes: every launch
// returns the counters it used to zero.
constexpr unsigned long long kSplitCtrBytes = 65536;

// the plan for piece length T (64-key tiles), or none if a query block would
// need more than 8 pieces (the merge's limit) or the launch has more query
// blocks than counters
static SplitPlan plan_for(long long bh, int seq_len, int T) {
  SplitPlan sp;
  const int nqb = (seq_len + 255) / 256;
  if (bh * nqb > (long long)(kSplitCtrBytes / 4)) return sp;
  long long items = 0;
  int pmax = 1;
  for (int qb = 0; qb < nqb; ++qb) {
    const int tiles = (std::min(256 * (qb + 1), seq_len) + 63) / 64;
    const int np = (tiles + T - 1) / T;
    items += bh * np;
    pmax = std::max(pmax, np);
  }
  if (pmax > 8) return sp;
  sp.T = T;
  sp.pmax = pmax;
  sp.nqb = nqb;
  sp.items = items;
  sp.ctr_bytes = kSplitCtrBytes;
  sp.lse_bytes = (unsigned long long)bh * nqb * pmax * 256 * 4;
  sp.o_bytes = (unsigned long long)bh * nqb * pmax * 256 * ROW_BYTES;
  return sp;
}

// piece_tiles > 0: that piece length (causal, head_dim 128; T = 0 if it
// needs more than 8 pieces); 0: the dispatcher's choice -- long causal
// launches short of the persistent tier (S >= 4096, fewer than 384 256-row
// items): the split beats the KV-quad tier there (B=1 H=8 S=4096 662 vs 612
// TFLOP/s, H=4 S=8192 801 vs 716, H=2 S=16384 923 vs 810, H=4 S=4096 481 vs
// 414) and loses below S=4096 (H=8 S=2048 303 vs 349, B=1 H=32 S=1024 335
// vs KV-pair 434: a W4 item's ~11k-cycle prologue and the merge outweigh
// the balance; profiles/r03_ab_split_tier*.jsonl)
static SplitPlan split_plan(int batch, int heads, int seq_len, int head_dim, int causal,
                            int piece_tiles = 0) {
  SplitPlan none;
  if (!causal || head_dim != HD || batch <= 0 || heads <= 0 || seq_len <= 0) return none;
  const long long bh = (long long)batch * heads;
  if (piece_tiles > 0) {
    SplitPlan sp = plan_for(bh, seq_len, piece_tiles);
    return sp.pmax > 1 ? sp : none;  // one piece per block: not a split
  }
  const int nqb = (seq_len + 255) / 256;
  const long long wg256 = bh * nqb;
  if (seq_len < 4096 || wg256 >= 384) return none;  // short, or the persistent tier's shapes
  // the paired tier's shapes (B=1 H=8 S=4096: 755 vs the split's 714)
  if (kConfigs[select_tier(batch, heads, seq_len, causal, true)].kind >= 6) return none;
  const long long cus = num_cus();
  // the shortest piece (>= 4 tiles: the diagonal piece keeps every wave
  // busy) whose pieces all fit one round on the device's CUs
  for (int T = 4; T <= 4 * nqb; ++T) {
    const SplitPlan sp = plan_for(bh, seq_len, T);
    if (sp.T && sp.items <= cus) return sp.pmax > 1 ? sp : none;
  }
  return none;
}

template <bool BF16>
static int launch_split(const SplitPlan& sp, const void* q, const void* k, const void* v, void* o,
                        int bh, int seq_len, void* ws, hipStream_t stream) {
  // K/V images + the item table, as the non-split program lays them out (a
  // one-piece query block runs it)
  constexpr int kLds = w4_lds_bytes<128>();
  static std::once_flag flags[64];
  static hipError_t errs[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return FA_ERR_HIP;
  std::call_once(flags[dev], [dev] {
    errs[dev] = hipFuncSetAttribute((const void*)fa_fwd_f16_w4s_kernel<BF16>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, kLds);
  });
  if (errs[dev] != hipSuccess) return FA_ERR_HIP;
  FwdParams p = {};
  p.q = static_cast<const f16*>(q);
  p.k = static_cast<const f16*>(k);
  p.v = static_cast<const f16*>(v);
  p.o = static_cast<f16*>(o);
  p.seq_len = seq_len;
  p.bh = bh;
  p.nqb = sp.nqb;
  p.num_splits = 1;
  p.scale = 1.0f / sqrtf((float)HD);
  p.c = p.scale * 1.4426950408889634f;
  p.band = 1;
  char* w = static_cast<char*>(ws);
  p.ws_ctr = reinterpret_cast<unsigned*>(w);
  p.ws_lse = reinterpret_cast<float*>(w + sp.ctr_bytes);
  p.ws_o = w + sp.ctr_bytes + sp.lse_bytes;
  p.piece_tiles = sp.T;
  p.pmax = sp.pmax;
  hipLaunchKernelGGL(fa_fwd_f16_w4s_kernel<BF16>, dim3((unsigned)sp.items), dim3(256), kLds,
                     stream, p);
  return hipGetLastError() == hipSuccess ? FA_OK : FA_ERR_LAUNCH;
}

static int launch_ws(int dtype, const void* q, const void* k, const void* v, void* o, int batch,
                     int heads, int seq_len, int head_dim, int causal, int piece_tiles, void* ws,
                     unsigned long long ws_bytes, void* hip_stream) {
  int rc = check_args(q, k, v, o, batch, heads, seq_len, head_dim);
  if (rc != FA_OK) return rc;
  if (batch == 0 || heads == 0 || seq_len == 0) return FA_OK;
  const SplitPlan sp = split_plan(batch, heads, seq_len, head_dim, causal, piece_tiles);
  if (piece_tiles > 0 && sp.T == 0) return FA_ERR_BAD_CONFIG;  // not a causal d128 split
  if (sp.T == 0) {
    // the W4 tier's tail pool when the workspace holds its counters (else
    // the static order: a workspace is optional there)
    // (its 64-bit claim counters need an 8-byte aligned workspace: a
    // misaligned one runs the static order, as no workspace does)
    const bool pool = ws && ws_bytes >= kSplitCtrBytes && (reinterpret_cast<uintptr_t>(ws) & 7) == 0 &&
                      auto_pool(batch, heads, seq_len, head_dim, causal);
    return launch_auto(dtype, q, k, v, o, batch, heads, seq_len, head_dim, causal, hip_stream,
                       pool ? static_cast<unsigned*>(ws) : nullptr);
  }
  // the slabs take 16-B sc1 stores / loads: a 16-byte aligned workspace
  if (!ws || ws_bytes < sp.bytes() || (reinterpret_cast<uintptr_t>(ws) & 15) != 0) return FA_ERR_WORKSPACE;
  const int bh = batch * heads;
  return dtype == FA_DTYPE_BF16
             ? launch_split<true>(sp, q, k, v, o, bh, seq_len, ws, (hipStream_t)hip_stream)
             : launch_split<false>(sp, q, k, v, o, bh, seq_len, ws, (hipStream_t)hip_stream);
}

extern "C" unsigned long long fa_fwd_ws_bytes(int batch, int heads, int seq_len, int head_dim,
                                              int causal, int piece_tiles) {
  const unsigned long long split = split_plan(batch, heads, seq_len, head_dim, causal, piece_tiles).bytes();
  if (split || piece_tiles > 0) return split;
  return auto_pool(batch, heads, seq_len, head_dim, causal) ? kSplitCtrBytes : 0;
}

extern "C" int fa_fwd_split_pieces(int batch, int heads, int seq_len, int head_dim, int causal) {
  return split_plan(batch, heads, seq_len, head_dim, causal).T;
}

extern "C" int fa_fwd_f16_ws(const void* q, const void* k, const void* v, void* o, int batch,
                             int heads, int seq_len, int head_dim, int causal, int piece_tiles,
                             void* workspace, unsigned long long ws_bytes, void* hip_stream) {
  return launch_ws(FA_DTYPE_F16, q, k, v, o, batch, heads, seq_len, head_dim, causal, piece_tiles,
                   workspace, ws_bytes, hip_stream);
}

extern "C" int fa_fwd_bf16_ws(const void* q, const void* k, const void* v, void* o, int batch,
                              int heads, int seq_len, int head_dim, int causal, int piece_tiles,
                              void* workspace, unsigned long long ws_bytes, void* hip_stream) {
  return launch_ws(FA_DTYPE_BF16, q, k, v, o, batch, heads, seq_len, head_dim, causal, piece_tiles,
                   workspace, ws_bytes, hip_stream);
}

// ---- split-KV ---------------------------------------------------------------
static int splitkv_cfg(int causal) { return cfg_for(128, 4, 64, causal ? 1 : 0, 0, 1); }

extern "C" int fa_splitkv_num_splits(int batch, int heads, int seq_len, int causal) {
  // enough workgroups to cover 256 CUs twice, at most one split per key tile
  if (batch <= 0 || heads <= 0 || seq_len <= 0) return 1;
  const int bm = kConfigs[splitkv_cfg(causal)].info.block_m;
  const int bn = kConfigs[splitkv_cfg(causal)].info.block_n;
  const long long items = (long long)batch * heads * ((seq_len + bm - 1) / bm);
  const int tiles = (seq_len + bn - 1) / bn;
  long long s = (512 + items - 1) / items;
  if (s > tiles) s = tiles;
  if (s > 16) s = 16;
  return s < 1 ? 1 : (int)s;
}

extern "C" unsigned long long fa_splitkv_o_bytes(int batch, int heads, int seq_len, int head_dim,
                                                 int num_splits) {
  if (batch <= 0 || heads <= 0 || seq_len <= 0 || head_dim <= 0 || num_splits <= 0) return 0;
  return (unsigned long long)num_splits * batch * heads * seq_len * head_dim * sizeof(float);
}

extern "C" unsigned long long fa_splitkv_ml_bytes(int batch, int heads, int seq_len, int head_dim,
                                                  int num_splits) {
  (void)head_dim;
  if (batch <= 0 || heads <= 0 || seq_len <= 0 || num_splits <= 0) return 0;
  return (unsigned long long)num_splits * batch * heads * seq_len * 2 * sizeof(float);
}

extern "C" int fa_fwd_f16_splitkv(const void* q, const void* k, const void* v, void* o,
                                  int batch, int heads, int seq_len, int head_dim, int causal,
                                  int num_splits, float* part_o, float* part_ml,
                                  void* hip_stream) {
  if (head_dim != HD) return FA_ERR_UNSUPPORTED_HEAD_DIM;  // split-KV: head_dim 128 only
  int rc = check_args(q, k, v, o, batch, heads, seq_len, head_dim);
  if (rc != FA_OK) return rc;
  // fp32 partial rows: the same 32-bit range at 4 bytes per element
  if ((long long)seq_len * 4 * head_dim > 0x7fffffffLL) return FA_ERR_BAD_SHAPE;
  if (batch == 0 || heads == 0 || seq_len == 0) return FA_OK;
  if (num_splits <= 0) num_splits = fa_splitkv_num_splits(batch, heads, seq_len, causal);
  if (num_splits > 64) return FA_ERR_BAD_CONFIG;
  if (!part_o || !part_ml) return FA_ERR_WORKSPACE;
  const int bh = batch * heads;
  const unsigned long long rows = (unsigned long long)bh * seq_len;
  if (rows > 0x7fffffffULL) return FA_ERR_BAD_SHAPE;
  hipStream_t stream = (hipStream_t)hip_stream;
  rc = launch(splitkv_cfg(causal), q, k, v, o, bh, seq_len, num_splits, part_o, part_ml, stream);
  if (rc != FA_OK) return rc;
  hipLaunchKernelGGL(fa_splitkv_merge_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0,
                     stream, part_o, part_ml, static_cast<f16*>(o), (int)rows, num_splits);
  return hipGetLastError() == hipSuccess ? FA_OK : FA_ERR_LAUNCH;
}

// ---- introspection -----------------------------------------------------------
extern "C" int fa_num_configs(void) { return kNumConfigs; }

extern "C" int fa_config_info(int config_id, fa_config_info_t* out) {
  if (config_id < 0 || config_id >= kNumConfigs) return FA_ERR_BAD_CONFIG;
  if (!out) return FA_ERR_NULL_POINTER;
  *out = kConfigs[config_id].info;
  return FA_OK;
}

extern "C" int fa_kernel_attrs(int config_id, fa_kernel_attrs_t* out) {
  if (config_id < 0 || config_id >= kNumConfigs) return FA_ERR_BAD_CONFIG;
  if (!out) return FA_ERR_NULL_POINTER;
  hipFuncAttributes a;
  if (hipFuncGetAttributes(&a, (const void*)kConfigs[config_id].fn) != hipSuccess)
    return FA_ERR_HIP;
  out->num_regs = a.numRegs;
  out->local_size_bytes = (int)a.localSizeBytes;
  out->shared_size_bytes = (int)a.sharedSizeBytes;
  out->max_threads_per_block = a.maxThreadsPerBlock;
  out->blocks_per_cu = -1;
  if (prepare(config_id) == FA_OK) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)kConfigs[config_id].fn,
                                                     kConfigs[config_id].info.waves * 64,
                                                     kConfigs[config_id].info.lds_bytes) ==
        hipSuccess)
      out->blocks_per_cu = nb;
  }
  return FA_OK;
}

extern "C" const char* fa_status_string(int status) {
  switch (status) {
    case FA_OK: return "ok";
    case FA_ERR_NULL_POINTER: return "null device pointer";
    case FA_ERR_UNSUPPORTED_HEAD_DIM: return "unsupported head_dim (128 or 64)";
    case FA_ERR_BAD_SHAPE: return "bad shape";
    case FA_ERR_LAUNCH: return "kernel launch failed";
    case FA_ERR_BAD_CONFIG: return "bad tile config";
    case FA_ERR_HIP: return "HIP runtime error";
    case FA_ERR_WORKSPACE: return "split-KV buffers or workspace missing or too small";
    default: return "unknown status";
  }
}

extern "C" const char* fa_version(void) { return "fa_mi355x 0.1 (gfx950)"; }

#ifdef FA_STAMPS
extern "C" int fa_debug_timeline(unsigned long long* out, int n) {
  if (n > FA_MAX_TIMELINE) n = FA_MAX_TIMELINE;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(fa::g_fa_timeline), (size_t)n * 32) == hipSuccess
             ? FA_OK
             : FA_ERR_HIP;
}
extern "C" int fa_debug_stamps(unsigned long long* out, int reset) {
  static unsigned long long all[64][8][12];  // the first 64 workgroups' slots, summed below
  static_assert(sizeof(all) == sizeof(fa::g_fa_stamps), "one slot per workgroup");
  if (hipMemcpyFromSymbol(all, HIP_SYMBOL(fa::g_fa_stamps), sizeof(all)) != hipSuccess)
    return FA_ERR_HIP;
  for (int w = 0; w < 8; ++w)
    for (int i = 0; i < 12; ++i) {
      unsigned long long t = 0;
      for (int b = 0; b < 64; ++b) t += all[b][w][i];
      out[w * 12 + i] = t;
    }
  if (reset) {
    static const unsigned long long z[64][8][12] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(fa::g_fa_stamps), z, sizeof(z)) != hipSuccess) return FA_ERR_HIP;
  }
  return FA_OK;
}
#endif
