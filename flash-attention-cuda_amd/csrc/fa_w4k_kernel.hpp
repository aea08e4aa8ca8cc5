// fa_w4k_kernel.hpp -- short-launch tier: one-wave-per-SIMD segments over a
// workgroup's flattened key tiles (gfx950).
//
// A short launch (B*H*S/64 query blocks of 64 rows within about two per CU)
// has too little work per CU for the persistent W4 kernel's 256-row items:
// config 2 (B=1 H=32 S=1024 causal) is 128 such items whose costs run from
// 4 to 16 key tiles.  Here a workgroup takes one or two 64-row query blocks
// (causal: a heavy and a light block of one head, q and nqb-1-q, so every
// workgroup holds nqb+1 key tiles) and its four waves split the flattened
// list of the blocks' key tiles into contiguous quarters.  Each wave runs
// one segment per block its quarter touches (gen_w4k_item.py: its 64 query
// rows against a run of key tiles, K straight into registers, V by LDS-DMA
// into its own double-buffered image, no barrier) and leaves the segment's
// normalised O (fp16) and per-row log2-sum-exp in LDS; the workgroup then
// merges each block's segments -- the reference's split-K LSE merge
// (flash_attention.cu:559-598) in LDS.
//
// LDS: four 32 KiB V image pairs (a wave's last partial goes into its own
// pair), one 16 KiB slot for the one partial that can end before its wave's
// quarter does (the wave whose quarter crosses from the first block into the
// second), and five 256-B log2-sum-exp rows.
#pragma once

#include "fa_fwd_kernel.hpp"

namespace fa {

constexpr int kW4kPair = 32768;                 // a wave's two V images
constexpr int kW4kEarly = 4 * kW4kPair;          // the crossing wave's first partial
constexpr int kW4kLse = kW4kEarly + 16384;       // log2-sum-exp rows: waves 0-3, early
constexpr int kW4kRec = kW4kLse + 5 * 256;      // segment records: [wave][segment] x 128 B
constexpr int kW4kLdsBytes = kW4kRec + 4 * 2 * 128;

// one segment's scalars, a 32-dword LDS record the segment program reads
// into SGPRs (as inline-asm operands they would leave the register
// allocator too few SGPRs around a statement that clobbers 36 of them)
struct W4kSeg {
  unsigned kd[4], vd[4], qd[4];  // K / V (from the segment's first key) and Q buffer descriptors
  int n;       // key tiles
  int maskj;   // n if the last tile needs a mask (causal diagonal / key bound), else -1
  int kvhi;    // key bound, relative to the segment's first key
  int qm;      // the block's first row, relative to the segment's first key
  unsigned vimg, pslot, lslot;  // LDS: this wave's V image pair, partial O, log2-sum-exp row
  unsigned pad[13];
};
static_assert(sizeof(W4kSeg) == 128, "W4kSeg is one 128-B record");

// per-lane constants (VGPR operands)
struct W4kLane {
  int kg;     // K fragment source: row krow (W4's sigma order), chunk g
  int vd0;    // LDS-DMA source of this lane's 16 B of V piece 0
  int va[2];  // V^T transposed reads (W4's image A addresses, + the wave's pair)
  int vt;     // r16 - 4 sg
  int r16;
  int qoff;   // Q row r16, chunk g
  int pl[4];  // partial row r16, 16-B chunk (c0 + 4 ep) ^ r16
};

__device__ __forceinline__ void put_rsrc(unsigned* w, const void* p, int bytes) {
  const unsigned long long a = (unsigned long long)(uintptr_t)p;
  w[0] = (unsigned)a;
  w[1] = (unsigned)(a >> 32) & 0xffffu;
  w[2] = (unsigned)(bytes < 0 ? 0 : bytes);
  w[3] = 0x00020000u;
}

#include <fa_w4k_item.inc>

template <bool CAUSAL, bool BF16>
__device__ __forceinline__ void w4k_seg(unsigned tab, float c, const W4kLane& ln) {
  if constexpr (CAUSAL && BF16)
    w4k_seg_causal_bf16(tab, c, ln);
  else if constexpr (CAUSAL)
    w4k_seg_causal_f16(tab, c, ln);
  else if constexpr (BF16)
    w4k_seg_noncausal_bf16(tab, c, ln);
  else
    w4k_seg_noncausal_f16(tab, c, ln);
}

__device__ __forceinline__ W4kLane w4k_lane(int vimg, int lane) {
  W4kLane ln;
  const int r16 = lane & 15, g = lane >> 4, sg = ((g & 1) << 1) | (g >> 1);
  const int krow = 4 * ((((r16 >> 2) & 1) << 1) | (r16 >> 3)) + (r16 & 3);
  ln.kg = krow * ROW_BYTES + 16 * g;
  ln.vd0 = lds_off_src(16 * lane);
  const int qq = r16 >> 2, pp = r16 & 3;
#pragma unroll
  for (int ep = 0; ep < 2; ++ep)
    ln.va[ep] = vimg + 2048 * (sg >> 1) + 64 * (4 * (sg & 1) + qq) + 16 * ((2 * ep + (pp >> 1)) ^ sg) +
                8 * (pp & 1);
  ln.vt = r16 - 4 * sg;
  ln.r16 = r16;
  ln.qoff = r16 * ROW_BYTES + 16 * g;
  const int c0 = 2 * (g & 1) + (g >> 1);
#pragma unroll
  for (int ep = 0; ep < 4; ++ep) ln.pl[ep] = 256 * r16 + 16 * ((c0 + 4 * ep) ^ r16);
  return ln;
}

// the workgroup's blocks: causal pairs (heavy nqb-1-i, light i) of one head
// when two blocks per workgroup, else consecutive blocks
struct W4kBlocks {
  int nb;
  int bh[2], qb[2], nt[2];
  // block s's fields by select (a dynamic index would put the arrays in scratch)
  __device__ __forceinline__ int BH(int s) const { return s ? bh[1] : bh[0]; }
  __device__ __forceinline__ int QB(int s) const { return s ? qb[1] : qb[0]; }
  __device__ __forceinline__ int NT(int s) const { return s ? nt[1] : nt[0]; }
};

template <bool CAUSAL>
__device__ __forceinline__ W4kBlocks w4k_blocks(const FwdParams& p, int work) {
  W4kBlocks wb;
  const int nqb = p.nqb, ntk = (p.seq_len + 63) >> 6;
  const long long total = (long long)p.bh * nqb;
  const long long first = (long long)work * p.w4k_per;
  wb.nb = (int)min((long long)p.w4k_per, total - first);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const long long idx = first + (i < wb.nb ? i : 0);
    const int h = (int)(idx / nqb), r = (int)(idx - (long long)h * nqb);
    const int qb = (CAUSAL && p.w4k_per == 2) ? ((r & 1) ? (r >> 1) : nqb - 1 - (r >> 1)) : r;
    wb.bh[i] = h;
    wb.qb[i] = qb;
    wb.nt[i] = CAUSAL ? min(qb + 1, ntk) : ntk;
  }
  return wb;
}

// wave w's quarter [c0, c1) of the flattened tiles, clipped to block s: the
// segment's tiles [a, e) within the block (a >= e: none)
__device__ __forceinline__ void w4k_quarter(const W4kBlocks& wb, int w, int s, int& a, int& e) {
  const int T = wb.nt[0] + (wb.nb > 1 ? wb.nt[1] : 0);
  const int c0 = (w * T) >> 2, c1 = ((w + 1) * T) >> 2;
  const int off = s == 0 ? 0 : wb.nt[0];
  a = max(c0, off) - off;
  e = min(c1, off + wb.NT(s)) - off;
}

// partial slot of wave w's segment in block s: its V image pair when it is
// the wave's last segment (the quarter ends in block s), else the early slot
__device__ __forceinline__ bool w4k_is_last(const W4kBlocks& wb, int w, int s) {
  if (s == wb.nb - 1) return true;
  int a, e;
  w4k_quarter(wb, w, s + 1, a, e);
  return a >= e;  // no segment in the next block
}

template <bool CAUSAL, bool BF16>
__global__ __launch_bounds__(256, 1) void fa_fwd_f16_w4k_kernel(FwdParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lds = lds_addr(smem);
  // XCD-affine: the workgroups of one XCD take consecutive work (the blocks
  // of a head stay on one L2)
  const int c8 = (p.w4k_groups + 7) >> 3;
  const int work = (blockIdx.x & 7) * c8 + (blockIdx.x >> 3);
  if (work >= p.w4k_groups) return;
  const int S = p.seq_len;
  const W4kBlocks wb = w4k_blocks<CAUSAL>(p, work);
  const int vimg = lds + kW4kPair * wave;
  for (int s = 0; s < wb.nb; ++s) {
    int a, e;
    w4k_quarter(wb, wave, s, a, e);
    if (a >= e) continue;
    const bool last = w4k_is_last(wb, wave, s);
    const int q0 = 64 * wb.QB(s), k0 = 64 * a;
    const int kvlim = CAUSAL ? min(q0 + 64, S) : S;
    const size_t head_off = (size_t)wb.BH(s) * (size_t)S * HD;
    const int kbytes = (min(64 * e, kvlim) - k0) * ROW_BYTES;
    W4kSeg sg;
    put_rsrc(sg.kd, p.k + head_off + (size_t)k0 * HD, kbytes);
    put_rsrc(sg.vd, p.v + head_off + (size_t)k0 * HD, kbytes);
    put_rsrc(sg.qd, p.q + head_off + (size_t)q0 * HD, (min(q0 + 64, S) - q0) * ROW_BYTES);
    sg.n = e - a;
    sg.kvhi = kvlim - k0;
    sg.qm = q0 - k0;
    // the last tile (keys [64 (n-1), 64 n) of the segment) needs a mask iff it
    // reaches the key bound or (causal) passes the block's first row
    const bool m = 64 * sg.n > sg.kvhi || (CAUSAL && 64 * sg.n - 1 > sg.qm);
    sg.maskj = m ? sg.n : -1;
    sg.vimg = (unsigned)vimg;
    sg.pslot = (unsigned)(last ? vimg : lds + kW4kEarly);
    sg.lslot = (unsigned)(lds + kW4kLse + 256 * (last ? wave : 4));
    const int rec = kW4kRec + 128 * (2 * wave + s);
    if (lane == 0) {
      u32x4* r = reinterpret_cast<u32x4*>(smem + rec);
      r[0] = u32x4{sg.kd[0], sg.kd[1], sg.kd[2], sg.kd[3]};
      r[1] = u32x4{sg.vd[0], sg.vd[1], sg.vd[2], sg.vd[3]};
      r[2] = u32x4{sg.qd[0], sg.qd[1], sg.qd[2], sg.qd[3]};
      r[3] = u32x4{(unsigned)sg.n, (unsigned)sg.maskj, (unsigned)sg.kvhi, (unsigned)sg.qm};
      r[4] = u32x4{sg.vimg, sg.pslot, sg.lslot, 0u};
    }
    // rebuilt per segment so none of the lane constants is live across the
    // statement (it leaves the compiler 20 VGPRs)
    int lane_c = lane;
    asm volatile("" : "+v"(lane_c));
    const W4kLane ln = w4k_lane(vimg, lane_c);
    w4k_seg<CAUSAL, BF16>((unsigned)(lds + rec), p.c, ln);
  }
  __syncthreads();
#ifdef FA_W4K_STAMPS
  // diagnostic build: each (wave, segment)'s four s_memtime stamps (start,
  // prologue done, drain, epilogue done) to O row q0(block 0) + 2 wave + s
  if (lane < 2 * 4) {
    const int w = lane >> 1, s = lane & 1;
    const u32x4* st = reinterpret_cast<const u32x4*>(smem + kW4kLse + 256 * (w4k_is_last(wb, w, s) ? w : 4));
    int a, e;
    w4k_quarter(wb, w, s, a, e);
    if (s < wb.nb && a < e) {
      f16* row = p.o + (size_t)wb.BH(0) * (size_t)S * HD + (size_t)(64 * wb.QB(0) + 2 * w + s) * HD;
      reinterpret_cast<u32x4*>(row)[0] = st[0];
      reinterpret_cast<u32x4*>(row)[1] = st[1];
      reinterpret_cast<u32x4*>(row)[2] = u32x4{(unsigned)e - (unsigned)a, (unsigned)blockIdx.x, 0u, 0u};
    }
  }
  return;
#endif
  // merge: per block, the partials of the waves whose quarters touch it,
  // O = sum_s 2^(lse_s - M) O_s / sum_s 2^(lse_s - M)
  for (int s = 0; s < wb.nb; ++s) {
    int so[4], lo[4], np = 0;
    bool has[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      int a, e;
      w4k_quarter(wb, w, s, a, e);
      has[w] = a < e;
      const bool last = w4k_is_last(wb, w, s);
      so[w] = last ? kW4kPair * w : kW4kEarly;
      lo[w] = kW4kLse + 256 * (last ? w : 4);
      np += has[w] ? 1 : 0;
    }
    const int q0 = 64 * wb.QB(s);
    f16* const orow = p.o + (size_t)wb.BH(s) * (size_t)S * HD + (size_t)q0 * HD;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int u = tid + 256 * r, row = u >> 4, ch = u & 15;
      if (q0 + row >= S) continue;
      const int off = 256 * row + 16 * (ch ^ (row & 15));
      u32x4 out;
      if (np == 1) {
        int one = so[0];
#pragma unroll
        for (int w = 1; w < 4; ++w) one = has[w] ? so[w] : one;
        out = *reinterpret_cast<const u32x4*>(smem + one + off);
      } else {
        float lse[4], M = -__builtin_inff();
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          lse[w] = has[w] ? *reinterpret_cast<const float*>(smem + lo[w] + 4 * row) : -__builtin_inff();
          M = fmaxf(M, lse[w]);
        }
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, den = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          if (!has[w]) continue;
          const float wgt = M == -__builtin_inff() ? 0.f : __builtin_amdgcn_exp2f(lse[w] - M);
          den += wgt;
          const u32x4 raw = *reinterpret_cast<const u32x4*>(smem + so[w] + off);
#pragma unroll
          for (int x = 0; x < 4; ++x) {
            float flo, fhi;
            if constexpr (BF16) {
              flo = __builtin_bit_cast(float, raw[x] << 16);
              fhi = __builtin_bit_cast(float, raw[x] & 0xffff0000u);
            } else {
              flo = (float)__builtin_bit_cast(f16, (unsigned short)(raw[x] & 0xffffu));
              fhi = (float)__builtin_bit_cast(f16, (unsigned short)(raw[x] >> 16));
            }
            acc[2 * x] = fmaf(wgt, flo, acc[2 * x]);
            acc[2 * x + 1] = fmaf(wgt, fhi, acc[2 * x + 1]);
          }
        }
        const float inv = den > 0.f ? 1.0f / den : 0.f;
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          unsigned ulo, uhi;
          if constexpr (BF16) {
            ulo = __builtin_bit_cast(unsigned short, (__bf16)(acc[2 * x] * inv));
            uhi = __builtin_bit_cast(unsigned short, (__bf16)(acc[2 * x + 1] * inv));
          } else {
            ulo = __builtin_bit_cast(unsigned short, (f16)(acc[2 * x] * inv));
            uhi = __builtin_bit_cast(unsigned short, (f16)(acc[2 * x + 1] * inv));
          }
          out[x] = ulo | (uhi << 16);
        }
      }
      *reinterpret_cast<u32x4*>(orow + (size_t)row * HD + 8 * ch) = out;
    }
  }
}

}  // namespace fa
