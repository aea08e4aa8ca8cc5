// fa_fwd_kernel.hpp -- gfx950 (MI355X, CDNA4) fused attention forward tile loop.
//
// Re-designed for 64-lane waves and MFMA, not a translation of the reference's
// mma.sync/ldmatrix kernel (flash_attention.cu:67-554).  What it computes is
// the reference's contract: per (batch*head, query block) one workgroup runs
// QK^T -> online softmax -> PV over key/value tiles and writes O in fp16
// (:103-122 work mapping, :188-334 tile math, :497-553 epilogue).
//
// Structure (per wave = 32 query rows, per workgroup = WAVES*32 rows):
//  * Swapped first product  S^T = K . Q^T : A = K tile rows from LDS
//    (ds_read_b128), B = Q held in 32 VGPRs for the whole key loop.  The
//    accumulator puts the query on the lane and keys in registers, so row
//    max / row sum are per-lane scalars plus cross-row v_permlane*_swap
//    exchanges -- no LDS round trip, no shuffles.
//  * Second product  O^T = V^T . P^T : P^T is the first product's accumulator
//    converted to fp16 in place (B operand, no lane movement); V^T comes from
//    the row-major V tile through ds_read_b64_tr_b16 (hardware transpose
//    read) -- the MI355X replacement for ldmatrix.x2.trans (:305-310).
//  * K/V tiles: raw buffer loads (hardware range check zero-fills rows past
//    the key range -- no per-lane bounds branches; scalar descriptor math),
//    register-staged, double-buffered in LDS, one barrier per tile: the loads
//    of tile j+1 are issued before tile j's MFMAs and written to the other
//    LDS buffer after them.  The loop is unrolled by two so every LDS address
//    is a per-lane base + immediate.
//  * Online softmax in the exp2 domain with the scale folded into one FMA
//    and a lazy rescale: O and l are rescaled only when some row max grew
//    by more than RESCALE_LOG2 (P stays <= 2^RESCALE_LOG2, exact fp16 range),
//    wave-uniform branch.
//  * Causal: waves skip key tiles entirely above their diagonal; the block
//    ordering (heaviest first, XCD-aware) lives in fa_fwd.hip.
//
// The tile math is the M16 policy below: v_mfma_f32_16x16x32_f16, two
// 16-query blocks per wave (the shape that holds the higher clock under load,
// profiles/r01_mfma_rate_probe.jsonl).  The one-wave-per-SIMD persistent
// kernel (64 rows per wave, asm-owned register file) is fa_w4_kernel.hpp.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace fa {

typedef _Float16 f16;
typedef f16 f16x8 __attribute__((ext_vector_type(8)));
typedef f16 f16x4 __attribute__((ext_vector_type(4)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

constexpr int HD = 128;            // head_dim (the reference hard-codes 128, :613)
constexpr int ROW_BYTES = HD * 2;  // one K/V/Q row in bytes
constexpr float RESCALE_LOG2 = 8.0f;
// The product library is built from these sources as they stand: no build
// flag may change what a kernel computes.  Timing-only diagnostic builds
// (wrong results by design) live in git history, not behind macros here.
#if defined(FA_DIAG_NO_LDS) || defined(FA_DIAG_NO_MERGE) || defined(FA_DIAG_W4_NO_STAGE) || \
    defined(FA_DIAG_FREE_CONTRACT) || defined(FA_NARROW_STORE) || defined(FA_ROWSUM_VALU)
#error "removed A/B knob: the product sources take no result-changing -D flags"
#endif
// attention_kvpair: 4 tile buffers (64 KB) + the shared Q block (4 x 8 KB);
// the merge region reuses the tile buffers
constexpr int kKvpairLdsBytes = 4 * 64 * 256 + 4 * 8 * 64 * 16;
// KV-quad: four double-width (128-key) stage buffers
constexpr int kKvquadLdsBytes = 4 * 2 * 64 * 256;

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
  int band;        // causal: query blocks of one head kept together on an XCD
  // causal split tier (fa_fwd_*_ws, fa_w4_kernel.hpp): the workspace's
  // arrival counters [bh][nqb], per-row log2-sum-exp and normalised partial
  // O slabs [bh][nqb][pmax][256 rows], and the 64-key tiles per key piece
  unsigned* ws_ctr;
  float* ws_lse;
  char* ws_o;
  int piece_tiles;
  int pmax;
  // W4P planned grouping (fa_w4p_kernel.hpp G = 4): workgroup rank r of a
  // head runs the 64-row blocks plan[4 r .. 4 r + 3] (0xff = none)
  unsigned char plan[256];
};

// ---------------------------------------------------------------------------
// small device helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes < 0 ? 0 : bytes,
                                           0x00020000);
}
__device__ __forceinline__ f16x8 buf_load16(__amdgpu_buffer_rsrc_t r, int voff) {
  return __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0));
}
// row offset in the scalar soffset operand: one address VGPR for all passes
__device__ __forceinline__ f16x8 buf_load16s(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
__device__ __forceinline__ void buf_store8(__amdgpu_buffer_rsrc_t r, int voff, f16x4 v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, voff, 0, 0);
}
__device__ __forceinline__ void buf_store16f(__amdgpu_buffer_rsrc_t r, int voff, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, voff, 0, 0);
}

// LDS-DMA: one 16-B global load per lane written straight into LDS at
// lds_base + 16*lane (buffer_load_dwordx4 ... lds; no VGPR destination).
// Completion is counted by vmcnt like any load.
// Inline asm, not the builtin: for the builtin hipcc inserts vmcnt(0) before
// every later LDS read (it cannot tell which buffer the DMA writes), which
// serialises each MFMA block behind the next tile's load.  The asm is
// invisible to hipcc's waitcnt bookkeeping, so completion is waited for
// explicitly (s_waitcnt vmcnt) before the barrier that publishes the tile.
// M0 (LDS base) is saved and restored inside the statement (hipcc reserves it).
__device__ __forceinline__ void buf_load16_lds(__amdgpu_buffer_rsrc_t r, void* lds_base, int voff) {
  const unsigned lds = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)lds_base;
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %2, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(voff), "s"(r)
      : "memory");
}

// LDS image A: 8-row x 32-column subtiles of 512 B, 16-B chunk XOR (row>>2)&3.
// Conflict-free for ds_read_b64_tr_b16 column reads (both MFMA shapes) and
// for the 32x32x16 ds_read_b128 row reads.
__device__ __forceinline__ int lds_off(int row, int ch) {
  return 2048 * (row >> 3) + 512 * (ch >> 2) + 64 * (row & 7) +
         16 * ((ch & 3) ^ ((row >> 2) & 3));
}
// LDS image B: plain 256-B rows, chunk XOR (row&15).  Conflict-free for the
// 16x16x32 ds_read_b128 row reads.
__device__ __forceinline__ int k_off16(int row, int ch) { return 256 * row + 16 * (ch ^ (row & 15)); }
// inverses (LDS byte offset o within a tile image -> tile-relative source
// byte offset row*256 + ch*16), for LDS-DMA, whose destination is lane-linear
__device__ __forceinline__ int k_off16_src(int o) {
  const int row = o >> 8;
  return 256 * row + 16 * (((o >> 4) & 15) ^ (row & 15));
}
__device__ __forceinline__ int lds_off_src(int o) {
  const int row = 8 * (o >> 11) + ((o >> 6) & 7);
  return 256 * row + 16 * (4 * ((o >> 9) & 3) + (((o >> 4) & 3) ^ ((row >> 2) & 3)));
}

__device__ __forceinline__ float max_xor32(float x) {
  // lanes l and l^32 exchange; r[0] = {x[0..31], x[0..31]}, r[1] = {x[32..63], x[32..63]}
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float sum_xor32(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float max_xor16(float x) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
}
__device__ __forceinline__ float sum_xor16(float x) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(a[0]) + __uint_as_float(a[1]);
}

__device__ __forceinline__ f16x4 lds_read_tr(const char* base, int off) {
  typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
  i16x4 t = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + off));
  return __builtin_bit_cast(f16x4, t);
}

__device__ __forceinline__ float ninf() { return -__builtin_inff(); }

// Cache policy of the O stores: sc1 (write-through; the line leaves the
// XCD's L2 with the store).  O is written once and never re-read by the
// kernel; on the short tiers, where every workgroup stores at the end of the
// launch, write-through drains the tail faster: B=1 H=32 S=512 non-causal
// 300 -> 316, S=1024 causal 392 -> 415 TFLOP/s; nt +1-3 %; the persistent
// tier is level (+-0.3 %) (profiles/r02_ab_o_store_policy.jsonl).  Buffer
// store aux bits: 2 = nt, 16 = sc1.
// head_dim 64 non-causal ping-pong schedule: the causal one (next tile's
// loads issued in the MFMA phase, written at the start of the softmax phase,
// O stored right after the last PV).  With half the MFMAs per tile the MFMA
// phase is the short one at d64, the reverse of d128; +15-20 % at S=2048-16384
// fp16 and bf16, bit-identical (profiles/r02_ab_d64_noncausal_sched.jsonl).
constexpr bool kNcD64IssueInSm = false;
constexpr bool kNcD64WriteEarly = true;
constexpr bool kNcD64EarlyStore = true;
constexpr int kOStoreAux = 16;

// 32-bit LDS address of a pointer into the workgroup's shared memory
__device__ __forceinline__ int lds_addr(const void* p) {
  return (int)(unsigned)(uintptr_t)(__attribute__((address_space(3))) const void*)p;
}

#ifdef FA_STAMPS
// diagnostic build only (lib/libfa_mi355x_stamps.so): per-wave cycles spent in
// [MFMA block, barrier after it, softmax block, barrier after it, LDS tile write] of
// the first 64 workgroups, one slot each (plain stores: atomics on shared
// counters would slow exactly those workgroups and show in the timeline),
// summed by fa_debug_stamps.  Never part of the product library.
__device__ unsigned long long g_fa_stamps[64][8][12];  // 5 phases, issue_tile, iterations, prologue, epilogue, items
// per-workgroup timeline: {start, end (s_memrealtime, 100 MHz), hw_id | xcc_id << 32 | qb << 40,
//                          shader cycles (s_memtime) start..end}
constexpr int FA_MAX_TIMELINE = 65536;
__device__ unsigned long long g_fa_timeline[FA_MAX_TIMELINE][4];  // + shader cycles
#endif

// ---------------------------------------------------------------------------
// Policies.  Each holds one wave's state (Q fragments, O accumulator, running
// max/sum, the current S^T tile and its fp16 P) and splits a key tile into
//   qk(kb)       : S^T = K . Q^T            (MFMA, K tile from LDS)
//   softmax(...) : mask, online max/rescale, P = exp2(S*c - m*c), row sums (VALU)
//   pv(vb)       : O^T += V^T . P^T          (MFMA, V tile from LDS)
// so the ping-pong skeleton can pair one wave's MFMA block with its SIMD
// partner's softmax.
// ---------------------------------------------------------------------------

// ---------------------------------------------------------------------------
// M16: v_mfma_f32_16x16x32_f16, two 16-query blocks b per wave
//   S^T[b][c] (16 keys x 16 q): lane holds q = 16b + (lane&15),
//       keys 16c + 4*sg + i, g = lane>>4, sg = swap2(g) -- the K rows are
//       read permuted (sigma) so the PV transposed reads of one 32-lane half
//       hit rows 8 apart: bank-conflict-free in image A.
//   O^T[b][e] (16 d x 16 q):  lane holds q = 16b + (lane&15), d = 16e + 4g + i
// K tile: image B (conflict-free 16x16x32 row reads); V tile: image A.
//
// Softmax (the reference's online softmax, flash_attention.cu:235-288, in the
// exp2 domain) with two VALU passes moved onto the matrix pipe:
//  * Q is pre-scaled once by c = scale*log2(e) (fp16), and every QK^T MFMA
//    chain starts from C = -m_ref (broadcast per query), so the accumulator
//    already holds x = s*c - m_ref and P = exp2(x) needs no FMA.
//  * Tile row sums come from one extra MFMA per 32 keys (ones . P): no VALU
//    adds, and l sums exactly the fp16-rounded P the PV product uses.
//  * m_ref moves (O and l rescaled) only when a row max grew by more than
//    RESCALE_LOG2 (wave-uniform branch).
// ---------------------------------------------------------------------------

// 16-bit element type of Q/K/V/O and of the MFMA operands: fp16 (the
// reference's type) or bf16.  Storage, LDS images and transposed reads are
// bit-identical for both; only the MFMA opcode and the fp32 <-> 16-bit
// conversions differ.
template <class T>
struct Elem {
  typedef T x8 __attribute__((ext_vector_type(8)));
  typedef T x4 __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ f32x4 mfma(x8 a, x8 b, f32x4 c) {
    if constexpr (std::is_same<T, __bf16>::value)
      return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    else
      return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};

template <int BN_, class T = f16, int HDIM_ = 128, int QB_ = 2>
struct M16 {
  static_assert(QB_ == 2, "two 16-row query blocks per wave (the merge layouts assume it)");
  static_assert(HDIM_ == 64 || HDIM_ == 128, "head_dim 64 or 128");
  static constexpr int BN = BN_;
  static constexpr int HDIM = HDIM_;      // head_dim
  static constexpr int ROW = 2 * HDIM;    // bytes per Q/K/V/O row in HBM
  static constexpr int NTQ = HDIM / 32;   // 32-wide k-steps of QK^T (Q fragments per 16 rows)
  static constexpr int NE = HDIM / 16;    // 16-wide d-blocks of O
  static constexpr int RPW = 512 / HDIM;  // tile rows one wave stages per pass (64 lanes x 16 B)
  // LDS images keep 256-B row slots at either head_dim (a 64-wide row uses
  // half of each slot), so every address formula and its bank analysis is
  // the head_dim-128 one.
  static constexpr int NKB = BN / 16;  // 16-key blocks per tile
  static constexpr int NU = BN / 32;   // 32-key PV steps per tile
  static constexpr int QB = QB_;       // 16-row query blocks per wave (32 rows)
  static constexpr int RW = 16 * QB;   // query rows per wave
  typedef typename Elem<T>::x8 tx8;
  typedef typename Elem<T>::x4 tx4;
  // bf16: Q enters the MFMA unscaled and the fp32 scores are multiplied by c
  // (C = -m_ref / c): a bf16-rounded Q * c (8 mantissa bits) cost 3x SDPA's
  // error on peaked inputs.  fp16 keeps Q * c.
  static constexpr bool kScaleS = std::is_same<T, __bf16>::value;
  int lane, r16, g, sg;
  int kaddr[4], vaddr[2];
  tx8 qf[QB][NTQ];
  f32x4 acc[QB][NE];
  f32x4 s[QB][NKB];
  tx8 pf[QB][NU];
  f32x4 negm[QB];     // C operand of the QK^T chains: -m_ref broadcast
  float m_ref[QB];    // reference max, log2 units (x = s*c - m_ref)
  f32x4 lacc[QB];     // running row sums l (ones . P on the matrix pipe, in the PV chain)
  bool have_ref;     // wave-uniform: a tile has set m_ref
  float c;

  __device__ __forceinline__ void init(int lane_, float c_) {
    lane = lane_;
    c = c_;
    r16 = lane & 15;
    g = lane >> 4;
    sg = ((g & 1) << 1) | (g >> 1);
    const int krow = 4 * ((((r16 >> 2) & 1) << 1) | (r16 >> 3)) + (r16 & 3);  // sigma(r16)
#pragma unroll
    for (int t = 0; t < 4; ++t) kaddr[t] = k_off16(krow, 4 * t + g);  // t < NTQ used
    const int i = lane & 15, qq = i >> 2, pp = i & 3;
#pragma unroll
    for (int ep = 0; ep < 2; ++ep)
      vaddr[ep] = 2048 * (sg >> 1) + 64 * (4 * (sg & 1) + qq) + 16 * ((2 * ep + (pp >> 1)) ^ sg) +
                  8 * (pp & 1);
#pragma unroll
    for (int b = 0; b < QB; ++b) {
#pragma unroll
      for (int e = 0; e < NE; ++e) acc[b][e] = f32x4{};
      negm[b] = f32x4{};
      m_ref[b] = 0.f;
      lacc[b] = f32x4{};
    }
    have_ref = false;
  }
  // Q: qf[b][t] = c * Q[qw + 16b + r16][32t + 8g .. +7]   (rounded to fp16)
  __device__ __forceinline__ void issue_q(__amdgpu_buffer_rsrc_t rq, int qw) {
#pragma unroll
    for (int b = 0; b < QB; ++b)
#pragma unroll
      for (int t = 0; t < NTQ; ++t)
        qf[b][t] = __builtin_bit_cast(
            tx8, buf_load16(rq, (qw + 16 * b + r16) * ROW + (4 * t + g) * 16));
  }
  __device__ __forceinline__ void scale_q() {
    if constexpr (kScaleS) {
      pin_q();
      return;
    }
#pragma unroll
    for (int b = 0; b < QB; ++b)
#pragma unroll
      for (int t = 0; t < NTQ; ++t)
#pragma unroll
        for (int j = 0; j < 8; ++j) qf[b][t][j] = (T)((float)qf[b][t][j] * c);
    pin_q();
  }
  // Q shared by the NPART partial waves of one row set (KV-quad): partial j
  // loads and scales only the chunks i = NTQ*b + t with i % NPART == j, parks them
  // lane-linearly in LDS, and reads the others' after the prologue barrier --
  // one global read of each Q chunk per workgroup instead of NPART
  static constexpr int Q_SHARE_BYTES = QB * NTQ * 64 * 16;
  template <int NPART>
  __device__ __forceinline__ void issue_q_part(__amdgpu_buffer_rsrc_t rq, int qw, int j) {
#pragma unroll
    for (int b = 0; b < QB; ++b)
#pragma unroll
      for (int t = 0; t < NTQ; ++t)
        if ((b * NTQ + t) % NPART == j)
          qf[b][t] = __builtin_bit_cast(
              tx8, buf_load16(rq, (qw + 16 * b + r16) * ROW + (4 * t + g) * 16));
  }
  template <int NPART>
  __device__ __forceinline__ void scale_put_q_part(char* region, int j) {
#pragma unroll
    for (int b = 0; b < QB; ++b)
#pragma unroll
      for (int t = 0; t < NTQ; ++t)
        if ((b * NTQ + t) % NPART == j) {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if constexpr (!kScaleS) qf[b][t][e] = (T)((float)qf[b][t][e] * c);
          reinterpret_cast<tx8*>(region)[(b * NTQ + t) * 64 + lane] = qf[b][t];
        }
  }
  template <int NPART>
  __device__ __forceinline__ void get_q_rest(const char* region, int j) {
#pragma unroll
    for (int b = 0; b < QB; ++b)
#pragma unroll
      for (int t = 0; t < NTQ; ++t)
        if ((b * NTQ + t) % NPART != j) qf[b][t] = reinterpret_cast<const tx8*>(region)[(b * NTQ + t) * 64 + lane];
    pin_q();
  }
  // materialise the scaled Q here: otherwise hipcc sinks the scaling VALU past
  // the prologue barrier to the first MFMA, where its vmcnt waits also cover
  // every tile load issued since (a full memory latency per item)
  __device__ __forceinline__ void pin_q() {
#pragma unroll
    for (int b = 0; b < QB; ++b)
#pragma unroll
      for (int t = 0; t < NTQ; ++t) asm volatile("" : "+v"(qf[b][t]));
  }
  __device__ __forceinline__ void load_q(__amdgpu_buffer_rsrc_t rq, int qw) {
    issue_q(rq, qw);
    scale_q();
  }
  // K staging: natural row-major lanes (8 lanes = 8 chunks of one row: conflict-free
  // writes into image B); V staging: each group of 8 lanes = two rows of opposite
  // parity x 4 chunks (conflict-free writes into image A).  A wave stages RPW rows
  // per pass: 4 rows x 16 chunks (head_dim 128) or 8 rows x 8 chunks (64).
  __device__ __forceinline__ int k_stage_row(int wave) const {
    return HDIM == 128 ? 4 * wave + (lane >> 4) : 8 * wave + (lane >> 3);
  }
  __device__ __forceinline__ int k_stage_ch() const { return HDIM == 128 ? lane & 15 : lane & 7; }
  __device__ __forceinline__ int v_stage_row(int wave) const {
    return HDIM == 128 ? 4 * wave + 2 * ((lane >> 5) & 1) + ((lane >> 2) & 1)
                       : 8 * wave + 2 * ((lane >> 4) & 3) + ((lane >> 2) & 1);
  }
  __device__ __forceinline__ int v_stage_ch() const {
    return HDIM == 128 ? 4 * ((lane >> 3) & 3) + (lane & 3) : 4 * ((lane >> 3) & 1) + (lane & 3);
  }
  static __device__ __forceinline__ int k_lds(int row, int ch) { return k_off16(row, ch); }
  static __device__ __forceinline__ int v_lds(int row, int ch) { return lds_off(row, ch); }
  static __device__ __forceinline__ int k_src(int o) { return k_off16_src(o); }
  static __device__ __forceinline__ int v_src(int o) { return lds_off_src(o); }

  __device__ __forceinline__ void qk(const char* kb) {
#pragma unroll
    for (int t = 0; t < NTQ; ++t)
#pragma unroll
      for (int cb = 0; cb < NKB; ++cb) {
        const tx8 kf = *reinterpret_cast<const tx8*>(kb + kaddr[t] + 4096 * cb);
#pragma unroll
        for (int b = 0; b < QB; ++b)
          s[b][cb] = Elem<T>::mfma(kf, qf[b][t], t == 0 ? negm[b] : s[b][cb]);
      }
  }
  // P = exp2(x) -> fp16, already in the B-operand layout of the PV product
  __device__ __forceinline__ void exp_p() {
#pragma unroll
    for (int b = 0; b < QB; ++b)
#pragma unroll
      for (int cb = 0; cb < NKB; ++cb)
#pragma unroll
        for (int i = 0; i < 4; ++i) pf[b][cb >> 1][4 * (cb & 1) + i] = (T)__builtin_amdgcn_exp2f(s[b][cb][i]);
  }
  template <bool CAUSAL>
  __device__ __forceinline__ void softmax(int kv0, int kv_hi, int qw, float /*c*/, bool need_mask) {
    if constexpr (kScaleS) {
#pragma unroll
      for (int b = 0; b < QB; ++b)
#pragma unroll
        for (int cb = 0; cb < NKB; ++cb) s[b][cb] *= c;
    }
    if (need_mask) {
#pragma unroll
      for (int b = 0; b < QB; ++b) {
        const int qrow = qw + 16 * b + r16;
#pragma unroll
        for (int cb = 0; cb < NKB; ++cb)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int kv = kv0 + 16 * cb + 4 * sg + i;
            const bool ok = kv < kv_hi && (!CAUSAL || kv <= qrow);
            s[b][cb][i] = ok ? s[b][cb][i] : ninf();
          }
      }
    }
    // row max relative to m_ref; shift m_ref (and rescale O, l) only when it
    // grew by more than RESCALE_LOG2 -- P then stays <= 2^RESCALE_LOG2
    float mx[QB];
    bool grow = !have_ref;
#pragma unroll
    for (int b = 0; b < QB; ++b) {
      float m = s[b][0][0];
#pragma unroll
      for (int cb = 0; cb < NKB; ++cb)
#pragma unroll
        for (int i = (cb == 0 ? 1 : 0); i < 4; ++i) m = fmaxf(m, s[b][cb][i]);
      // a row's max exceeds the threshold iff one of its 4 lanes' partial
      // maxima does: the cross-lane reduction is only needed on the rare
      // (wave-uniform) rescale path
      mx[b] = m;
      grow |= mx[b] > RESCALE_LOG2;
    }
    if (__any(grow)) {
#pragma unroll
      for (int b = 0; b < QB; ++b) mx[b] = max_xor32(max_xor16(mx[b]));
#pragma unroll
      for (int b = 0; b < QB; ++b) {
        // first tile: centre on the max; later: only ever move m_ref up.
        // A row with every key masked (mx = -inf) keeps m_ref.
        float sh = have_ref ? fmaxf(mx[b], 0.f) : mx[b];
        sh = sh == ninf() ? 0.f : sh;
        if (have_ref) {
          const float alpha = __builtin_amdgcn_exp2f(-sh);
#pragma unroll
          for (int e = 0; e < NE; ++e) acc[b][e] *= alpha;
          lacc[b] *= alpha;
        }
#pragma unroll
        for (int cb = 0; cb < NKB; ++cb) s[b][cb] -= sh;
        m_ref[b] += sh;
        const float nm = kScaleS ? -m_ref[b] / c : -m_ref[b];
        negm[b] = f32x4{nm, nm, nm, nm};
      }
      have_ref = true;
    }
    exp_p();
  }
  __device__ __forceinline__ void pv(const char* vb) {
    const tx8 ones = {(T)1.f, (T)1.f, (T)1.f, (T)1.f, (T)1.f, (T)1.f, (T)1.f, (T)1.f};
#pragma unroll
    for (int u = 0; u < NU; ++u) {
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        const int base = 8192 * u + 512 * (e >> 1) + vaddr[e & 1];
        const tx4 lo = __builtin_bit_cast(tx4, lds_read_tr(vb, base));
        const tx4 hi = __builtin_bit_cast(tx4, lds_read_tr(vb, base + 4096));
        const tx8 vf = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int b = 0; b < QB; ++b)
          acc[b][e] = Elem<T>::mfma(vf, pf[b][u], acc[b][e]);
      }
      // row sums of the same fp16 P: every register of lacc[b] = l for q = lane&15
#pragma unroll
      for (int b = 0; b < QB; ++b)
        lacc[b] = Elem<T>::mfma(ones, pf[b][u], lacc[b]);
    }
  }
  // the ping-pong MFMA block: PV(V_{k-1}) then QK^T(K_k); the barrier keeps the
  // scheduler from hoisting QK's LDS reads into PV (register pressure)
  // LDS reads kept in flight ahead of the MFMAs that consume them: 4 K reads
  // (A/B +3-6 %), 8 V reads (pins the schedule in every instantiation)
  static constexpr int kQkPipe = 4, kPvPipe = 8;
  __device__ __forceinline__ void mfma_block(const char* kb, const char* vb, bool do_pv, bool do_qk) {
    if (do_pv) {
      pv(vb);
      constexpr int PV_READS = 2 * NE * NU, PV_MFMAS = 2 * NE * NU + 2 * NU;
      constexpr int PV_AHEAD = kPvPipe < PV_READS ? kPvPipe : PV_READS;
      __builtin_amdgcn_sched_group_barrier(0x100, PV_AHEAD, 0);
#pragma unroll
      for (int i = 0; i < (PV_READS - PV_AHEAD) / 2; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, PV_MFMAS, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (do_qk) {
      qk(kb);
      constexpr int QK_READS = NTQ * NKB;
      __builtin_amdgcn_sched_group_barrier(0x100, kQkPipe, 0);
#pragma unroll
      for (int i = 0; i < QK_READS - kQkPipe; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * kQkPipe, 0);
    }
  }
  template <bool CAUSAL>
  __device__ __forceinline__ void tile(const char* kb, const char* vb, int kv0, int kv_hi, int qw,
                                       float c_, bool need_mask) {
    qk(kb);
    softmax<CAUSAL>(kv0, kv_hi, qw, c_, need_mask);
    pv(vb);
  }

  __device__ __forceinline__ float row_sum(int b) const {
    return lacc[b][0];  // already the full row sum (MFMA over all keys)
  }
  // Epilogue: lane (g, r16) holds d = 16e + 4g + 0..3 of row r16 for every e.
  // One v_permlane16_swap per dword of a d-block pair (e, e+1) exchanges the
  // odd 16-lane rows of block e with the even rows of block e+1, leaving each
  // lane 8 contiguous d of one row: g0 -> 16e+0..7, g1 -> 16(e+1)+0..7,
  // g2 -> 16e+8..15, g3 -> 16(e+1)+8..15.  Half the store instructions
  // (dwordx4 instead of dwordx2) at the same bytes; the store tail is
  // issue-bound (guide T21).
  // row blocks [B0, B1), d-block pairs [EP0, EP1) (symmetric merges store a part each)
  template <int B0 = 0, int B1 = QB, int EP0 = 0, int EP1 = NE / 2>
  __device__ __forceinline__ void store_o(__amdgpu_buffer_rsrc_t ro, int qw) {
#pragma unroll
    for (int b = B0; b < B1; ++b) {
      const float lt = row_sum(b);  // already the full row sum (MFMA over all keys)
      const float inv = lt > 0.f ? 1.0f / lt : 0.f;
      const int rowb = (qw + 16 * b + r16) * ROW;
      const int dlane = 16 * (g & 1) + 8 * (g >> 1);
#pragma unroll
      for (int ep = EP0; ep < EP1; ++ep) {
        tx4 wx, wy;
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          wx[x] = (T)(acc[b][2 * ep][x] * inv);
          wy[x] = (T)(acc[b][2 * ep + 1][x] * inv);
        }
        u32x2 X = __builtin_bit_cast(u32x2, wx), Y = __builtin_bit_cast(u32x2, wy);
#pragma unroll
        for (int dw = 0; dw < 2; ++dw) {
          const auto r = __builtin_amdgcn_permlane16_swap(X[dw], Y[dw], false, false);
          X[dw] = r[0];
          Y[dw] = r[1];
        }
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{X[0], X[1], Y[0], Y[1]}, ro,
                                               rowb + 2 * (32 * ep + dlane), 0, kOStoreAux);
      }
    }
  }
  // a*wa + b*wb with the contraction fixed (fma(a, wa, b*wb)): left to the
  // compiler, which product it fuses depends on which operand arrives from
  // LDS, so two merge paths of the same arithmetic could round differently
  static __device__ __forceinline__ float mix(float a, float wa, float b, float wb) {
    return __builtin_fmaf(a, wa, b * wb);
  }
  static __device__ __forceinline__ f32x4 mix(f32x4 a, float wa, f32x4 b, float wb) {
    return f32x4{mix(a[0], wa, b[0], wb), mix(a[1], wa, b[1], wb), mix(a[2], wa, b[2], wb),
                 mix(a[3], wa, b[3], wb)};
  }
  // KV-pair merge (attention_kvpair), symmetric: group A finalizes row block
  // 0 and parks block 1, group B the reverse (both waves of a SIMD hold the
  // same query rows in the same lanes).  Region per parked block: NE f32x4 of
  // O, then one float2 {m, l} per lane.  Both groups combine with group A's
  // term first:  O = O_a 2^(m_a-M) + O_b 2^(m_b-M), l likewise, M = max over
  // the partials that saw a key.
  static constexpr int HALF_MERGE_BYTES = NE * 64 * 16 + 64 * 8;
  template <int b>
  __device__ __forceinline__ void put_block(char* region) const {
    f32x4* d = reinterpret_cast<f32x4*>(region);
#pragma unroll
    for (int e = 0; e < NE; ++e) d[e * 64 + lane] = acc[b][e];
    reinterpret_cast<float2*>(region + NE * 64 * 16)[lane] = make_float2(m_ref[b], row_sum(b));
  }
  template <int b, bool OWN_IS_A>
  __device__ __forceinline__ void merge_block(const char* region) {
    const f32x4* d = reinterpret_cast<const f32x4*>(region);
    const float2 ml = reinterpret_cast<const float2*>(region + NE * 64 * 16)[lane];
    const float l_own = row_sum(b);
    const float la = OWN_IS_A ? l_own : ml.y, lb = OWN_IS_A ? ml.y : l_own;
    const float ma = la > 0.f ? (OWN_IS_A ? m_ref[b] : ml.x) : ninf();
    const float mb = lb > 0.f ? (OWN_IS_A ? ml.x : m_ref[b]) : ninf();
    float M = fmaxf(ma, mb);
    M = M == ninf() ? 0.f : M;
    const float wa = __builtin_amdgcn_exp2f(ma - M), wb = __builtin_amdgcn_exp2f(mb - M);
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const f32x4 oa = OWN_IS_A ? acc[b][e] : d[e * 64 + lane];
      const f32x4 ob = OWN_IS_A ? d[e * 64 + lane] : acc[b][e];
      acc[b][e] = mix(oa, wa, ob, wb);
    }
    const float l = mix(la, wa, lb, wb);
    lacc[b] = f32x4{l, l, l, l};
    m_ref[b] = M;
  }
  // Symmetric KV-quad merge: the four partials of a row set each finalize
  // one quarter -- partial P takes row block P & 1 and d-half P >> 1 -- and
  // park the three quarters the others finalize (slot (Q - P + 3) & 3 of
  // their region) plus {m_0, l_0, m_1, l_1}.  Each finalizer replays the
  // sequential merge of a single finalizer (partial 0, then 1, 2, 3; the
  // accumulated state is always the A side), so all four agree bit for bit
  // with that order.
  static constexpr int QE = NE / 2;  // d-blocks per quarter
  static constexpr int QUARTER_BYTES = QE * 64 * 16;
  static constexpr int QUAD_MERGE_BYTES = 3 * QUARTER_BYTES + 64 * 16;
  __device__ __forceinline__ void put_quarters(char* region, int P) const {
#pragma unroll
    for (int Q = 0; Q < 4; ++Q) {
      if (Q == P) continue;
      f32x4* d = reinterpret_cast<f32x4*>(region + ((Q - P + 3) & 3) * QUARTER_BYTES);
#pragma unroll
      for (int e = 0; e < QE; ++e) d[e * 64 + lane] = acc[Q & 1][(Q >> 1) * QE + e];
    }
    reinterpret_cast<f32x4*>(region + 3 * QUARTER_BYTES)[lane] =
        f32x4{m_ref[0], row_sum(0), m_ref[1], row_sum(1)};
  }
  // regions: partial j's region at regions + j * stride
  template <int P>
  __device__ __forceinline__ void merge_quarter(const char* regions, int stride) {
    constexpr int b = P & 1, e0 = (P >> 1) * QE;
    auto part = [&](int j) { return regions + j * stride; };
    auto slot = [&](int j) {  // partial j's copy of quarter P
      return reinterpret_cast<const f32x4*>(part(j) + ((P - j + 3) & 3) * QUARTER_BYTES);
    };
    auto ml_of = [&](int j) { return reinterpret_cast<const f32x4*>(part(j) + 3 * QUARTER_BYTES)[lane]; };
    f32x4 o[QE];
    float m, l;
    if constexpr (P == 0) {
#pragma unroll
      for (int e = 0; e < QE; ++e) o[e] = acc[b][e0 + e];
      m = m_ref[b];
      l = row_sum(b);
    } else {
      const f32x4 ml = ml_of(0);
#pragma unroll
      for (int e = 0; e < QE; ++e) o[e] = slot(0)[e * 64 + lane];
      m = ml[2 * b];
      l = ml[2 * b + 1];
    }
#pragma unroll
    for (int j = 1; j < 4; ++j) {
      float mj, lj;
      f32x4 oj[QE];
      if (j == P) {
#pragma unroll
        for (int e = 0; e < QE; ++e) oj[e] = acc[b][e0 + e];
        mj = m_ref[b];
        lj = row_sum(b);
      } else {
        const f32x4 ml = ml_of(j);
#pragma unroll
        for (int e = 0; e < QE; ++e) oj[e] = slot(j)[e * 64 + lane];
        mj = ml[2 * b];
        lj = ml[2 * b + 1];
      }
      const float ma = l > 0.f ? m : ninf();
      const float mb = lj > 0.f ? mj : ninf();
      float M = fmaxf(ma, mb);
      M = M == ninf() ? 0.f : M;
      const float wa = __builtin_amdgcn_exp2f(ma - M), wb = __builtin_amdgcn_exp2f(mb - M);
#pragma unroll
      for (int e = 0; e < QE; ++e) o[e] = mix(o[e], wa, oj[e], wb);
      l = mix(l, wa, lj, wb);
      m = M;
    }
#pragma unroll
    for (int e = 0; e < QE; ++e) acc[b][e0 + e] = o[e];
    lacc[b] = f32x4{l, l, l, l};
    m_ref[b] = m;
  }
  // m in the reference's units (scaled score, natural log): m_ref * ln 2
  __device__ __forceinline__ void store_partial(__amdgpu_buffer_rsrc_t rpo, float* pml, int qw,
                                                int S, float /*scale*/) {
#pragma unroll
    for (int b = 0; b < QB; ++b) {
      const float lt = row_sum(b);
      const int q = qw + 16 * b + r16;
#pragma unroll
      for (int e = 0; e < NE; ++e) buf_store16f(rpo, q * HDIM * 4 + 4 * (16 * e + 4 * g), acc[b][e]);
      if (g == 0 && q < S)
        *reinterpret_cast<float2*>(pml + (size_t)q * 2) =
            make_float2(lt > 0.f ? m_ref[b] * 0.6931471805599453f : ninf(), lt);
    }
  }
};

// ---------------------------------------------------------------------------
// The tile loop (shared skeleton)
//   Pol    : M16<BN, T, HDIM>
//   WAVES  : 64-lane waves per workgroup (BM = 32*WAVES query rows)
//   CAUSAL : top-left aligned causal mask (key j visible to query i iff j <= i)
//   SPLIT  : write unnormalised fp32 O + (m, l) instead of fp16 O
// ---------------------------------------------------------------------------
template <class Pol, int WAVES, bool CAUSAL, bool SPLIT>
__device__ __forceinline__ void attention_tile_loop(const FwdParams& p, int bh, int qb, int split,
                                                    char* smem) {
  constexpr int BN = Pol::BN;
  constexpr int NT = WAVES * 64;
  constexpr int RW = Pol::RW;              // query rows per wave (32)
  constexpr int BM = WAVES * RW;
  constexpr int HD = Pol::HDIM;            // shadows the head_dim-128 defaults
  constexpr int ROW_BYTES = 2 * HD;        // HBM row
  constexpr int TILE_BYTES = BN * 256;     // LDS image: 256-B row slots at any head_dim
  constexpr int NCH = (BN * (HD / 8)) / NT;  // 16-B chunks per thread per tile (K and V each)
  static_assert((BN * (HD / 8)) % NT == 0, "tile chunks must divide evenly");

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int S = p.seq_len;

  const size_t head_off = (size_t)bh * (size_t)S * HD;
  const f16* Qh = p.q + head_off;
  const f16* Kh = p.k + head_off;
  const f16* Vh = p.v + head_off;

  const int q0 = qb * BM;
  const int qw = q0 + wave * RW;  // first query row of this wave

  int kv_lo = 0, kv_hi = CAUSAL ? min(q0 + BM, S) : S;
  if constexpr (SPLIT) {
    const int ntot = (kv_hi + BN - 1) / BN;
    const int per = (ntot + p.num_splits - 1) / p.num_splits;
    kv_lo = min(split * per, ntot) * BN;
    kv_hi = min(kv_hi, min((split + 1) * per, ntot) * BN);
  }
  const int ntiles = kv_hi > kv_lo ? (kv_hi - kv_lo + BN - 1) / BN : 0;

  Pol pol;
  pol.init(lane, p.c);
  pol.issue_q(make_rsrc(Qh, S * ROW_BYTES), qw);  // scaled once tile 0's loads are in flight

  // staging offsets (compile-time slot i adds 4*WAVES rows)
  const int kr0 = pol.k_stage_row(wave), kc = pol.k_stage_ch();
  const int vr0 = pol.v_stage_row(wave), vc = pol.v_stage_ch();
  f16x8 kst[NCH], vst[NCH];
  // loads of the tile starting at key kv_base; rows at/after kv_hi read as 0
  auto issue_loads = [&](int kv_base) {
    const int bytes = (kv_hi - kv_base) * ROW_BYTES;
    const auto rk = make_rsrc(Kh + (size_t)kv_base * HD, bytes);
    const auto rv = make_rsrc(Vh + (size_t)kv_base * HD, bytes);
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      kst[i] = buf_load16(rk, (kr0 + Pol::RPW * WAVES * i) * ROW_BYTES + kc * 16);
      vst[i] = buf_load16(rv, (vr0 + Pol::RPW * WAVES * i) * ROW_BYTES + vc * 16);
    }
  };
  auto write_lds = [&](char* kb) {
    char* vb = kb + TILE_BYTES;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      *reinterpret_cast<f16x8*>(kb + Pol::k_lds(kr0 + Pol::RPW * WAVES * i, kc)) = kst[i];
      *reinterpret_cast<f16x8*>(vb + Pol::v_lds(vr0 + Pol::RPW * WAVES * i, vc)) = vst[i];
    }
  };

  // prologue: unconditional, so every earlier load (Q included) has retired
  // before the loop and no in-loop MFMA waits on the prefetch
  issue_loads(kv_lo);
  // every prologue load is issued before the first VALU that waits on one
  // (else the scheduler hoists Q's scaling above the K/V loads: two serial
  // memory latencies per item)
  __builtin_amdgcn_sched_barrier(0);
  pol.scale_q();
  write_lds(smem);
  // vmcnt(0): the compiler may order the Q loads after the K/V loads; without
  // this, its waitcnt analysis keeps Q "pending" at the loop header and every
  // iteration's first MFMAs wait for the in-flight prefetch (vmcnt(N) in QK^T)
  __builtin_amdgcn_s_waitcnt(0x0F70);
  __syncthreads();

  const float c = p.c;
#ifdef FA_STAMPS
  // diagnostic build: [0] tile body, [1] staged-load wait + LDS writes,
  // [2] barrier, [3] load issue; [6] tiles, [7] prologue (per item)
  unsigned long long st_acc[12] = {}, sa, sb, sc, sd, se;
  st_acc[9] = 1;
#define FA_TSTAMP(v)                                                          \
  do {                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                        \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                                        \
  } while (0)
#else
#define FA_TSTAMP(v) \
  do {               \
  } while (0)
#endif
  auto step = [&](int j, auto buf_c) {
    constexpr int BUF = decltype(buf_c)::value;
    char* kb = smem + BUF * 2 * TILE_BYTES;
    char* kb_next = smem + (BUF ^ 1) * 2 * TILE_BYTES;
    const int kv0 = kv_lo + j * BN;
    FA_TSTAMP(sa);
    issue_loads(kv0 + BN);  // past kv_hi: zero bytes, no memory traffic
    FA_TSTAMP(sb);
    // wave-uniform: does any key of this tile lie at/below some row of this wave?
    if (!CAUSAL || kv0 <= qw + RW - 1) {
      const bool need_mask = (kv0 + BN > kv_hi) || (CAUSAL && kv0 + BN - 1 > qw);
      pol.template tile<CAUSAL>(kb, kb + TILE_BYTES, kv0, kv_hi, qw, c, need_mask);
    }
    FA_TSTAMP(sc);
    write_lds(kb_next);
    FA_TSTAMP(sd);
    __syncthreads();
    FA_TSTAMP(se);
#ifdef FA_STAMPS
    st_acc[0] += sc - sb;
    st_acc[1] += sd - sc;
    st_acc[2] += se - sd;
    st_acc[3] += sb - sa;
    st_acc[6] += 1;
#endif
  };
  int j = 0;
  for (; j + 1 < ntiles; j += 2) {
    step(j, std::integral_constant<int, 0>{});
    step(j + 1, std::integral_constant<int, 1>{});
  }
  if (j < ntiles) step(j, std::integral_constant<int, 0>{});
#ifdef FA_STAMPS
  if (lane == 0 && blockIdx.x < 64)
    for (int i = 0; i < 12; ++i) g_fa_stamps[blockIdx.x][wave][i] += st_acc[i];  // this wave's own slot
#endif
#undef FA_TSTAMP

  if constexpr (!SPLIT) {
    pol.store_o(make_rsrc(p.o + head_off, S * ROW_BYTES), qw);
  } else {
    const size_t prow0 = ((size_t)split * p.bh + bh) * (size_t)S;
    pol.store_partial(make_rsrc(p.part_o + prow0 * HD, S * HD * 4), p.part_ml + prow0 * 2, qw, S,
                      p.scale);
  }
}


// ---------------------------------------------------------------------------
// Ping-pong skeleton (8 waves): group A = waves 0-3, group B = waves 4-7;
// wave w and w+4 share a SIMD.  Every wave runs the phase sequence
//   MFMA_0, SM_0, MFMA_1, SM_1, ..., SM_{n-1}, MFMA_n
//   MFMA_k = qk(K_k) [k < n] + pv(V_{k-1}) [k >= 1]   (matrix pipe only)
//   SM_k   = softmax(S_k)                              (VALU/transcendental)
// Group A runs phase p in half-step p, group B in half-step p+1, and every
// half-step ends at a workgroup barrier -- so on each SIMD one wave's MFMA
// block always runs beside its partner's softmax (matrix || VALU), instead of
// both waves hitting the same phase at once.
// LDS: K and V double-buffered.  Tile k = (K_{k+1}, V_k) is loaded by group A
// during MFMA_k and written during SM_k (half-steps 2k, 2k+1); group B loads
// it one half-step earlier and writes it in half-step 2k.  K_{k+1}/V_k are
// first read in half-step 2k+2 and their buffers were last read in half-step
// 2k-1, so two buffers suffice.
// ---------------------------------------------------------------------------
// DMA: K/V tiles go global -> LDS by LDS-DMA into three rotating buffers
// (a tile's buffer must be free when its loads are issued, one half-step
// before the register path would write it), no staging registers.
// Priority: the MFMA-phase wave runs at s_setprio 1 (every phase).  No
// priority, the static young-half form (guide T5) and priority to the softmax
// phase were each 1-6 % slower (profiles/r01_ab_priority_modes.jsonl,
// r02_ab_priority_modes_d64.jsonl).
template <class Pol, bool CAUSAL, bool SPLIT, bool PRIO = true, bool DMA = false>
__device__ __forceinline__ void attention_pingpong(const FwdParams& p, int bh, int qb, int split,
                                                   char* smem) {
  constexpr int WAVES = 8;
  constexpr int BN = Pol::BN;
  constexpr int NT = WAVES * 64;
  constexpr int BM = WAVES * 32;
  constexpr int HD = Pol::HDIM;            // shadows the head_dim-128 defaults
  constexpr int ROW_BYTES = 2 * HD;        // HBM row
  constexpr int TILE_BYTES = BN * 256;     // LDS image: 256-B row slots at any head_dim
  constexpr int NCH = (BN * (HD / 8)) / NT;
  static_assert((BN * (HD / 8)) % NT == 0, "tile chunks must divide evenly");

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2;  // 0 = A, 1 = B (wave-uniform)
  const int S = p.seq_len;

  const size_t head_off = (size_t)bh * (size_t)S * HD;
  const f16* Qh = p.q + head_off;
  const f16* Kh = p.k + head_off;
  const f16* Vh = p.v + head_off;

  const int q0 = qb * BM;
  const int qw = q0 + wave * 32;

  int kv_lo = 0, kv_hi = CAUSAL ? min(q0 + BM, S) : S;
  if constexpr (SPLIT) {
    const int ntot = (kv_hi + BN - 1) / BN;
    const int per = (ntot + p.num_splits - 1) / p.num_splits;
    kv_lo = min(split * per, ntot) * BN;
    kv_hi = min(kv_hi, min((split + 1) * per, ntot) * BN);
  }
  const int n = kv_hi > kv_lo ? (kv_hi - kv_lo + BN - 1) / BN : 0;
  // where the next tile's global loads are issued: at the start of the MFMA
  // phase (causal), or at the end of the softmax phase, by the wave whose
  // phase is the shorter one (non-causal: +2 % at S=8192; causal: -5 %, its
  // masked/inactive tiles shorten the MFMA phases instead)
  constexpr bool kIssueInSm =
      DMA || (!CAUSAL && (Pol::HDIM == 128 || kNcD64IssueInSm));  // DMA: three buffers
  // where a tile is written to LDS: at the start of the softmax phase (beside
  // the partner's MFMAs; causal: +0.3-0.7 % A/B) or at its end (non-causal:
  // early was -0.8 %, its loads are issued in the softmax phase and need it
  // to land)
  constexpr bool kWriteEarly = !DMA && (CAUSAL || (Pol::HDIM == 64 && kNcD64WriteEarly));
  static_assert(!DMA || Pol::HDIM == 128, "LDS-DMA path: head_dim 128");

#ifdef FA_STAMPS
  const unsigned long long t_in = __builtin_amdgcn_s_memtime();
#endif
  Pol pol;
  pol.init(lane, p.c);
  pol.issue_q(make_rsrc(Qh, S * ROW_BYTES), qw);  // scaled once K_0 / tile 0 are in flight

  constexpr int NBUF = DMA ? 3 : 2;  // tile buffers per tensor
  char* kbuf0 = smem;
  char* vbuf0 = smem + NBUF * TILE_BYTES;
  auto kbuf = [&](int x) { return kbuf0 + (DMA ? x % 3 : x & 1) * TILE_BYTES; };
  auto vbuf = [&](int x) { return vbuf0 + (DMA ? (x + 3) % 3 : x & 1) * TILE_BYTES; };
  // LDS-DMA: this wave's 1-KB pieces of a tile image (pieces wave, wave + 8, ...)
  int k_src[NCH], v_src[NCH];
  if constexpr (DMA) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      k_src[i] = Pol::k_src(1024 * (wave + WAVES * i) + 16 * lane);
      v_src[i] = Pol::v_src(1024 * (wave + WAVES * i) + 16 * lane);
    }
  }
  const int kr0 = pol.k_stage_row(wave), kc = pol.k_stage_ch();
  const int vr0 = pol.v_stage_row(wave), vc = pol.v_stage_ch();
  f16x8 kst[NCH], vst[NCH];
  // tile k = (K_{k+1}, V_k); rows at/after kv_hi (or k >= n) read as 0
  auto issue_tile = [&](int k) {
    const int kb_row = kv_lo + (k + 1) * BN, vb_row = kv_lo + k * BN;
    const auto rk = make_rsrc(Kh + (size_t)kb_row * HD, (kv_hi - kb_row) * ROW_BYTES);
    const auto rv = make_rsrc(Vh + (size_t)vb_row * HD, (kv_hi - vb_row) * ROW_BYTES);
    if constexpr (DMA) {
      char* kb = kbuf(k + 1);
      char* vb = vbuf(k);
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        buf_load16_lds(rk, kb + 1024 * (wave + WAVES * i), k_src[i]);
        buf_load16_lds(rv, vb + 1024 * (wave + WAVES * i), v_src[i]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        kst[i] = buf_load16(rk, (kr0 + Pol::RPW * WAVES * i) * ROW_BYTES + kc * 16);
        vst[i] = buf_load16(rv, (vr0 + Pol::RPW * WAVES * i) * ROW_BYTES + vc * 16);
      }
    }
  };
  auto write_tile = [&](int k) {
    if constexpr (DMA) {
      __builtin_amdgcn_s_waitcnt(0x0F70);  // this wave's pieces of tile k have landed
    } else {
      char* kb = kbuf(k + 1);
      char* vb = vbuf(k);
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        *reinterpret_cast<f16x8*>(kb + Pol::k_lds(kr0 + Pol::RPW * WAVES * i, kc)) = kst[i];
        *reinterpret_cast<f16x8*>(vb + Pol::v_lds(vr0 + Pol::RPW * WAVES * i, vc)) = vst[i];
      }
    }
  };

  // prologue: Q, K_0 (everyone) and tile 0 (group B, written in half-step 0)
  // are all in flight together, so the item start pays one memory latency
  {
    const auto rk = make_rsrc(Kh + (size_t)kv_lo * HD, (kv_hi - kv_lo) * ROW_BYTES);
    f16x8 k0[NCH];
#pragma unroll
    for (int i = 0; i < NCH; ++i)
      k0[i] = buf_load16(rk, (kr0 + Pol::RPW * WAVES * i) * ROW_BYTES + kc * 16);
    if ((kIssueInSm || grp == 1) && n > 0) issue_tile(0);
    __builtin_amdgcn_sched_barrier(0);  // all prologue loads issued first (attention_tile_loop)
    pol.scale_q();
#pragma unroll
    for (int i = 0; i < NCH; ++i)
      *reinterpret_cast<f16x8*>(kbuf0 + Pol::k_lds(kr0 + Pol::RPW * WAVES * i, kc)) = k0[i];
  }
  // Q and K_0 retired before the loop (see attention_tile_loop); group B's
  // tile-0 loads may stay in flight (they are the 2*NCH most recent)
  if (kIssueInSm || grp == 1)
    __builtin_amdgcn_s_waitcnt(0x0F70 | (2 * NCH));
  else
    __builtin_amdgcn_s_waitcnt(0x0F70);
  __syncthreads();

  const float c = p.c;
  auto active = [&](int k) { return !CAUSAL || (kv_lo + k * BN <= qw + 31); };
  auto mfma_block = [&](int k) {
    // the MFMA-phase wave wins VALU/MFMA issue arbitration against its SIMD
    // partner (which is in its softmax phase), so its matrix stream stays dense
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
    pol.mfma_block(kbuf(k), vbuf(k - 1), k >= 1 && active(k - 1), k < n && active(k));
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  };
  auto softmax_block = [&](int k) {
    if (k < n && active(k)) {
      const int kv0 = kv_lo + k * BN;
      const bool need_mask = (kv0 + BN > kv_hi) || (CAUSAL && kv0 + BN - 1 > qw);
      pol.template softmax<CAUSAL>(kv0, kv_hi, qw, c, need_mask);
    }
  };

  // Every wave runs the same loop [MFMA_k] barrier [SM_k] barrier; group B
  // executes one extra barrier first (while A runs MFMA_0) and A one extra at
  // the end, so B trails A by exactly one half-step with no group-specific
  // code path.  Tile t = k + grp is loaded during MFMA_k and written during SM_k.
  if (grp == 1) {
    if (n > 0) write_tile(0);
    if (kIssueInSm && 1 < n) issue_tile(1);
    __syncthreads();
  }
#ifdef FA_STAMPS
  unsigned long long st_acc[11] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0}, st0, st01, st1, st2, st3, st4;
  st_acc[7] = __builtin_amdgcn_s_memtime() - t_in;
#define FA_STAMP(v)                                                                   \
  do {                                                                                \
    __builtin_amdgcn_sched_barrier(0);                                                \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");         \
    __builtin_amdgcn_sched_barrier(0);                                                \
  } while (0)
#else
#define FA_STAMP(v) \
  do {              \
  } while (0)
#endif
  // The last MFMA phase (k = n: the PV of tile n-1 alone) is peeled so each
  // group's O leaves right after it -- group A's a half-step before group
  // B's, so B's stores no longer queue behind A's (round-1 stamps: group B
  // epilogue 6.2k cycles vs A 2.2k per item); the barriers after it only
  // keep the LDS hand-off order for the next item.  Causal only: +1-3 % on
  // the causal persistent shapes, while the non-causal build took more SGPR
  // spills (35 -> 42) and was level to 4 % slower
  // (profiles/r02_ab_early_o_store.jsonl).  Non-causal d128: both groups
  // store after the final barrier.
  constexpr bool kEarlyStore = CAUSAL || (Pol::HDIM == 64 && kNcD64EarlyStore);
  auto store_out = [&]() {
    if constexpr (!SPLIT) {
      pol.store_o(make_rsrc(p.o + head_off, S * ROW_BYTES), qw);
    } else {
      const size_t prow0 = ((size_t)split * p.bh + bh) * (size_t)S;
      pol.store_partial(make_rsrc(p.part_o + prow0 * HD, S * HD * 4), p.part_ml + prow0 * 2, qw, S,
                        p.scale);
    }
  };
  for (int k = 0; k < (kEarlyStore ? n : n + 1); ++k) {
    const int t = k + grp;
    FA_STAMP(st0);
    if (!kIssueInSm && t < n) issue_tile(t);
#ifdef FA_STAMPS
    FA_STAMP(st01);
#endif
    mfma_block(k);
    FA_STAMP(st1);
    __syncthreads();
    FA_STAMP(st2);
    if constexpr (kWriteEarly) {
      if (t < n) write_tile(t);
      if (kIssueInSm && t + 1 < n) issue_tile(t + 1);
    }
    softmax_block(k);
#ifdef FA_STAMPS
    unsigned long long st25;
    FA_STAMP(st25);
#endif
#ifdef FA_STAMPS
    unsigned long long st_w;
    __builtin_amdgcn_s_waitcnt(0x0F70);  // diagnostic: split the load wait from the LDS writes
    FA_STAMP(st_w);
    st_acc[10] += st_w - st25;
#endif
    if constexpr (!kWriteEarly) {
      if (t < n) write_tile(t);
      if (kIssueInSm && t + 1 < n) issue_tile(t + 1);
    }
    FA_STAMP(st3);
    __syncthreads();
    FA_STAMP(st4);
#ifdef FA_STAMPS
    st_acc[0] += st1 - st01;
    st_acc[1] += st2 - st1;
    st_acc[2] += st25 - st2;
    st_acc[3] += st4 - st3;
    st_acc[4] += st3 - st25;
    st_acc[5] += st01 - st0;
    st_acc[6] += 1;
#endif
  }
  if constexpr (kEarlyStore) {
    mfma_block(n);  // PV of tile n-1 (no tile n: the softmax half-step is empty)
    store_out();
    __syncthreads();
    __syncthreads();
  }
  if (grp == 0) __syncthreads();
#ifdef FA_STAMPS
  const unsigned long long t_le = __builtin_amdgcn_s_memtime();
#endif

  if constexpr (!kEarlyStore) store_out();
#ifdef FA_STAMPS
  __builtin_amdgcn_s_waitcnt(0);  // stores issued and retired
  st_acc[8] = __builtin_amdgcn_s_memtime() - t_le;
  if (lane == 0 && blockIdx.x < 64)
    for (int i = 0; i < 11; ++i) g_fa_stamps[blockIdx.x][wave][i] += st_acc[i];  // this wave's own slot
#endif
#undef FA_STAMP
}

// ---------------------------------------------------------------------------
// KV-pair skeleton (8 waves, 128 query rows): short sequences.
// The two waves of a SIMD hold the SAME 32 query rows and split the key range
// between them -- wave w (group A) takes key tiles 0, 2, 4, ..., wave w+4
// (group B) tiles 1, 3, 5, ... -- and merge (O, m, l) through LDS at the end.
// Half the query rows per workgroup of the 256-row ping-pong, so twice the
// workgroups on a short launch (S=1024, B=1, H=32: 256 instead of 128, one
// per CU), and the heaviest causal block's key loop is halved.
//
// Every wave runs the ping-pong phase pair [MFMA] barrier [softmax] barrier,
// group B one half-step behind group A.  On the shared half-step clock h:
//   MFMA phase at h (group h & 1): QK^T of tile h, PV of tile h-2
//   softmax phase at h:            tile h-1 (the other group's QK^T of h-1)
// so K_t is read only at half-step t and V_t only at t+2: at the end of
// half-step h every wave writes its staged share of stage h = (K_{h+1},
// V_{h-1}) (one tile of each per half-step, two LDS buffers per tensor) and
// issues the loads of stage h+2, two half-steps ahead (two staging sets: one
// for the wave's MFMA half-steps, one for its softmax half-steps).
// Measured and not kept: only the softmax-phase group staging each tile, at
// the start of its phase (-1.5 %, the softmax side is already the long pole);
// one staging set, loads one half-step ahead (equal).
// ---------------------------------------------------------------------------
//
// KV-quad (SUB = 2): 64 query rows per workgroup, four waves per 32 rows.  A
// half-step stage is a 128-key super-tile (two 64-key images back to back);
// in its MFMA half-step a group's waves 0-1 take the first image and waves
// 2-3 the second, so wave w sees key tiles 2h + ((w & 3) >> 1) of the
// half-steps h of its group: a four-way key split merged through LDS.  Twice
// the workgroups of the KV-pair and half its per-wave key loop, for launches
// that leave CUs idle even at 128 rows (B=1 H=32 S=512: 128 KV-pair
// workgroups on 256 CUs).  One staging set (loads one half-step ahead): two
// sets of the double-width stage would not fit the 256 VGPRs.
// Merges are symmetric: in the KV-pair each group parks one 16-row block and
// finalizes and stores the other, in the KV-quad each of a row set's four
// partials finalizes and stores a quarter, so all eight waves share the merge
// and the O stores (bit-identical to one finalizer; +1-7 %,
// profiles/r02_ab_kvpair_sym_merge.jsonl, r02_ab_merge_contraction.jsonl).
// Q is read once per workgroup and shared through LDS by the row set's
// partial waves (bit-identical; KV-quad +3.5-12.6 %,
// profiles/r02_ab_short_q_share.jsonl).  The MFMA half-step runs at
// s_setprio 1.
template <class Pol, bool CAUSAL, int SUB = 1>
__device__ __forceinline__ void attention_kvpair(const FwdParams& p, int bh, int qb, char* smem) {
  static_assert(SUB == 1 || SUB == 2, "key split 2 (KV-pair) or 4 (KV-quad)");
  constexpr int WAVES = 8;
  constexpr int BN = Pol::BN;
  constexpr int NT = WAVES * 64;
  constexpr int RW = 4 / SUB;       // row waves per group (32 query rows each)
  constexpr int BM = 32 * RW;       // 128 (KV-pair) or 64 (KV-quad)
  constexpr int NP = 2 * SUB;       // partial states per query row (key splits)
  constexpr int SBN = SUB * BN;     // keys per stage
  constexpr int HD = Pol::HDIM;
  constexpr int ROW_BYTES = 2 * HD;
  constexpr int TILE_BYTES = BN * 256;
  constexpr int STAGE_BYTES = SUB * TILE_BYTES;
  constexpr int NCH = (SBN * (HD / 8)) / NT;
  constexpr bool TWO_SETS = SUB == 1;
  constexpr int NSET = TWO_SETS ? 2 : 1;
  static_assert((SBN * (HD / 8)) % NT == 0, "tile chunks must divide evenly");
  static_assert(4 * STAGE_BYTES <= (SUB == 1 ? kKvpairLdsBytes : kKvquadLdsBytes),
                "stage buffers fit the LDS allocation");

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2;          // 0 = A (even half-steps), 1 = B (odd)
  const int rw = wave & (RW - 1);     // row wave: rows q0 + 32 rw ...
  const int sub = (wave & 3) / RW;    // image of the stage this wave consumes
  const int pidx = wave / RW;         // partial index; 0 merges and stores
  const int S = p.seq_len;

  const size_t head_off = (size_t)bh * (size_t)S * HD;
  const f16* Qh = p.q + head_off;
  const f16* Kh = p.k + head_off;
  const f16* Vh = p.v + head_off;

  const int q0 = qb * BM;
  const int qw = q0 + rw * 32;
  const int kv_hi = CAUSAL ? min(q0 + BM, S) : S;
  const int nt = (kv_hi + BN - 1) / BN;    // 64-key tiles
  const int n = (kv_hi + SBN - 1) / SBN;   // stages

#ifdef FA_STAMPS
  unsigned long long st_acc[12] = {}, sa, sb;
  const unsigned long long t_in = __builtin_amdgcn_s_memtime();
#define FA_KSTAMP(v)                                                          \
  do {                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                        \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                                        \
  } while (0)
#else
#define FA_KSTAMP(v) \
  do {               \
  } while (0)
#endif

  Pol pol;
  pol.init(lane, p.c);
  // the partials of a row set share one read of its Q through LDS: KV-quad
  // through the stage-0 V buffer (first written after a later barrier),
  // KV-pair past the four tile buffers (its stage-0 V buffer is too small)
  char* qshare = smem + (SUB == 2 ? 2 : 4) * STAGE_BYTES + rw * Pol::Q_SHARE_BYTES;
  static_assert(SUB == 1 || RW * Pol::Q_SHARE_BYTES <= STAGE_BYTES, "Q share fits one V buffer");
  static_assert(SUB == 2 || 4 * STAGE_BYTES + RW * Pol::Q_SHARE_BYTES <= kKvpairLdsBytes,
                "Q share fits past the tile buffers");
  pol.template issue_q_part<NP>(make_rsrc(Qh, S * ROW_BYTES), qw, pidx);

  auto kbuf = [&](int x) { return smem + (x & 1) * STAGE_BYTES; };
  auto vbuf = [&](int x) { return smem + (2 + (x & 1)) * STAGE_BYTES; };
  const int kr0 = pol.k_stage_row(wave), kc = pol.k_stage_ch();
  const int vr0 = pol.v_stage_row(wave), vc = pol.v_stage_ch();
  // two sets: set 0 carries the stages of this wave's MFMA half-steps, set 1
  // those of its softmax half-steps (they alternate); one set: every stage
  f16x8 kst[NSET][NCH], vst[NSET][NCH];
  // loads of stage h = (K_{h+1}, V_{h-1}); rows at/after kv_hi, and tiles
  // outside [0, n), read as 0 with no memory traffic
  auto issue_stage = [&](int h, auto set_c) {
    constexpr int X = decltype(set_c)::value;
    const int kb_row = (h + 1) * SBN, vb_row = (h - 1) * SBN;
    const auto rk = make_rsrc(Kh + (size_t)min(kb_row, S) * HD, (kv_hi - kb_row) * ROW_BYTES);
    const auto rv = make_rsrc(Vh + (size_t)max(vb_row, 0) * HD,
                              vb_row < 0 ? 0 : (kv_hi - vb_row) * ROW_BYTES);
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      // KV-quad: per-pass row offsets in the scalar soffset (with four
      // passes in VGPRs the kernel spilled); KV-pair: in VGPRs (+1-4 % A/B,
      // profiles/r01_ab_kvpair_soffset.jsonl)
      if constexpr (SUB == 1) {
        kst[X][i] = buf_load16(rk, (kr0 + Pol::RPW * WAVES * i) * ROW_BYTES + kc * 16);
        vst[X][i] = buf_load16(rv, (vr0 + Pol::RPW * WAVES * i) * ROW_BYTES + vc * 16);
      } else {
        kst[X][i] = buf_load16s(rk, kr0 * ROW_BYTES + kc * 16, Pol::RPW * WAVES * i * ROW_BYTES);
        vst[X][i] = buf_load16s(rv, vr0 * ROW_BYTES + vc * 16, Pol::RPW * WAVES * i * ROW_BYTES);
      }
    }
  };
  auto write_stage = [&](int h, auto set_c) {
    constexpr int X = decltype(set_c)::value;
    char* kb = kbuf(h + 1);
    char* vb = vbuf(h - 1);
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      *reinterpret_cast<f16x8*>(kb + Pol::k_lds(kr0 + Pol::RPW * WAVES * i, kc)) = kst[X][i];
      *reinterpret_cast<f16x8*>(vb + Pol::v_lds(vr0 + Pol::RPW * WAVES * i, vc)) = vst[X][i];
    }
  };
  using Set0 = std::integral_constant<int, 0>;
  using Set1 = std::integral_constant<int, 1>;

  // prologue: Q, K_0 and the first two stages' loads in flight together
  {
    const auto rk = make_rsrc(Kh, kv_hi * ROW_BYTES);
    f16x8 k0[NCH];
#pragma unroll
    for (int i = 0; i < NCH; ++i)
      k0[i] = buf_load16(rk, (kr0 + Pol::RPW * WAVES * i) * ROW_BYTES + kc * 16);
    // set 0 = this wave's first MFMA half-step (A: h=0, B: h=1), set 1 = its
    // first softmax one (A: h=1, B: the idle h=0); branch-free: a per-group
    // branch makes hipcc merge the paths with register copies that wait for
    // the loads
    if constexpr (TWO_SETS) {
      issue_stage(grp, Set0{});
      issue_stage(1 - grp, Set1{});
    } else {
      issue_stage(0, Set0{});
    }
    __builtin_amdgcn_sched_barrier(0);  // all prologue loads issued first (attention_tile_loop)
    pol.template scale_put_q_part<NP>(qshare, pidx);
#pragma unroll
    for (int i = 0; i < NCH; ++i)
      *reinterpret_cast<f16x8*>(kbuf(0) + Pol::k_lds(kr0 + Pol::RPW * WAVES * i, kc)) = k0[i];
  }
  // Q and K_0 retired (see attention_tile_loop); the stage loads may stay in flight
  __builtin_amdgcn_s_waitcnt(0x0F70 | (2 * NSET * NCH));
  __syncthreads();
  pol.template get_q_rest<NP>(qshare, pidx);
#ifdef FA_STAMPS
  st_acc[7] = __builtin_amdgcn_s_memtime() - t_in;
#endif

  const float c = p.c;
  // this wave's key tile of stage h is t = SUB h + sub
  auto active = [&](int h) {
    const int t = SUB * h + sub;
    return h >= 0 && t < nt && (!CAUSAL || t * BN <= qw + 31);
  };
  // end of half-step h: publish its stage, refill the staging set, barrier
  auto half_step_end = [&](int h, auto set_c, int bar_slot) {
#ifdef FA_STAMPS
    unsigned long long w0, w1, w2, w3;
    FA_KSTAMP(w0);
    __builtin_amdgcn_s_waitcnt(0x0F70 | (TWO_SETS ? 2 * NCH : 0));
    FA_KSTAMP(w1);
#endif
    using SetX = std::integral_constant<int, TWO_SETS ? decltype(set_c)::value : 0>;
    write_stage(h, SetX{});
    issue_stage(h + NSET, SetX{});
#ifdef FA_STAMPS
    FA_KSTAMP(w2);
#endif
    __syncthreads();
#ifdef FA_STAMPS
    FA_KSTAMP(w3);
    st_acc[10] += w1 - w0;
    st_acc[4] += w2 - w1;
    st_acc[bar_slot] += w3 - w2;
#endif
    (void)bar_slot;
  };
  // pairs of half-steps per wave: covers h = 0 .. n+1 (the last PV is at n+1)
  const int P = (n + 3) >> 1;
  if (grp == 1) half_step_end(0, Set1{}, 3);  // group B: idle leading half-step
  for (int m = 0; m < P; ++m) {
    const int h = 2 * m + grp;
    FA_KSTAMP(sa);
    __builtin_amdgcn_s_setprio(1);
    pol.mfma_block(kbuf(h) + sub * TILE_BYTES, vbuf(h - 2) + sub * TILE_BYTES, active(h - 2),
                   active(h));
    __builtin_amdgcn_s_setprio(0);
    FA_KSTAMP(sb);
#ifdef FA_STAMPS
    st_acc[0] += sb - sa;
#endif
    half_step_end(h, Set0{}, 1);
    FA_KSTAMP(sa);
    if (active(h)) {
      const int kv0 = (SUB * h + sub) * BN;
      const bool need_mask = (kv0 + BN > kv_hi) || (CAUSAL && kv0 + BN - 1 > qw);
      pol.template softmax<CAUSAL>(kv0, kv_hi, qw, c, need_mask);
    }
    FA_KSTAMP(sb);
#ifdef FA_STAMPS
    st_acc[2] += sb - sa;
    st_acc[6] += 1;
#endif
    half_step_end(h + 1, Set1{}, 3);
  }
  if (grp == 0) half_step_end(2 * P, Set0{}, 1);  // group A: idle trailing half-step
  __builtin_amdgcn_s_waitcnt(0x0F70);            // the last (zero-size) stage loads
#ifdef FA_STAMPS
  const unsigned long long t_le = __builtin_amdgcn_s_memtime();
#endif

  // merge (symmetric, see above)
  if constexpr (SUB == 2) {
    // each of a row set's four partials finalizes one quarter
    static_assert(NP * RW * Pol::QUAD_MERGE_BYTES <= kKvquadLdsBytes, "quarter-merge region fits");
    const int stride = RW * Pol::QUAD_MERGE_BYTES;
    char* regions = smem + rw * Pol::QUAD_MERGE_BYTES;  // partial j at regions + j * stride
    pol.put_quarters(regions + pidx * stride, pidx);
    __syncthreads();
    const auto ro = make_rsrc(p.o + head_off, S * ROW_BYTES);
    constexpr int H = Pol::QE / 2;  // d-block pairs per quarter
    if (pidx == 0) {
      pol.template merge_quarter<0>(regions, stride);
      pol.template store_o<0, 1, 0, H>(ro, qw);
    } else if (pidx == 1) {
      pol.template merge_quarter<1>(regions, stride);
      pol.template store_o<1, 2, 0, H>(ro, qw);
    } else if (pidx == 2) {
      pol.template merge_quarter<2>(regions, stride);
      pol.template store_o<0, 1, H, 2 * H>(ro, qw);
    } else {
      pol.template merge_quarter<3>(regions, stride);
      pol.template store_o<1, 2, H, 2 * H>(ro, qw);
    }
  } else {
    // each group parks one row block and finalizes the other
    static_assert(2 * RW * Pol::HALF_MERGE_BYTES <= kKvpairLdsBytes, "half-merge region fits");
    if (grp == 0)
      pol.template put_block<1>(smem + rw * Pol::HALF_MERGE_BYTES);
    else
      pol.template put_block<0>(smem + (RW + rw) * Pol::HALF_MERGE_BYTES);
    __syncthreads();
    const auto ro = make_rsrc(p.o + head_off, S * ROW_BYTES);
    if (grp == 0) {
      pol.template merge_block<0, true>(smem + (RW + rw) * Pol::HALF_MERGE_BYTES);
      pol.template store_o<0, 1>(ro, qw);
    } else {
      pol.template merge_block<1, false>(smem + rw * Pol::HALF_MERGE_BYTES);
      pol.template store_o<1, 2>(ro, qw);
    }
  }
#ifdef FA_STAMPS
  __builtin_amdgcn_s_waitcnt(0);
  st_acc[8] = __builtin_amdgcn_s_memtime() - t_le;  // merge + stores retired
  st_acc[9] = 1;
  if (lane == 0 && blockIdx.x < 64)
    for (int i = 0; i < 12; ++i) g_fa_stamps[blockIdx.x][wave][i] += st_acc[i];  // this wave's own slot
#endif
#undef FA_KSTAMP
}

}  // namespace fa
