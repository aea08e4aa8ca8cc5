// Compile-only probe of the 4-wave x 64-rows-per-wave (one wave per SIMD)
// skeleton, attention_w4 in csrc/fa_fwd_kernel.hpp (FA_W4_EXPERIMENT), and of
// the plain, un-pipelined 64-row loop beside it.  Not part of the library:
// run tools/experiments/w4_spill_probe.sh and read the register report.
#define FA_W4_EXPERIMENT
#include "fa_fwd_kernel.hpp"
using namespace fa;

// software-pipelined W4 (softmax(j) beside PV(j-1) / QK^T(j+1)); the MFMAs
// are the pinned-register asm of M16<.., QB = 4>
__global__ __launch_bounds__(256, 1) void w4_pipelined_noncausal(FwdParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  attention_w4<M16<64, f16, 128, 4>, false>(p, blockIdx.x >> 5, blockIdx.x & 31, smem);
}

// plain per-tile qk -> softmax -> pv at 64 rows per wave (no pipelining, no
// K/V staging): the loop of configs 46-49
__global__ __launch_bounds__(256, 1) void w4_plain_noncausal(FwdParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int S = p.seq_len;
  const size_t ho = (size_t)(blockIdx.x >> 5) * S * 128;
  const int qw = (blockIdx.x & 31) * 256 + wave * 64;
  M16<64, f16, 128, 4> pol;
  pol.init(lane, p.c);
  pol.load_q(make_rsrc(p.q + ho, S * 256), qw);
  for (int j = 0; j < S / 64; ++j) {
    char* kb = smem + (j & 1) * 32768;
    pol.tile<false>(kb, kb + 16384, j * 64, S, qw, p.c, false);
    __syncthreads();
  }
  pol.store_o(make_rsrc(p.o + ho, S * 256), qw);
}

// the 8-wave ping-pong at BN = 128 (32 rows per wave, two waves per SIMD:
// 256 registers per wave): VERDICT r01 item 3
__global__ __launch_bounds__(512, 2) void pingpong_bn128_causal(FwdParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  attention_pingpong<M16<128, f16, 128, 2>, true, false, true, false>(p, blockIdx.x >> 5,
                                                                      blockIdx.x & 31, 0, smem);
}
__global__ __launch_bounds__(512, 2) void pingpong_bn128_dma_causal(FwdParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  attention_pingpong<M16<128, f16, 128, 2>, true, false, true, true>(p, blockIdx.x >> 5,
                                                                     blockIdx.x & 31, 0, smem);
}
