// mfma_rate_probe.hip -- measures sustained fp16 MFMA throughput on gfx950 for
// the shapes the attention loop could use (north_star names 16x16x16; gfx950
// also has 16x16x32 and 32x32x16).  One wave per SIMD, 4 independent
// accumulators, random operands, whole chip.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

template <int KIND>
__global__ __launch_bounds__(256) void probe(const float* seed, float* out, int iters) {
  const int l = threadIdx.x;
  h8 a8, b8; h4 a4, b4;
  for (int j = 0; j < 8; ++j) { a8[j] = (_Float16)(seed[(l + j) & 255] - 0.5f); b8[j] = (_Float16)(seed[(l * 3 + j) & 255] - 0.5f); }
  for (int j = 0; j < 4; ++j) { a4[j] = a8[j]; b4[j] = b8[j]; }
  f4 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  f16v d0 = {}, d1 = {}, d2 = {}, d3 = {};
  for (int i = 0; i < iters; ++i) {
    if constexpr (KIND == 0) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, c3, 0, 0, 0);
    } else if constexpr (KIND == 1) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, c3, 0, 0, 0);
    } else if constexpr (KIND == 2) {
      d0 = __builtin_amdgcn_mfma_f32_32x32x8f16(a4, b4, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_32x32x8f16(a4, b4, d1, 0, 0, 0);
      d2 = __builtin_amdgcn_mfma_f32_32x32x8f16(a4, b4, d2, 0, 0, 0);
      d3 = __builtin_amdgcn_mfma_f32_32x32x8f16(a4, b4, d3, 0, 0, 0);
    } else {
      d0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, b8, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, b8, d1, 0, 0, 0);
      d2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, b8, d2, 0, 0, 0);
      d3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, b8, d3, 0, 0, 0);
    }
  }
  float s = 0;
  for (int j = 0; j < 4; ++j) s += c0[j] + c1[j] + c2[j] + c3[j];
  for (int j = 0; j < 16; ++j) s += d0[j] + d1[j] + d2[j] + d3[j];
  out[blockIdx.x * 256 + l] = s;
}

int main() {
  const int blocks = 256 * 4, iters = 20000;
  float *seed, *out;
  hipMalloc(&seed, 256 * 4); hipMalloc(&out, blocks * 256 * 4);
  float h[256]; for (int i = 0; i < 256; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f;
  hipMemcpy(seed, h, sizeof h, hipMemcpyHostToDevice);
  const char* names[4] = {"v_mfma_f32_16x16x16_f16", "v_mfma_f32_16x16x32_f16", "v_mfma_f32_32x32x8_f16", "v_mfma_f32_32x32x16_f16"};
  const double flop_per[4] = {16.*16*16*2, 16.*16*32*2, 32.*32*8*2, 32.*32*16*2};
  void (*k[4])(const float*, float*, int) = {probe<0>, probe<1>, probe<2>, probe<3>};
  for (int kind = 0; kind < 4; ++kind) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
      hipLaunchKernelGGL(k[kind], dim3(blocks), dim3(256), 0, 0, seed, out, iters / 10);
      hipEventRecord(a);
      hipLaunchKernelGGL(k[kind], dim3(blocks), dim3(256), 0, 0, seed, out, iters);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      const double flops = (double)blocks * 4 /*waves*/ * iters * 4 /*mfma*/ * flop_per[kind];
      if (rep) printf("{\"mfma\": \"%s\", \"tflops\": %.1f, \"ms\": %.3f}\n", names[kind], flops / ms / 1e9, ms);
    }
  }
  return 0;
}
