// launch_probe.hip -- fixed per-launch costs on the box (diagnostic executable).
// What a short-sequence attention launch cannot go below:
//   empty      : back-to-back launches of an empty kernel (grid G x 256/512 threads)
//   rw         : each workgroup loads `kb` KB of fresh HBM data per wave and stores it back
//                (the attention prologue + epilogue with no key loop)
// usage: launch_probe   (prints one JSON line per case)
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 1023) p[0] = 1;  // never true: keeps the kernel non-trivial
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// each thread loads `per` 16-B chunks (strided by the grid) and stores them to `out`
__global__ __launch_bounds__(512) void rw_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out,
                                                 int per) {
  const size_t nthr = (size_t)gridDim.x * blockDim.x;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  u32x4 acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (i < per) acc[i] = in[t + i * nthr];
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (i < per) out[t + i * nthr] = acc[i];
}

static float time_ms(hipStream_t s, int iters, void (*fn)(hipStream_t, void*), void* arg) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 20; ++i) fn(s, arg);
  CK(hipStreamSynchronize(s));
  CK(hipEventRecord(a, s));
  for (int i = 0; i < iters; ++i) fn(s, arg);
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms / iters;
}

struct EmptyArg {
  int grid, threads;
};
static void run_empty(hipStream_t s, void* v) {
  EmptyArg* a = (EmptyArg*)v;
  hipLaunchKernelGGL(empty_kernel, dim3(a->grid), dim3(a->threads), 0, s, (int*)nullptr);
}

struct RwArg {
  const u32x4* in;
  u32x4* out;
  int grid, threads, per;
  size_t stride;  // elements between launches' regions (rotates through a large buffer)
  int rot, nrot;
};
static void run_rw(hipStream_t s, void* v) {
  RwArg* a = (RwArg*)v;
  const size_t off = (size_t)a->rot * a->stride;
  a->rot = (a->rot + 1) % a->nrot;
  hipLaunchKernelGGL(rw_kernel, dim3(a->grid), dim3(a->threads), 0, s, a->in + off, a->out + off,
                     a->per);
}

int main() {
  hipStream_t s;
  CK(hipStreamCreate(&s));
  for (int grid : {1, 256, 512, 2048})
    for (int thr : {256, 512}) {
      EmptyArg a{grid, thr};
      const float ms = time_ms(s, 2000, run_empty, &a);
      printf("{\"case\": \"empty\", \"grid\": %d, \"threads\": %d, \"us_per_launch\": %.3f}\n", grid,
             thr, ms * 1e3);
    }
  // rw: 256 workgroups x 512 threads x per x 16 B (per = 8 -> 16 MB = B=1 H=32 S=1024 Q-sized
  // read + O-sized write); rotate over 1 GB so every launch reads cold HBM
  const size_t total = (size_t)1 << 30;
  u32x4 *in, *out;
  CK(hipMalloc(&in, total));
  CK(hipMalloc(&out, total));
  CK(hipMemset(in, 0, total));
  for (int grid : {256, 512})
    for (int per : {1, 4, 8, 16}) {
      const size_t elems = (size_t)grid * 512 * per;
      RwArg a{in, out, grid, 512, per, elems, 0, (int)(total / 16 / elems)};
      const float ms = time_ms(s, 500, run_rw, &a);
      printf("{\"case\": \"rw\", \"grid\": %d, \"threads\": 512, \"bytes_each_way\": %zu, "
             "\"us_per_launch\": %.3f}\n",
             grid, elems * 16, ms * 1e3);
    }
  // graph of 100 empty launches
  {
    hipGraph_t g;
    hipGraphExec_t ge;
    EmptyArg a{256, 512};
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < 100; ++i) run_empty(s, &a);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < 10; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"case\": \"graph_empty\", \"grid\": 256, \"threads\": 512, \"us_per_launch\": %.3f}\n",
           ms * 1e3 / 1000);
  }
  CK(hipFree(in));
  CK(hipFree(out));
  return 0;
}
