// flash_attention_v9.cpp -- the reference's C++ dispatcher signature
// (flash_attention.cu:606-663) on top of the C ABI, with the reference's
// error convention (CUDA_CHECK -> fprintf + exit(EXIT_FAILURE), :22-30, :662).
//
// The signature carries no workspace, but the tiers that need one -- the
// causal split tier and the W4 tier's cross-XCD tail pool (fa_mi355x.h,
// fa_fwd_f16_ws) -- are the dispatcher's choice for their shapes, so this
// wrapper owns one zero-filled workspace per (device, stream), created on the
// first call that needs it and grown (never shrunk) outside graph capture.
// A reference caller therefore runs exactly the tier a torch caller runs.
#include "flash_attention_v9.h"

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <map>
#include <mutex>
#include <utility>

#include "fa_mi355x.h"

static void fa_check(int status, const char* file, int line) {
  if (status != FA_OK) {
    const hipError_t e = hipGetLastError();
    fprintf(stderr, "HIP error at %s:%d: %s (%s)\n", file, line, fa_status_string(status),
            hipGetErrorString(e));
    exit(EXIT_FAILURE);
  }
}

static void hip_check(hipError_t e, const char* file, int line) {
  if (e != hipSuccess) {
    fprintf(stderr, "HIP error at %s:%d: %s\n", file, line, hipGetErrorString(e));
    exit(EXIT_FAILURE);
  }
}

namespace {

struct Slab {
  void* ptr = nullptr;
  unsigned long long bytes = 0;
};

std::mutex g_mu;
// (device, stream) -> workspace; kept for the process (a stream's launches may
// still be queued on it when the call returns)
std::map<std::pair<int, hipStream_t>, Slab> g_slabs;

// A workspace of >= need bytes for launches on `stream`, zero-filled in stream
// order before its first use (fa_fwd_f16_ws leaves its counters zero after
// every launch, so it stays valid for any later shape on this stream).
// nullptr if it would have to be created or grown while `stream` is being
// captured into a graph: allocation is not a stream operation, so the call
// then runs the workspace-free tiers, as fa_fwd_f16 does.
void* workspace(unsigned long long need, hipStream_t stream, unsigned long long* bytes) {
  int dev = 0;
  hip_check(hipGetDevice(&dev), __FILE__, __LINE__);
  std::lock_guard<std::mutex> lock(g_mu);
  Slab& s = g_slabs[{dev, stream}];
  if (s.bytes < need) {
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    hip_check(hipStreamIsCapturing(stream, &cap), __FILE__, __LINE__);
    if (cap != hipStreamCaptureStatusNone) return nullptr;
    if (s.ptr) {
      // launches queued on the old slab are done before it is freed
      hip_check(hipStreamSynchronize(stream), __FILE__, __LINE__);
      hip_check(hipFree(s.ptr), __FILE__, __LINE__);
      s = Slab();
    }
    void* p = nullptr;
    hip_check(hipMalloc(&p, need), __FILE__, __LINE__);  // 256-B aligned
    hip_check(hipMemsetAsync(p, 0, need, stream), __FILE__, __LINE__);
    s.ptr = p;
    s.bytes = need;
  }
  *bytes = s.bytes;
  return s.ptr;
}

}  // namespace

void flash_attention_v9_dispatch(const half* Q, const half* K, const half* V, half* Output,
                                 float* splitk_buf_O, float* splitk_buf_ml, int batch_size,
                                 int num_heads, int seq_len, int head_dim, bool causal,
                                 hipStream_t stream) {
  // The reference accepts the split-K buffers and never touches them (its
  // dispatcher launches split_k = 1 only, :606-663).  Same here: a caller
  // cannot learn a split count or buffer size through this signature, so
  // writing into them could run past a buffer sized for the caller's own
  // split count.  Split-KV is the explicit fa_fwd_f16_splitkv entry point.
  (void)splitk_buf_O;
  (void)splitk_buf_ml;
  const int c = causal ? 1 : 0;
  const unsigned long long need = fa_fwd_ws_bytes(batch_size, num_heads, seq_len, head_dim, c, 0);
  unsigned long long ws_bytes = 0;
  void* ws = need ? workspace(need, stream, &ws_bytes) : nullptr;
  const int rc = ws ? fa_fwd_f16_ws(Q, K, V, Output, batch_size, num_heads, seq_len, head_dim, c, 0,
                                    ws, ws_bytes, stream)
                    : fa_fwd_f16(Q, K, V, Output, batch_size, num_heads, seq_len, head_dim, c, stream);
  fa_check(rc, __FILE__, __LINE__);
}
