// flash_attention_main.cpp -- the reference's executable harness
// (flash_attention.cu:702-971) rebuilt on the MI355X library: register/occupancy
// report, the four correctness checks against the CPU oracle, then the
// non-causal and causal benchmark sweeps with the reference's timing loop
// (20 warm-up + 100 timed dispatches x 3 runs, event-timed).
//
// Test infrastructure: it links the oracle (oracle/fa_oracle.c) as the
// reference's main() links cpu_attention.  Calls the kernel only through the
// reference-signature wrapper flash_attention_v9_dispatch (include/).
//
// Differences from the reference, all additive:
//  * the checks gate at 1e-3 (BASELINE.json) and also print the reference's
//    0.1 verdict; extra checks cover the causal-long tier and ragged seq;
//  * optional CLI from README.md:83-85: `flash_attention [seq [causal]]` runs
//    only that one benchmark shape; env FA_COOLDOWN_S overrides the 5 s
//    cooldown (:900-902), FA_SKIP_BENCH=1 stops after the checks.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <vector>

#include "fa_mi355x.h"
#include "fa_oracle.h"
#include "flash_attention_v9.h"

#define HIP_CHECK(call)                                                                    \
  do {                                                                                     \
    hipError_t err = call;                                                                 \
    if (err != hipSuccess) {                                                               \
      fprintf(stderr, "HIP error at %s:%d: %s\n", __FILE__, __LINE__, hipGetErrorString(err)); \
      exit(EXIT_FAILURE);                                                                  \
    }                                                                                      \
  } while (0)

static const float kGate = 1e-3f;

static bool correctness_check(const char* label, int batch, int heads, int seq, bool causal) {
  printf("Correctness check (%s)...\n", label);
  const int hd = 128;
  const size_t n = (size_t)batch * heads * seq * hd;
  std::vector<uint16_t> q(n), k(n), v(n), o(n), ref(n);
  fa_oracle_gen_inputs(q.data(), k.data(), v.data(), n, 42);
  fa_oracle_attention(q.data(), k.data(), v.data(), ref.data(), batch, heads, seq, hd,
                      causal ? 1 : 0, 16);
  half *dq, *dk, *dv, *dout;
  const size_t sz = n * sizeof(uint16_t);
  HIP_CHECK(hipMalloc(&dq, sz));
  HIP_CHECK(hipMalloc(&dk, sz));
  HIP_CHECK(hipMalloc(&dv, sz));
  HIP_CHECK(hipMalloc(&dout, sz));
  HIP_CHECK(hipMemcpy(dq, q.data(), sz, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(dk, k.data(), sz, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(dv, v.data(), sz, hipMemcpyHostToDevice));
  flash_attention_v9_dispatch(dq, dk, dv, dout, nullptr, nullptr, batch, heads, seq, hd, causal);
  HIP_CHECK(hipDeviceSynchronize());
  HIP_CHECK(hipMemcpy(o.data(), dout, sz, hipMemcpyDeviceToHost));
  const float maxdiff = fa_oracle_max_abs_diff(o.data(), ref.data(), n);
  const bool ok = maxdiff <= kGate;
  printf("  max_diff=%.6f %s (gate 1e-3; reference gate 0.1: %s)\n", maxdiff,
         ok ? "PASS" : "FAIL", maxdiff < 0.1f ? "PASS" : "FAIL");
  HIP_CHECK(hipFree(dq));
  HIP_CHECK(hipFree(dk));
  HIP_CHECK(hipFree(dv));
  HIP_CHECK(hipFree(dout));
  return ok;
}

static void register_report() {
  const int n = fa_num_configs();
  for (int i = 0; i < n; ++i) {
    fa_config_info_t ci;
    fa_kernel_attrs_t ka;
    if (fa_config_info(i, &ci) != FA_OK || fa_kernel_attrs(i, &ka) != FA_OK) continue;
    printf("%-34s BM%-3d BN%-3d %dw  %3d VGPR, %d spill, %6d B LDS, %d blk/CU\n", ci.name,
           ci.block_m, ci.block_n, ci.waves, ka.num_regs, ka.local_size_bytes, ci.lds_bytes,
           ka.blocks_per_cu);
  }
  printf("\n");
}

// the tier flash_attention_v9_dispatch runs for a shape (it owns a workspace,
// so it takes the split tier / the W4 tail pool where the dispatcher does)
static const char* tier_label(int batch, int heads, int seq, bool causal, char* buf, size_t n) {
  const int c = causal ? 1 : 0;
  const int T = fa_fwd_split_pieces(batch, heads, seq, 128, c);
  if (T > 0) {
    snprintf(buf, n, "causal_split_T%d", T);
    return buf;
  }
  fa_config_info_t ci;
  fa_config_info(fa_select_config(batch, heads, seq, c), &ci);
  const bool pool = fa_fwd_ws_bytes(batch, heads, seq, 128, c, 0) > 0;
  snprintf(buf, n, "%s%s", ci.name, pool ? "+pool" : "");
  return buf;
}

static void bench_one(int seq, int heads, bool causal, int batch = 1) {
  const int hd = 128, runs_n = 3;
  const size_t n = (size_t)batch * heads * seq * hd, sz = n * sizeof(uint16_t);
  char label[128];
  const char* name = tier_label(batch, heads, seq, causal, label, sizeof(label));
  if (sz * 4 > 15ULL * 1024 * 1024 * 1024) {  // :918-921
    printf("%-3d %-6d  %-5d  %-28s  SKIP\n", batch, seq, heads, name);
    return;
  }
  // the reference's srand(42) inputs for one batch entry (:924-929), copied to
  // every batch entry (the generator would take minutes at B = 64)
  const size_t n1 = (size_t)heads * seq * hd, sz1 = n1 * sizeof(uint16_t);
  std::vector<uint16_t> q(n1), k(n1), v(n1);
  fa_oracle_gen_inputs(q.data(), k.data(), v.data(), n1, 42);
  half *dq, *dk, *dv, *dout;
  HIP_CHECK(hipMalloc(&dq, sz));
  HIP_CHECK(hipMalloc(&dk, sz));
  HIP_CHECK(hipMalloc(&dv, sz));
  HIP_CHECK(hipMalloc(&dout, sz));
  for (int b = 0; b < batch; ++b) {
    HIP_CHECK(hipMemcpy(dq + b * n1, q.data(), sz1, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dk + b * n1, k.data(), sz1, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(dv + b * n1, v.data(), sz1, hipMemcpyHostToDevice));
  }
  double flops = 4.0 * batch * heads * (double)seq * seq * hd;
  if (causal) flops /= 2;
  float runs[runs_n], sum = 0;
  for (int r = 0; r < runs_n; ++r) {
    if (r > 0) {
      HIP_CHECK(hipDeviceSynchronize());
      usleep(1000000);
    }
    for (int i = 0; i < 20; ++i)
      flash_attention_v9_dispatch(dq, dk, dv, dout, nullptr, nullptr, batch, heads, seq, hd,
                                  causal);
    HIP_CHECK(hipDeviceSynchronize());
    hipEvent_t start, stop;
    HIP_CHECK(hipEventCreate(&start));
    HIP_CHECK(hipEventCreate(&stop));
    HIP_CHECK(hipEventRecord(start));
    for (int i = 0; i < 100; ++i)
      flash_attention_v9_dispatch(dq, dk, dv, dout, nullptr, nullptr, batch, heads, seq, hd,
                                  causal);
    HIP_CHECK(hipEventRecord(stop));
    HIP_CHECK(hipEventSynchronize(stop));
    float ms;
    HIP_CHECK(hipEventElapsedTime(&ms, start, stop));
    ms /= 100;
    runs[r] = (float)(flops / (ms / 1000.0) / 1e12);
    sum += runs[r];
    HIP_CHECK(hipEventDestroy(start));
    HIP_CHECK(hipEventDestroy(stop));
  }
  const float avg = sum / runs_n;
  const double peak = 256 * 2.4e9 * 4096 / 1e12;
  printf("%-3d %-6d  %-5d  %-28s  %7.1f  %7.1f  %7.1f  %7.1f  (%4.1f%% MFMA peak)\n", batch, seq,
         heads, name, runs[0], runs[1], runs[2], avg, 100.0 * avg / peak);
  HIP_CHECK(hipFree(dq));
  HIP_CHECK(hipFree(dk));
  HIP_CHECK(hipFree(dv));
  HIP_CHECK(hipFree(dout));
}

int main(int argc, char** argv) {
  printf("=== Flash Attention MI355X (gfx950) -- %s ===\n", fa_version());
  printf("batch=1, head_dim=128, fp16 in/out, fp32 accumulate\n\n");
  register_report();

  bool all_ok = true;
  const bool causal = true;  // :709
  all_ok &= correctness_check("seq=256, causal", 1, 32, 256, causal);      // :757-788
  all_ok &= correctness_check("seq=1024, causal", 1, 32, 1024, true);      // :790-820
  all_ok &= correctness_check("seq=1024, non-causal", 1, 32, 1024, false); // :822-852
  all_ok &= correctness_check("seq=2048, non-causal", 1, 2, 2048, false);  // :854-884
  // beyond the reference: causal-long tier and ragged lengths
  all_ok &= correctness_check("seq=4096, causal, h4", 1, 4, 4096, true);
  all_ok &= correctness_check("seq=1000, causal, b2 h3", 2, 3, 1000, true);
  all_ok &= correctness_check("seq=77, non-causal, b2 h3", 2, 3, 77, false);
  printf("\n");
  if (getenv("FA_SKIP_BENCH")) return all_ok ? 0 : 1;

  int cooldown = 5;
  if (getenv("FA_COOLDOWN_S")) cooldown = atoi(getenv("FA_COOLDOWN_S"));
  if (argc > 1) {  // README.md:83-85 CLI: seq [causal]
    const int seq = atoi(argv[1]);
    const bool c = argc > 2 ? atoi(argv[2]) != 0 : true;
    printf("%-3s %-6s  %-5s  %-28s  Run1     Run2     Run3     Avg (TFLOPS)\n", "B", "seq",
           "heads", "tier");
    bench_one(seq, 32, c);
    return all_ok ? 0 : 1;
  }
  const int seqs[] = {512, 768, 1024, 2048, 4096, 8192, 16384};  // :888-896
  for (int pass = 0; pass < 2; ++pass) {
    const bool bc = pass == 1;  // non-causal first, causal second (:900)
    if (pass > 0) {
      printf("\nCooldown %ds...\n", cooldown);
      HIP_CHECK(hipDeviceSynchronize());
      sleep(cooldown);
    }
    printf("\n=== %s ===\n", bc ? "CAUSAL" : "NON-CAUSAL");
    printf("%-3s %-6s  %-5s  %-28s  Run1     Run2     Run3     Avg (TFLOPS)\n", "B", "seq",
           "heads", "tier");
    printf("-----------------------------------------------------------------------------\n");
    for (int s : seqs) bench_one(s, 32, bc);
  }
  // beyond the reference: the shapes whose tier needs the wrapper's workspace
  // -- BASELINE config 5 on one GPU (the W4 tail pool) and long few-head
  // causal launches (the causal split tier)
  printf("\n=== WORKSPACE TIERS (causal) ===\n");
  printf("%-3s %-6s  %-5s  %-28s  Run1     Run2     Run3     Avg (TFLOPS)\n", "B", "seq", "heads",
         "tier");
  bench_one(4096, 32, true, 64);
  bench_one(8192, 4, true);
  bench_one(16384, 2, true);
  return all_ok ? 0 : 1;
}
