/*
 * fa_mi355x.h -- C ABI of the MI355X (gfx950) flash-attention forward path.
 *
 * This is the drop-in boundary for the reference's host dispatcher
 *   void flash_attention_v9_dispatch(const half* Q, const half* K,
 *       const half* V, half* Output, float* splitk_buf_O,
 *       float* splitk_buf_ml, int batch_size, int num_heads, int seq_len,
 *       int head_dim, bool causal, cudaStream_t stream = 0)
 * (/root/reference/flash_attention.cu:606-663).  The C++ signature itself is
 * kept in flash_attention_v9.h and forwards here.
 *
 * Conventions shared by every entry point:
 *  - q, k, v, o are DEVICE pointers owned by the caller (the reference
 *    allocates them in main, :772-787), fp16 (IEEE binary16), layout BHSD:
 *    [batch*heads][seq_len][head_dim] contiguous, bh stride seq_len*head_dim
 *    (:119-122, :672-675).
 *  - Stream-ordered and non-blocking: the call enqueues on hip_stream (a
 *    hipStream_t, NULL = default stream) and returns; no allocation, no
 *    synchronisation, safe to capture into a hipGraph.
 *  - Return value: FA_OK (0) or a nonzero fa_status_t.  The reference's
 *    equivalent is CUDA_CHECK(cudaGetLastError()) -> exit (:22-30, :662);
 *    flash_attention_v9_dispatch() keeps that behaviour on top of this ABI.
 */
#ifndef FA_MI355X_H
#define FA_MI355X_H

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  FA_OK = 0,
  FA_ERR_NULL_POINTER = 1,        /* q/k/v/o NULL with a non-empty problem */
  FA_ERR_UNSUPPORTED_HEAD_DIM = 2,/* head_dim not 128 (ref :613 HD=128) or 64 */
  FA_ERR_BAD_SHAPE = 3,           /* negative sizes, int overflow of B*H, or
                                     seq_len*2*head_dim (split-KV: *4) past
                                     INT_MAX: S <= 8388607 at head_dim 128 */
  FA_ERR_LAUNCH = 4,              /* hipGetLastError() after the launch */
  FA_ERR_BAD_CONFIG = 5,          /* config id out of range / wrong causal */
  FA_ERR_HIP = 6,                 /* other HIP runtime failure */
  FA_ERR_WORKSPACE = 7            /* split-KV buffers / workspace missing or short */
} fa_status_t;

/* Tile configuration descriptor (the reference's template switches
 * BLOCK_M/BLOCK_N/NWARPS/IS_CAUSAL, :67-70, re-expressed for 64-wide waves). */
typedef struct {
  int id;
  int block_m;      /* query rows per workgroup */
  int block_n;      /* key/value rows per LDS tile */
  int waves;        /* 64-lane wavefronts per workgroup */
  int causal;       /* 1 = causal instantiation */
  int split_kv;     /* 1 = writes fp32 partials for the LSE merge */
  int lds_bytes;    /* dynamic LDS per workgroup */
  const char* name;
  int dtype;        /* FA_DTYPE_F16 or FA_DTYPE_BF16: element type of Q/K/V/O */
  int head_dim;     /* 128 (the reference's) or 64 */
} fa_config_info_t;

enum { FA_DTYPE_F16 = 0, FA_DTYPE_BF16 = 1 };

/* Per-config compiled resource usage: the reference's register/occupancy
 * report (cudaFuncGetAttributes + cudaOccupancyMaxActiveBlocksPerMultiprocessor,
 * :711-755).  Requires a visible GPU for the occupancy field. */
typedef struct {
  int num_regs;           /* arch VGPRs per lane (hipFuncAttributes.numRegs) */
  int local_size_bytes;   /* scratch (spill) bytes per lane */
  int shared_size_bytes;  /* static LDS */
  int max_threads_per_block;
  int blocks_per_cu;      /* occupancy query at the config's LDS size; -1 if no GPU */
} fa_kernel_attrs_t;

/* Main entry: fused QK^T -> online softmax -> PV forward, fp16 in/out,
 * fp32 accumulate, scale = 1/sqrt(head_dim) (ref :612).  Chooses the tile
 * config with fa_select_config(). Replaces flash_attention_v9_dispatch
 * (flash_attention.cu:606-663). */
int fa_fwd_f16(const void* q, const void* k, const void* v, void* o,
               int batch, int heads, int seq_len, int head_dim, int causal,
               void* hip_stream);

/* Same, forcing one tile config (used to report each (BM,BN,waves) config,
 * as the reference's bench labels its tiers, :905-916).  The config's causal
 * flag must equal `causal`. */
int fa_fwd_f16_config(const void* q, const void* k, const void* v, void* o,
                      int batch, int heads, int seq_len, int head_dim,
                      int causal, int config_id, void* hip_stream);

/* bf16 in/out (fp32 accumulate, P rounded to bf16 before PV): the same
 * kernels on v_mfma_f32_16x16x32_bf16.  Not in the reference (fp16 only,
 * :613); SURVEY.md §8(f) rank 4.  fa_fwd_bf16 uses the bf16 twin of
 * fa_select_config()'s tier; fa_fwd_bf16_config accepts bf16 configs only
 * (fa_config_info().dtype == FA_DTYPE_BF16), fa_fwd_f16_config fp16 only. */
int fa_fwd_bf16(const void* q, const void* k, const void* v, void* o,
                int batch, int heads, int seq_len, int head_dim, int causal,
                void* hip_stream);
int fa_fwd_bf16_config(const void* q, const void* k, const void* v, void* o,
                       int batch, int heads, int seq_len, int head_dim,
                       int causal, int config_id, void* hip_stream);

/* Split-KV (flash-decoding) forward: the reference's dead IS_SPLITK path
 * (:169-180, :460-496) and its merge kernel flash_attention_splitk_merge
 * (:559-598), made live.  Buffers use the reference's layout:
 *   part_o  fp32 [num_splits][batch*heads][seq_len][head_dim]  (unnormalised O)
 *   part_ml fp32 [num_splits][batch*heads][seq_len][2]          (m, l) per row,
 *           m = running max of the scaled scores (natural-log units, as the
 *           reference's m_i), l = running sum; an empty split writes (-inf, 0).
 * num_splits <= 0 uses fa_splitkv_num_splits().  Device buffers are owned by
 * the caller and must hold fa_splitkv_o_bytes()/fa_splitkv_ml_bytes(). */
int fa_fwd_f16_splitkv(const void* q, const void* k, const void* v, void* o,
                       int batch, int heads, int seq_len, int head_dim,
                       int causal, int num_splits, float* part_o,
                       float* part_ml, void* hip_stream);
int fa_splitkv_num_splits(int batch, int heads, int seq_len, int causal);
unsigned long long fa_splitkv_o_bytes(int batch, int heads, int seq_len,
                                      int head_dim, int num_splits);
unsigned long long fa_splitkv_ml_bytes(int batch, int heads, int seq_len,
                                       int head_dim, int num_splits);

/* Workspace forward: fa_fwd_f16 / fa_fwd_bf16 plus a caller-owned device
 * workspace that lets causal launches short of the persistent tier split each
 * 256-row query block's key range into pieces run by separate workgroups and
 * merge them in the same launch (the reference's split-K log-sum-exp merge,
 * :559-598, without its second kernel; fp16 / bf16 normalised partial rows
 * plus an fp32 log2-sum-exp per row).
 *   piece_tiles = 0: the dispatcher's choice -- fa_fwd_split_pieces() is its
 *     piece length in 64-key tiles, 0 when it does not split this shape (the
 *     _ws entries then run the tier fa_fwd_f16 / fa_fwd_bf16 runs; on the
 *     persistent W4 tier with >= 64 rounds of items per XCD (the B=64
 *     headline) the workspace's counter region also carries a cross-XCD tail
 *     pool: the last 1/16 of every XCD's items are claimed at run time, which
 *     evens out XCDs that run a few % slower -- bit-identical output);
 *   piece_tiles > 0: that piece length (causal, head_dim 128, at most 8
 *     pieces per query block, else FA_ERR_BAD_CONFIG).
 * fa_fwd_ws_bytes() is the workspace the call needs (0: neither a split nor
 * a tail pool; 65536: the tail pool's counters only).  Its first 64 KB
 * (counters, the same place for every shape) must be zero before the first
 * use; every launch returns the counters it used to zero, so one buffer of
 * the largest size needed serves any sequence of shapes on ONE stream
 * (launches on different streams need their own).  A counter region that is
 * not zero (a fresh buffer never cleared, or one shared by two streams at
 * once) is not detected: pool items can be skipped and their rows left
 * unwritten, and the split merge can run early.  The workspace must be
 * 16-byte aligned (any hipMalloc / torch allocation is): FA_ERR_WORKSPACE if
 * the call splits and workspace is NULL, misaligned or ws_bytes is short; a
 * tail-pool shape with no, a short or a misaligned (not 8-byte) workspace
 * runs the static item order.  The reference-signature wrapper
 * flash_attention_v9_dispatch (flash_attention_v9.h) owns such a workspace
 * per (device, stream), so it runs the same tiers as these entries. */
unsigned long long fa_fwd_ws_bytes(int batch, int heads, int seq_len, int head_dim,
                                   int causal, int piece_tiles);
int fa_fwd_split_pieces(int batch, int heads, int seq_len, int head_dim, int causal);
int fa_fwd_f16_ws(const void* q, const void* k, const void* v, void* o,
                  int batch, int heads, int seq_len, int head_dim, int causal,
                  int piece_tiles, void* workspace, unsigned long long ws_bytes,
                  void* hip_stream);
int fa_fwd_bf16_ws(const void* q, const void* k, const void* v, void* o,
                   int batch, int heads, int seq_len, int head_dim, int causal,
                   int piece_tiles, void* workspace, unsigned long long ws_bytes,
                   void* hip_stream);

/* The dispatcher's decision (ref tier table :620-661): config id used by
 * fa_fwd_f16 for this shape.  The _ws entries may run the causal split tier
 * instead: check fa_fwd_split_pieces() first (> 0: the split tier runs with
 * that many 64-key tiles per piece, and this config is not used).
 *
 * The answer depends on the shape and on the CU count of the calling
 * thread's current HIP device (the W4 tier's tail and the paired tier's
 * one-round test size the grid from it, as the launch does; 256 if the
 * query fails).  The tier is the same for fp16 and bf16; fa_fwd_f16 /
 * fa_fwd_bf16 at head_dim 64 run the head_dim-64 twin of this tier, except
 * that non-causal head_dim-64 launches skip the paired tier (its d64 twin
 * trails the tier below there) and take the one-block-per-workgroup tier
 * only up to 16 blocks per head (S <= 1024), running the tier below it
 * otherwise.
 *
 * Config ids are positions in this build's table (fa_num_configs /
 * fa_config_info): they are not stable across releases (round 3 renumbered
 * 0-49 to 0-43 when the table was trimmed to the dispatched tiers; round 4
 * appended the head_dim-64 W4 configs 44-47; round 5 the paired
 * short-sequence configs 48-51, their four-block twins 52-55 and the
 * head_dim-64 twins of both, 56-63; round 6 the one-block-per-workgroup
 * configs 64-71, the causal singles-and-pairs mix 72-75 and the causal
 * groups planned on the host 76-79).  Select a tier by its
 * fa_config_info().name, not by a remembered id. */
int fa_select_config(int batch, int heads, int seq_len, int causal);

int fa_num_configs(void);
int fa_config_info(int config_id, fa_config_info_t* out);
int fa_kernel_attrs(int config_id, fa_kernel_attrs_t* out);

const char* fa_status_string(int status);
const char* fa_version(void);

#ifdef __cplusplus
}
#endif

#endif /* FA_MI355X_H */
