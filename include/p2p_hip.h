/*
 * p2p_hip.h -- C ABI of the MI355X (gfx950) Prompt-to-Prompt attention-control library.
 *
 * Every entry point replaces one call site of the reference's attention-control hot path
 * (KIMGEONUNG/prompt-to-prompt; file:line below).  Conventions:
 *   - all tensor pointers are DEVICE pointers, row-major, caller-owned; the library never
 *     allocates, never synchronises, and launches on the given stream only;
 *   - small per-call tables (batch index maps, group lists) are HOST arrays, copied into the
 *     kernel arguments (no device upload per call);
 *   - the return value is 0 on success, a hipError_t value (> 0) on a launch failure, or a
 *     negative P2P_E_* code when the arguments are rejected before anything is launched.
 *   - q/k/v/o use the projection layout [n_batch, tokens, n_heads * head_dim] (the to_q /
 *     to_k / to_v outputs); the head split of ptp_utils.py:191-193 and the merge of :207 are
 *     done by strides, not copies.
 */
#ifndef P2P_HIP_H
#define P2P_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define P2P_ABI_VERSION 15
#define P2P_MAX_BATCH 64  /* entries per launch (U-Net batch: 2 x prompts x groups)   */
#define P2P_MAX_GROUPS 32 /* prompt groups per cross-attention launch                 */
#define P2P_MAX_KEYS_CROSS 96
#define P2P_PROGRAM_COLS 128 /* column stride of an edit program (>= n_key)          */
#define P2P_PROGRAM_TMAX 8   /* term planes per edit (source words per target word)  */
/* bytes of one edit's record: c_rep f32[COLS] | post f32[COLS] | {i32 row, f32 val}[TMAX][COLS] */
#define P2P_PROGRAM_REC_BYTES (2 * 4 * P2P_PROGRAM_COLS + 8 * P2P_PROGRAM_TMAX * P2P_PROGRAM_COLS)
#define P2P_PROGRAM_HEADER_BYTES 32
#define P2P_PROGRAM_DENSE 96 /* dense mapper tile: f16 [DENSE][DENSE] per edit              */
enum {
  P2P_PROGRAM_F_DENSE = 1, /* p2p_group.flags: the program carries the dense f16 tile           */
  /* p2p_group.flags (ABI 14), a per-call hint: for this call's alpha row every edit's blend
   * coefficient A[w] = alpha[w] * post[w] * c_rep[w] + 1 - alpha[w] is 0 (a Replace or Reweight
   * step inside cross_replace_steps, main.py:189), so P_e' = R and the edit entries' own Q K^T
   * softmax, Q and K are not needed -- the bf16 dense kernels then load only their V.  The
   * kernel re-derives A from the program and falls back to the full edit if the hint is wrong. */
  P2P_GROUP_F_R_ONLY = 2,
  /* p2p_group.flags (ABI 15), a caller guarantee, also for groups without a program: every entry
   * of the group has the SAME K and V values as its first entry (the uncond prompts "" of a group,
   * ptp_utils.py:150-156, whose context rows are equal).  The group kernel then stages them once
   * per workgroup instead of per entry; results are bit-identical when the guarantee holds. */
  P2P_GROUP_F_SHARED_KV = 4
};

enum { P2P_DTYPE_F32 = 0, P2P_DTYPE_BF16 = 1 };
enum { P2P_COMPUTE_BF16 = 0, P2P_COMPUTE_F32 = 1 };

enum {
  P2P_E_ARG = -1,       /* null pointer / inconsistent sizes                             */
  P2P_E_HEAD_DIM = -2,  /* head_dim without a compiled kernel                             */
  P2P_E_DTYPE = -3,     /* io_dtype / compute combination not supported                   */
  P2P_E_KEYS = -4,      /* n_key above P2P_MAX_KEYS_CROSS for the cross kernel            */
  P2P_E_BATCH = -5,     /* n_batch above P2P_MAX_BATCH or group list inconsistent         */
  P2P_E_ALIGN = -6      /* a pointer / stride breaks the 16-byte vector-load alignment    */
};

typedef void* p2p_stream_t; /* a hipStream_t */

/* One attention call: q [n_batch, n_query, *], k/v [n_batch, n_key, *], o like q.
 * Strides are in elements.  scale is CrossAttention.scale (head_dim ** -0.5,
 * ptp_utils.py:195). */
typedef struct {
  const void* q;
  const void* k;
  const void* v;
  void* o;
  int64_t q_row_stride, k_row_stride, v_row_stride, o_row_stride;
  int64_t q_batch_stride, k_batch_stride, v_batch_stride, o_batch_stride;
  int32_t n_batch, n_query, n_key, n_heads, head_dim;
  int32_t io_dtype; /* P2P_DTYPE_*  (element type of q, k, v, o)                      */
  int32_t compute;  /* P2P_COMPUTE_* (bf16 MFMA, or exact-f32 MFMA check mode)          */
  float scale;
} p2p_attn_tensors;

/* Self-attention (ptp_utils.py:183-208 with context=None) fused with the controller's
 * self-attention edit and the AttentionStore epilogue:
 *   O[n] = softmax(Q[qk_src[n]] K[qk_src[n]]^T * scale) V[n]
 * qk_src (host, n_batch entries, NULL = identity) implements the source-map injection of
 * AttentionControlEdit.replace_self_attention (main.py:169-174, null_text.py:224-230): an
 * edit inside the self_replace window reads the SOURCE prompt's probabilities and its OWN
 * values.  store (nullable) receives the normalised probabilities of every entry whose
 * store_slot (host) is >= 0 at maps [store_slot[n] + head] of a [*, n_query, n_key] f32
 * tensor, overwritten (store_accumulate = 0, first step) or added (= 1): the running sum
 * of AttentionStore.between_steps (main.py:135-142).  lse_workspace: f32
 * [n_batch * n_heads, n_query] scratch, required (16-byte aligned) when some entry stores its
 * maps, else ignored: the fused pass leaves each row's log-sum-exp there and the map pass
 * recomputes the probabilities from it. */
int p2p_self_attn_fwd(const p2p_attn_tensors* t, const int32_t* qk_src, float* store,
                      const int32_t* store_slot, int32_t store_accumulate, float* lse_workspace,
                      p2p_stream_t stream);

/* A prompt group of a cross-attention launch: entries [first, first + count) of the batch;
 * entry `first` is the source prompt, the others its edits (main.py:187).  program is the
 * device edit program or NULL
 * for no edit; alpha is the device [count - 1][n_key] row cross_replace_alpha[cur_step]
 * (main.py:189).  Program layout (p2p_amd/programs.py): int32 header[8] {n_edits, n_cols, tmax,
 * P2P_PROGRAM_COLS, dense, dense_offset, 0, 0}, then per edit e at byte
 * P2P_PROGRAM_HEADER_BYTES + e * P2P_PROGRAM_REC_BYTES: c_rep f32[COLS],
 * post f32[COLS], term planes {i32 row, f32 val}[P2P_PROGRAM_TMAX][COLS] -- plane t of column
 * w is the t-th source row feeding target word w, (0, 0.0) past its last term; tmax <= TMAX is
 * the number of planes the kernel walks:
 *   R[w] = post[w] * (c_rep[w] * P_e[w] + sum_{t < tmax} val[t][w] * P_0[row[t][w]])
 *   P_e'[w] = alpha[w] * R[w] + (1 - alpha[w]) * P_e[w]
 * When every term value is exact in f16 the program also holds, at byte dense_offset, the
 * dense mapper of each edit as f16 [P2P_PROGRAM_DENSE rows (source word)][P2P_PROGRAM_DENSE
 * cols (target word)] (zeros elsewhere), and the host sets P2P_PROGRAM_F_DENSE in flags: the
 * bf16 kernels then form sum_t val * P_0[row] as one f16 MFMA product P_0 . M_e (P_0 rounded
 * to 11 significant bits, <= 2^-12 relative) instead of an LDS gather.  (ABI 12: f16 tile.)  */
typedef struct {
  int32_t first;
  int32_t count;
  const void* program;
  const float* alpha;
  int32_t flags;   /* P2P_PROGRAM_F_* of program (host-known: sizes the launch's LDS) */
  int32_t n_edits; /* edit records the program holds (its header[0]); a group with
                      count - 1 > n_edits is rejected (P2P_E_BATCH) before any launch */
  /* LocalBlend's word reduction folded into the store epilogue (null_text.py:41-46,
   * main.py:37-44: (maps * alpha).sum(-1) of the five 16x16 cross layers), nullable: for entry
   * b of the group, head h and query row p
   *   blend_sums[((b * 2 + s) * blend_lh + blend_col + h) * n_query + p]  = / +=
   *       sum_w P'[p][w] * alpha_s[b][w],   alpha_0 = blend_alpha, alpha_1 = blend_sub (or 0)
   * with P' the post-edit probabilities the store receives, written when store_accumulate = 0
   * and added otherwise -- the running sum of the word sums, which is what p2p_localblend
   * (word_sums_ready) reads instead of re-reading the maps.  Needs every entry of the group to
   * store (store_slot >= 0). */
  float* blend_sums;
  const float* blend_alpha; /* [count][n_key] f32                                          */
  const float* blend_sub;   /* [count][n_key] f32 or NULL                                  */
  int32_t blend_col;        /* this layer's first column (layer index * n_heads)            */
  int32_t blend_lh;         /* columns of the sums: blended layers * n_heads                */
} p2p_group;

/* Cross-attention (ptp_utils.py:183-208 with context=...) with the controller's cross edit
 * applied in registers between softmax and PV (AttentionControlEdit.forward, main.py:180-197:
 * Replace :217-218, Refine :235-239, Reweight :258-264) and the AttentionStore epilogue
 * (store/store_slot/store_accumulate as for p2p_self_attn_fwd; stored maps are the
 * post-edit probabilities, as the reference's aliasing store holds). */
int p2p_cross_attn_fwd(const p2p_attn_tensors* t, const p2p_group* groups, int32_t n_groups,
                       float* store, const int32_t* store_slot, int32_t store_accumulate,
                       p2p_stream_t stream);

/* Materialise mode, for controllers that override forward(attn, ...) (the reference
 * protocol, main.py:85-98): probs[n*H + h] = softmax(Q K^T * scale) as an f32
 * [n_batch * n_heads, n_query, n_key] tensor (ptp_utils.py:195-204).  key_mask (nullable,
 * uint8 [n_batch, n_key], nonzero = keep) reproduces ptp_utils.py:197-201, including its
 * head-major repeat of the mask rows: a masked key scores -FLT_MAX after the scale, so it gets
 * p = 0 beside any kept key and a fully masked row is uniform, 1/n_key. */
int p2p_attn_probs(const p2p_attn_tensors* t, const uint8_t* key_mask, float* probs,
                   p2p_stream_t stream);

/* Materialise mode, second half: O[n] = probs[n*H + h] V[n] (ptp_utils.py:206-207). */
int p2p_attn_pv(const p2p_attn_tensors* t, const float* probs, p2p_stream_t stream);

/* Attention with its gradient -- what null-text inversion needs (null_text.py:574-606: Adam on
 * the null embedding through every patched attention of the U-Net).  Forward: O as
 * p2p_self_attn_fwd with no controller edit, plus lse [n_batch * n_heads, n_query] f32, the row
 * log-sum-exp in the log2 domain with the scale folded in (softmax row = exp2(scale * log2(e) *
 * s - lse)).  Any n_key (self- or cross-attention); bf16 compute only. */
int p2p_attn_fwd_lse(const p2p_attn_tensors* t, float* lse, p2p_stream_t stream);

/* Backward of O = softmax(Q K^T * scale) V for the same tensors (t->o = the forward's O):
 *   dV = P^T dO,  dS = P o (dO V^T - rowsum(dO o O)),  dQ = scale dS K,  dK = scale dS^T Q.
 * dout and dq use q's layout (strides of t->q / t->o); dk, dv are packed [n_batch, n_key,
 * n_heads * head_dim], written (not accumulated) in io_dtype, or in f32 when kv_f32 = 1.
 * delta: workspace [n_batch * n_heads, n_query] f32.  workspace: p2p_attn_bwd_workspace(t)
 * bytes (NULL when that is 0): when the key tiles alone would leave the chip idle (cross
 * attention, small batches) the key/value pass splits the queries over workgroups, each split
 * stores its partial dK/dV there and a reduction adds them in split order -- deterministic,
 * no atomics.  P is recomputed from lse; bf16 MFMA operands, f32 accumulation. */
int64_t p2p_attn_bwd_workspace(const p2p_attn_tensors* t);
int p2p_attn_bwd(const p2p_attn_tensors* t, const void* dout, const float* lse, float* delta, void* dq,
                 void* dk, void* dv, int32_t kv_f32, void* workspace, int64_t workspace_bytes,
                 p2p_stream_t stream);

/* LocalBlend (null_text.py:41-70; main.py:35-52 is the B=2 special case) for one prompt
 * group: maps[l] are the running-sum cross maps of the five 16x16 layers
 * (down_cross[2:4] + up_cross[:3]), each [n_prompts * heads_per_map, 256, n_words] f32. */
typedef struct {
  const float* maps[8];
  int32_t n_maps;
  int32_t heads_per_map;
  int32_t n_prompts;
  int32_t n_words;
  int32_t map_res;                 /* 16                                               */
  const float* alpha_layers;       /* [n_prompts, n_words]                             */
  const float* substruct_layers;   /* [n_prompts, n_words] or NULL                     */
  float th_pool, th_sub;           /* th[0], th[1] (main form: threshold, unused)      */
  float* x_t;                      /* [n_prompts, channels, lat_h, lat_w] in/out       */
  int32_t channels, lat_h, lat_w;
  float* word_sums;                /* workspace [n_prompts, 2, n_maps*heads, res*res]  */
  uint8_t* mask_out;               /* optional [n_prompts, lat_h, lat_w] final mask    */
  int32_t word_sums_ready;         /* 1: word_sums already hold the word reductions (the
                                      running sums folded by p2p_cross_attn_fwd's
                                      blend_sums); maps are then not read (may be NULL)   */
} p2p_blend_args;

/* x_t may be NULL when mask_out is given: the mask is computed and nothing is blended (the
 * latent blend then happens inside p2p_latent_step). */
int p2p_localblend(const p2p_blend_args* a, p2p_stream_t stream);

/* One denoising step's latent update, fused (ptp_utils.py:72-75 diffusion_step tail):
 *   noise = eps_u + guidance * (eps_c - eps_u)                      (cfg = 1; else noise = eps)
 *   x0    = (x - sqrt_beta_t * noise) / sqrt_alpha_t                 (null_text.py:475-479:
 *   out   = sqrt_alpha_prev * x0 + sqrt_one_minus_alpha_prev * noise  prev_step; next_step with
 *                                                                      the inversion coefficients)
 *   out[b] = out[g0] + mask[b] * (out[b] - out[g0])  b not a group's  (LocalBlend, mask nullable;
 *                                                    first prompt g0     g0 = first prompt of b's
 *                                                                        group of group_size)
 * eps [cfg ? 2B : B, C, H, W] in eps_dtype (uncond block first, as torch.cat([latents] * 2)),
 * x / out [B, C, H, W] f32 (out may alias x), mask uint8 [B, H, W] (p2p_localblend mask_out).
 * The four coefficients are the host-side 0-dim values the scheduler computes (beta_t ** 0.5 ...).
 * Intermediates are rounded as the reference's eager torch ops round them (bf16 products for a
 * bf16 eps), so the result is bit-identical to the unfused sequence. */
typedef struct {
  const void* eps;
  int32_t eps_dtype;               /* P2P_DTYPE_*                                      */
  int32_t cfg;
  float guidance;
  const float* x;
  float* out;
  int32_t n_prompts, channels, height, width;
  float sqrt_beta_t, sqrt_alpha_t, sqrt_alpha_prev, sqrt_one_minus_alpha_prev;
  const uint8_t* mask;
  int32_t group_size;              /* prompts per prompt group (0 = one group of n_prompts) */
  const uint8_t* group_blend;      /* [n_prompts / group_size] 1 = blend this group, NULL = all */
  /* LocalBlend in the same launch (one kernel per denoising step): when blend_sums[g] is set,
   * prompt group g's mask is built here from the running word sums the cross-attention store
   * epilogue folded (p2p_group.blend_sums: [group_size, 2, blend_lh, blend_res^2] f32) --
   * mean over the blend_lh layer x head maps, 3x3 max-pool, nearest upsampling, per-image max
   * normalisation, thresholds, mask[:1] | mask and the substruct gate (null_text.py:41-67),
   * exactly as p2p_localblend with word_sums_ready = 1 builds it -- and the blend of
   * null_text.py:68-70 follows.  `mask` must then be NULL; NULL entries do not blend.
   * (ptp_utils.py:75 step_callback + null_text.py:41-70, fused with the CFG/DDIM update.) */
  const float* blend_sums[P2P_MAX_GROUPS];
  int32_t blend_lh;                /* layer x head maps per prompt (5 x 8)                   */
  int32_t blend_res;               /* map resolution (16); res^2 <= 256, <= lat_h, lat_w     */
  float blend_th_pool, blend_th_sub;
  int32_t blend_sub;               /* 1: the substruct sums (index 1) gate the mask          */
} p2p_latent_step_args;

int p2p_latent_step(const p2p_latent_step_args* a, p2p_stream_t stream);

/* AttentionStore.get_average_attention (main.py:144-149): dst = src / divisor, computed as
 * src * (1.0f / divisor) -- what torch does for `cuda_tensor / python_scalar` on the
 * reference's cuda:0 device. */
int p2p_store_scale(const float* src, float* dst, float divisor, int64_t n, p2p_stream_t stream);

/* Measurement only (ABI 15; bench.py's roofline clock, not part of the reference's interface):
 * n_workgroups one-wave workgroups each read the shader-cycle counter and the constant 100 MHz
 * counter, spin until `ticks` (1..1e6) of the 100 MHz counter have passed, and read both again:
 * out[2 w] = shader cycles, out[2 w + 1] = 100 MHz ticks of workgroup w, so the shader clock is
 * out[2 w] / out[2 w + 1] x 100 MHz.  Consecutive workgroups run on different XCDs.  out: device
 * memory, 2 x n_workgroups (1..1024) u64. */
int p2p_clock_probe(uint64_t* out, int32_t n_workgroups, int32_t ticks, p2p_stream_t stream);

/* Measurement only (ABI 15): kernel timing events (hipEvent_t, created by the caller) for the
 * next p2p_* calls of the calling thread -- their kernels are launched with hipExtLaunchKernel,
 * the first one recording `start`, each one `stop` (the last kernel's stands), from the kernels'
 * own dispatch timestamps.  Clear with (NULL, NULL).  Always returns 0. */
int p2p_set_launch_events(void* start, void* stop);

/* Build/runtime information.  p2p_source_hash: content hash of the HIP sources the library
 * was built from (p2p_amd/_srchash.py), so a host can refuse a stale prebuilt binary. */
int p2p_abi_version(void);
const char* p2p_source_hash(void);
const char* p2p_error_string(int code);

#ifdef __cplusplus
}
#endif
#endif /* P2P_HIP_H */
