// extern "C" entry points of libp2p_hip.so (declared in include/p2p_hip.h).
// Validation happens here, before anything is launched: a rejected call returns a negative
// P2P_E_* code and touches nothing.
#include <stdlib.h>

#include "p2p_kernels.h"

using namespace p2p;

namespace {

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

int check_tensors(const p2p_attn_tensors* t, bool need_q, bool need_k, bool need_v, bool need_o) {
  if (!t) return P2P_E_ARG;
  if ((need_q && !t->q) || (need_k && !t->k) || (need_v && !t->v) || (need_o && !t->o)) return P2P_E_ARG;
  if (t->n_batch < 1 || t->n_query < 1 || t->n_key < 1 || t->n_heads < 1 || t->head_dim < 8) return P2P_E_ARG;
  if (t->n_batch > P2P_MAX_BATCH) return P2P_E_BATCH;
  if (t->head_dim % 8) return P2P_E_HEAD_DIM;
  if (t->io_dtype != P2P_DTYPE_F32 && t->io_dtype != P2P_DTYPE_BF16) return P2P_E_DTYPE;
  if (t->compute != P2P_COMPUTE_BF16 && t->compute != P2P_COMPUTE_F32) return P2P_E_DTYPE;
  const int es = t->io_dtype == P2P_DTYPE_F32 ? 4 : 2;
  // 16-byte vector loads of 8-element chunks need every row/head offset 8-element aligned
  const int64_t strides[8] = {t->q_row_stride, t->k_row_stride, t->v_row_stride, t->o_row_stride,
                              t->q_batch_stride, t->k_batch_stride, t->v_batch_stride, t->o_batch_stride};
  for (int i = 0; i < 8; ++i)
    if ((strides[i] * es) % 16) return P2P_E_ALIGN;
  if ((need_q && !aligned16(t->q)) || (need_k && !aligned16(t->k)) || (need_v && !aligned16(t->v)) ||
      (need_o && !aligned16(t->o)))
    return P2P_E_ALIGN;
  return 0;
}

void no_maps(SelfArgs& a) { a.n_maps = 0; }
void no_maps(CrossArgs&) {}

template <typename A>
void fill_common(A& a, const p2p_attn_tensors* t) {
  a.q = t->q; a.k = t->k; a.v = t->v; a.o = t->o;
  a.ldq = t->q_row_stride; a.ldk = t->k_row_stride; a.ldv = t->v_row_stride; a.ldo = t->o_row_stride;
  a.bsq = t->q_batch_stride; a.bsk = t->k_batch_stride; a.bsv = t->v_batch_stride; a.bso = t->o_batch_stride;
  a.N = t->n_batch; a.P = t->n_query; a.K = t->n_key; a.H = t->n_heads;
  a.scale_log2 = t->scale * 1.4426950408889634f;
  a.n_qtiles = 0;
  a.store = nullptr;
  a.store_accumulate = 0;
  no_maps(a);
}

// Kernel variants for A/B timing (tools/self_variants.py): honoured only by a library built with
// `make EXPERIMENTS=1`, and read once at load -- a production library always runs the default
// kernels whatever the environment says.
#ifdef P2P_EXPERIMENTS
const int kSelfVariant = [] {
  const char* e = getenv("P2P_SELF_VARIANT");
  return e ? atoi(e) : 0;
}();
#else
constexpr int kSelfVariant = 0;
#endif
int self_variant() { return kSelfVariant; }

#ifndef P2P_SOURCE_HASH
#define P2P_SOURCE_HASH "unstamped"
#endif

}  // namespace

namespace p2p {
LaunchEvents& launch_events() {
  static thread_local LaunchEvents ev;
  return ev;
}
}  // namespace p2p

extern "C" {

int p2p_set_launch_events(void* start, void* stop) {
  LaunchEvents& ev = launch_events();
  ev.start = static_cast<hipEvent_t>(start);
  ev.stop = static_cast<hipEvent_t>(stop);
  return 0;
}

int p2p_abi_version(void) { return P2P_ABI_VERSION; }

const char* p2p_source_hash(void) { return P2P_SOURCE_HASH; }

const char* p2p_error_string(int code) {
  switch (code) {
    case 0: return "ok";
    case P2P_E_ARG: return "invalid argument";
    case P2P_E_HEAD_DIM: return "head_dim has no compiled kernel";
    case P2P_E_DTYPE: return "unsupported io_dtype/compute combination";
    case P2P_E_KEYS: return "n_key above P2P_MAX_KEYS_CROSS";
    case P2P_E_BATCH: return "batch / group list out of range";
    case P2P_E_ALIGN: return "pointer or stride breaks 16-byte alignment";
    default: return code > 0 ? hipGetErrorString((hipError_t)code) : "unknown error";
  }
}

int p2p_self_attn_fwd(const p2p_attn_tensors* t, const int32_t* qk_src, float* store, const int32_t* store_slot,
                      int32_t store_accumulate, float* lse_workspace, p2p_stream_t stream) {
  int rc = check_tensors(t, true, true, true, true);
  if (rc) return rc;
  SelfArgs a;
  fill_common(a, t);
  a.variant = self_variant();
  a.lse = nullptr;
  a.probs = nullptr;
  a.key_mask = nullptr;
  for (int n = 0; n < t->n_batch; ++n) {
    a.qk_src[n] = qk_src ? qk_src[n] : n;
    if (a.qk_src[n] < 0 || a.qk_src[n] >= t->n_batch) return P2P_E_BATCH;
    a.store_slot[n] = (store && store_slot) ? store_slot[n] : -1;
    if (a.store_slot[n] >= 0) a.map_entry[a.n_maps++] = n;
  }
  if (a.n_maps > 0) {
    if (!lse_workspace) return P2P_E_ARG;
    if (!aligned16(store) || !aligned16(lse_workspace)) return P2P_E_ALIGN;
    a.store = store;
    a.store_accumulate = store_accumulate ? 1 : 0;
    a.lse = lse_workspace;
  }
  // O (and, when maps are kept, every row's lse) in one fused pass; then the stored maps
  rc = run_self(a, t->io_dtype, t->compute, t->head_dim, MODE_FUSED_, (hipStream_t)stream);
  if (rc || a.n_maps == 0) return rc;
  return run_self_maps(a, t->io_dtype, t->compute, t->head_dim, (hipStream_t)stream);
}

int p2p_cross_attn_fwd(const p2p_attn_tensors* t, const p2p_group* groups, int32_t n_groups, float* store,
                       const int32_t* store_slot, int32_t store_accumulate, p2p_stream_t stream) {
  int rc = check_tensors(t, true, true, true, true);
  if (rc) return rc;
  if (t->n_key > P2P_MAX_KEYS_CROSS) return P2P_E_KEYS;
  if (!groups || n_groups < 1 || n_groups > P2P_MAX_GROUPS) return P2P_E_BATCH;
  CrossArgs a;
  a.variant = self_variant();
  fill_common(a, t);
  int covered = 0;
  for (int n = 0; n < t->n_batch; ++n) a.ent_group[n] = -1;
  for (int g = 0; g < n_groups; ++g) {
    const p2p_group& G = groups[g];
    if (G.first < 0 || G.count < 1 || G.first + G.count > t->n_batch) return P2P_E_BATCH;
    if (G.program && G.count > 1 && !G.alpha) return P2P_E_ARG;
    // the kernel reads edit record / dense tile / alpha row b - 1 for b < count: a program built
    // for fewer edits than the group has would be read past its end
    if (G.program && G.count - 1 > G.n_edits) return P2P_E_BATCH;
    a.grp_first[g] = G.first;
    a.grp_count[g] = G.count;
    a.grp_prog[g] = G.program;
    // dense tiles follow the header and the n_edits records (programs.py layout)
    a.grp_dense[g] = (G.program && (G.flags & P2P_PROGRAM_F_DENSE))
                         ? static_cast<const char*>(G.program) + P2P_PROGRAM_HEADER_BYTES +
                               (int64_t)G.n_edits * P2P_PROGRAM_REC_BYTES
                         : nullptr;
    a.grp_alpha[g] = G.alpha;
    a.grp_flags[g] = G.program ? G.flags : (G.flags & P2P_GROUP_F_SHARED_KV);
    a.grp_bsum[g] = G.blend_sums;
    a.grp_balpha[g] = G.blend_alpha;
    a.grp_bsub[g] = G.blend_sub;
    a.grp_bcol[g] = G.blend_col;
    a.grp_blh[g] = G.blend_lh;
    if (G.blend_sums && (!G.blend_alpha || G.blend_lh < 1 || G.blend_col < 0 ||
                         G.blend_col + t->n_heads > G.blend_lh))
      return P2P_E_ARG;
    for (int e = G.first; e < G.first + G.count; ++e) {
      if (a.ent_group[e] >= 0) return P2P_E_BATCH;  // groups overlap
      a.ent_group[e] = g;
    }
    covered += G.count;
  }
  if (covered != t->n_batch) return P2P_E_BATCH;
  a.n_groups = n_groups;
  bool any_store = false;
  for (int n = 0; n < t->n_batch; ++n) {
    a.store_slot[n] = (store && store_slot) ? store_slot[n] : -1;
    any_store |= a.store_slot[n] >= 0;
  }
  // folded LocalBlend sums ride on the store epilogue: every entry of such a group must store
  for (int g = 0; g < n_groups; ++g)
    if (groups[g].blend_sums)
      for (int e = groups[g].first; e < groups[g].first + groups[g].count; ++e)
        if (a.store_slot[e] < 0) return P2P_E_ARG;
  for (int n = 0; n < t->n_batch; ++n) {
    const int g = a.ent_group[n];
    const int b = n - a.grp_first[g];
    const bool edit = a.grp_prog[g] != nullptr && b > 0;
    const bool r_only = edit && (a.grp_flags[g] & P2P_PROGRAM_F_DENSE) && (a.grp_flags[g] & P2P_GROUP_F_R_ONLY);
    a.ent_info[n] = g | (b << 8) | (edit ? 1 << 16 : 0) | (a.store_slot[n] >= 0 ? 1 << 17 : 0) |
                    (r_only ? 1 << 18 : 0);
  }
  a.store = any_store ? store : nullptr;
  a.store_accumulate = store_accumulate ? 1 : 0;
  a.any_store = any_store ? 1 : 0;
  a.edit_terms = a.edit_dense = 0;
  for (int g = 0; g < n_groups; ++g)
    if (groups[g].program && groups[g].count > 1) {
      if (groups[g].flags & P2P_PROGRAM_F_DENSE) a.edit_dense = 1;
      else a.edit_terms = 1;
    }
  return run_cross(a, t->io_dtype, t->compute, t->head_dim, (hipStream_t)stream);
}

int p2p_attn_probs(const p2p_attn_tensors* t, const uint8_t* key_mask, float* probs, p2p_stream_t stream) {
  int rc = check_tensors(t, true, true, false, false);
  if (rc) return rc;
  if (!probs) return P2P_E_ARG;
  SelfArgs a;
  fill_common(a, t);
  a.variant = self_variant();
  a.lse = nullptr;
  a.probs = nullptr;
  a.key_mask = key_mask;
  a.store = probs;
  a.store_accumulate = 0;
  for (int n = 0; n < t->n_batch; ++n) {
    a.qk_src[n] = n;
    a.store_slot[n] = n * t->n_heads;
  }
  return run_self_probs(a, t->io_dtype, t->compute, t->head_dim, (hipStream_t)stream);
}

int p2p_attn_pv(const p2p_attn_tensors* t, const float* probs, p2p_stream_t stream) {
  int rc = check_tensors(t, false, false, true, true);
  if (rc) return rc;
  if (!probs) return P2P_E_ARG;
  SelfArgs a;
  fill_common(a, t);
  a.variant = 0;
  a.lse = nullptr;
  a.probs = probs;
  a.key_mask = nullptr;
  for (int n = 0; n < t->n_batch; ++n) {
    a.qk_src[n] = n;
    a.store_slot[n] = -1;
  }
  return run_self(a, t->io_dtype, t->compute, t->head_dim, MODE_PV_, (hipStream_t)stream);
}

int p2p_localblend(const p2p_blend_args* a, p2p_stream_t stream) {
  if (!a) return P2P_E_ARG;
  return run_localblend(*a, (hipStream_t)stream);
}

int p2p_attn_fwd_lse(const p2p_attn_tensors* t, float* lse, p2p_stream_t stream) {
  int rc = check_tensors(t, true, true, true, true);
  if (rc) return rc;
  if (!lse) return P2P_E_ARG;
  if (t->compute != P2P_COMPUTE_BF16) return P2P_E_DTYPE;
  SelfArgs a;
  fill_common(a, t);
  a.variant = 0;
  a.lse = lse;
  a.probs = nullptr;
  a.key_mask = nullptr;
  for (int n = 0; n < t->n_batch; ++n) {
    a.qk_src[n] = n;
    a.store_slot[n] = -1;
  }
  return run_self(a, t->io_dtype, t->compute, t->head_dim, MODE_FUSED_, (hipStream_t)stream);
}

int64_t p2p_attn_bwd_workspace(const p2p_attn_tensors* t) {
  if (!t || t->n_batch < 1 || t->n_query < 1 || t->n_key < 1 || t->n_heads < 1 || t->head_dim < 1) return 0;
  const int split = bwd_kv_split(t->n_batch, t->n_heads, t->n_query, t->n_key, t->head_dim);
  if (split <= 1) return 0;
  return (int64_t)2 * split * t->n_batch * t->n_key * t->n_heads * t->head_dim * (int64_t)sizeof(float);
}

int p2p_attn_bwd(const p2p_attn_tensors* t, const void* dout, const float* lse, float* delta, void* dq,
                 void* dk, void* dv, int32_t kv_f32, void* workspace, int64_t workspace_bytes,
                 p2p_stream_t stream) {
  int rc = check_tensors(t, true, true, true, true);
  if (rc) return rc;
  if (!dout || !lse || !delta || !dq || !dk || !dv) return P2P_E_ARG;
  const int64_t need = p2p_attn_bwd_workspace(t);
  if (need > 0 && (!workspace || workspace_bytes < need)) return P2P_E_ARG;
  if (need > 0 && !aligned16(workspace)) return P2P_E_ALIGN;
  if (t->compute != P2P_COMPUTE_BF16) return P2P_E_DTYPE;
  if (!aligned16(dout) || !aligned16(dq) || !aligned16(dk) || !aligned16(dv)) return P2P_E_ALIGN;
  BwdArgs a;
  a.q = t->q; a.k = t->k; a.v = t->v; a.o = t->o; a.dout = dout;
  a.dq = dq; a.dk = dk; a.dv = dv; a.lse = lse; a.delta = delta;
  // dout / dq share q's layout, dk / dv are packed [N, K, H*d]
  a.ldq = t->q_row_stride; a.ldk = t->k_row_stride; a.ldv = t->v_row_stride; a.ldo = t->o_row_stride;
  a.lddo = t->o_row_stride; a.lddq = t->q_row_stride;
  a.bsq = t->q_batch_stride; a.bsk = t->k_batch_stride; a.bsv = t->v_batch_stride; a.bso = t->o_batch_stride;
  a.bsdo = t->o_batch_stride; a.bsdq = t->q_batch_stride;
  const int64_t C = (int64_t)t->n_heads * t->head_dim;
  a.lddk = a.lddv = C;
  a.bsdk = a.bsdv = C * t->n_key;
  a.N = t->n_batch; a.P = t->n_query; a.K = t->n_key; a.H = t->n_heads;
  a.scale = t->scale;
  a.scale_log2 = t->scale * 1.4426950408889634f;
  a.n_tiles = 0;
  a.kv_split = 1;
  a.kv_f32 = kv_f32 ? 1 : 0;
  a.ws = need > 0 ? static_cast<float*>(workspace) : nullptr;
  return run_attn_bwd(a, t->io_dtype, t->head_dim, (hipStream_t)stream);
}

int p2p_latent_step(const p2p_latent_step_args* a, p2p_stream_t stream) {
  if (!a) return P2P_E_ARG;
  return run_latent_step(*a, (hipStream_t)stream);
}

int p2p_store_scale(const float* src, float* dst, float divisor, int64_t n, p2p_stream_t stream) {
  if (!src || !dst) return P2P_E_ARG;
  return run_store_scale(src, dst, divisor, n, (hipStream_t)stream);
}

int p2p_clock_probe(uint64_t* out, int32_t n_workgroups, int32_t ticks, p2p_stream_t stream) {
  if (!out || n_workgroups < 1 || n_workgroups > 1024 || ticks < 1 || ticks > 1000000) return P2P_E_ARG;
  return run_clock_probe(reinterpret_cast<unsigned long long*>(out), n_workgroups, ticks, (hipStream_t)stream);
}

}  // extern "C"
