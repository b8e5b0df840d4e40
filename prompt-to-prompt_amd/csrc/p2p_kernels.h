// Kernel-argument structs shared by the kernels and the C-ABI shim (passed by value).
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/p2p_hip.h"

namespace p2p {

// Kernel timing events of the calling thread (p2p_set_launch_events, ABI 15; measurement only):
// while set, launches go through hipExtLaunchKernel, which records the events from the kernel's own
// dispatch -- the first kernel of a C-ABI call takes `start`, every kernel takes `stop` (the last
// one's stands) -- instead of extra marker packets queued around the call.
struct LaunchEvents {
  hipEvent_t start = nullptr, stop = nullptr;
};
LaunchEvents& launch_events();

template <typename F, typename... Args>
inline void launch_kernel(F kernel, const dim3& grid, const dim3& block, uint32_t shmem, hipStream_t st,
                          Args... args) {
  LaunchEvents& ev = launch_events();
  if (!ev.start && !ev.stop) {
    hipLaunchKernelGGL(kernel, grid, block, shmem, st, args...);
    return;
  }
  hipEvent_t start = ev.start;
  ev.start = nullptr;
  hipExtLaunchKernelGGL(kernel, grid, block, shmem, st, start, ev.stop, 0u, args...);
}

struct SelfArgs {
  const void* q;
  const void* k;
  const void* v;
  void* o;
  int64_t ldq, ldk, ldv, ldo;  // token strides (elements)
  int64_t bsq, bsk, bsv, bso;  // batch strides (elements)
  int N, P, K, H;
  float scale_log2;            // CrossAttention.scale * log2(e)
  int n_qtiles;
  float* store;                // AttentionStore maps [*, P, K] (or materialised probs)
  const float* probs;          // MODE_PV input [N*H, P, K]
  const uint8_t* key_mask;     // optional [N, K]
  int store_accumulate;
  int variant;                 // fused-kernel tile shape (P2P_SELF_VARIANT, timing experiments)
  float* lse;                  // optional [N*H, P] row log-sum-exp output (fused mode, autograd)
  int qk_src[P2P_MAX_BATCH];
  int store_slot[P2P_MAX_BATCH];
  int n_maps;                  // self_maps_kernel: entries in map_entry
  int map_entry[P2P_MAX_BATCH];  // self_maps_kernel: the stored entries (store_slot >= 0)
};

struct CrossArgs {
  const void* q;
  const void* k;
  const void* v;
  void* o;
  int64_t ldq, ldk, ldv, ldo;
  int64_t bsq, bsk, bsv, bso;
  int N, P, K, H;
  float scale_log2;
  int n_qtiles;
  int n_groups;                  // prompt groups (grp_* entries)
  float* store;
  int store_accumulate;
  int any_store;                 // some entry stores its maps
  int edit_terms;                // some group edits through the term planes (LDS gather)
  int edit_dense;                // some group carries the dense f16 mapper tile
  int slab;                      // launcher-filled: the launch allocates the LDS slab
  int slab_stride;               // launcher-filled
  int variant;                   // launch-shape experiments (P2P_SELF_VARIANT, experiments build only)
  int store_slot[P2P_MAX_BATCH];
  int ent_group[P2P_MAX_BATCH];  // prompt group of every batch entry
  // per entry, packed so ONE kernel-argument load after n decides the path: group (bits 0-7),
  // position in the group (8-15), edits (16), keeps its maps (17), dense edit whose group is
  // flagged P2P_GROUP_F_R_ONLY (18)
  int ent_info[P2P_MAX_BATCH];
  int grp_first[P2P_MAX_GROUPS];
  int grp_count[P2P_MAX_GROUPS];
  const void* grp_prog[P2P_MAX_GROUPS];
  const void* grp_dense[P2P_MAX_GROUPS];   // the program's dense f16 tiles (host-computed offset)
  const float* grp_alpha[P2P_MAX_GROUPS];
  int grp_flags[P2P_MAX_GROUPS];
  float* grp_bsum[P2P_MAX_GROUPS];         // LocalBlend word sums (p2p_group.blend_*)
  const float* grp_balpha[P2P_MAX_GROUPS];
  const float* grp_bsub[P2P_MAX_GROUPS];
  int grp_bcol[P2P_MAX_GROUPS];
  int grp_blh[P2P_MAX_GROUPS];
};

enum { MODE_FUSED_ = 0, MODE_PV_ = 3 };

int run_self(const SelfArgs& a, int io_dtype, int compute, int d, int mode, hipStream_t st);
// AttentionStore epilogue of the self layers whose maps are kept: p = exp2(c s - lse) for the
// entries a.map_entry[0 .. n_maps) (a.lse filled by a preceding MODE_FUSED launch)
int run_self_maps(const SelfArgs& a, int io_dtype, int compute, int d, hipStream_t st);
// materialise protocol: probs (a.store) [N*H, P, K] = softmax(Q K^T * scale), optional key mask
int run_self_probs(const SelfArgs& a, int io_dtype, int compute, int d, hipStream_t st);
int run_cross(const CrossArgs& a, int io_dtype, int compute, int d, hipStream_t st);
// group-coupled cross-attention (p2p_cross.hip): bf16 inputs and compute, dense or no programs
bool cross_group_eligible(const CrossArgs& a, int d);
int run_cross_group(const CrossArgs& a, int d, hipStream_t st);
// d = 40 / 80 self-attention with bf16 inputs, O only (p2p_self40.hip): the G1/G7 and G2/G6
// production kernels
bool self40_eligible(const SelfArgs& a, int d);
int run_self40(const SelfArgs& a, int d, hipStream_t st);
// d = 160 self-attention with bf16 inputs, O only, K <= 256 (p2p_selfsplit.hip): key-split waves
bool self_split_eligible(const SelfArgs& a, int d);
int run_self_split(const SelfArgs& a, int d, hipStream_t st);
// d = 160 self-attention with bf16 inputs, O only, K > 128: 4-stage global_load_lds ring
bool self_ring_eligible(const SelfArgs& a, int d);
int run_self_ring(const SelfArgs& a, int d, hipStream_t st);
int run_localblend(const p2p_blend_args& a, hipStream_t st);
int run_latent_step(const p2p_latent_step_args& a, hipStream_t st);

// attention backward (p2p_bwd.hip)
struct BwdArgs {
  const void *q, *k, *v, *o, *dout;
  void *dq, *dk, *dv;          // dq in IO dtype; dk/dv f32 accumulators when kv_split > 1 else IO dtype
  const float* lse;            // [N*H, P] from the forward
  float* delta;                // workspace [N*H, P]
  int64_t ldq, ldk, ldv, ldo, lddo, lddq, lddk, lddv;   // token strides (elements)
  int64_t bsq, bsk, bsv, bso, bsdo, bsdq, bsdk, bsdv;   // batch strides (elements)
  int N, P, K, H;
  float scale, scale_log2;
  int n_tiles;                 // launcher-filled
  int kv_split;                // query splits of the dK/dV pass (>1: partials in ws, then a reduction)
  int kv_f32;                  // dk/dv are f32 buffers
  float* ws;                   // [2 (dK, dV)][kv_split][N][K][H*D] f32 partials when kv_split > 1
};
int run_attn_bwd(const BwdArgs& a, int io_dtype, int d, hipStream_t st);
int bwd_kv_split(int N, int H, int P, int K, int d);   // launcher's query split (workspace sizing)
int run_store_scale(const float* src, float* dst, float divisor, int64_t n, hipStream_t st);
int run_clock_probe(unsigned long long* out, int n_wg, int ticks, hipStream_t st);

}  // namespace p2p
