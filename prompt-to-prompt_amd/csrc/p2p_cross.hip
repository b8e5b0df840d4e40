// Group-coupled cross-attention (K <= 96 text tokens): the production kernel for bf16 inputs.
//
// One workgroup = one prompt group x one head x one query tile of 32 W rows (wave w owns 32 of
// them).  The workgroup walks the group's entries in order -- the source prompt first, then its
// edits (main.py:185-193: every edit row is formed against attn_base = attn[0] of the SAME rows)
// -- so the source's exact softmax P0 is computed ONCE per query tile and kept in registers (f16,
// the dense-edit MFMA's operand) for the edits that follow.  Entries are software-pipelined: the
// next entry's K, V, mapper tile, per-column coefficients and Q rows are loaded into registers
// while the current entry computes, and written to the (single) LDS images between two barriers,
// so after the workgroup's first round trip no entry waits on global memory.  Uncond groups take
// the same loop without a program (plain entries).
//
// Per entry e of the group, rows p of this wave (S^T convention of p2p_device.h: query on the
// lane, 16 keys in the accumulator registers):
//   P_e  = softmax(c * K_e Q_e^T)                               (exact, f32, keys >= K masked)
//   R    = P0 . M_e                                           (edits: one f16 MFMA pass, M_e the
//                                                              dense f16 mapper of the program)
//   P_e' = P_e * A_e[w] + R * B_e[w]                            (A = alpha post c_rep + 1 - alpha,
//                                                              B = alpha post; host program terms)
//   store: running sum [slot + h][p][w] (+)= P_e' (the wave's LDS slab makes whole 128-byte rows)
//          and LocalBlend's word sums of the row (word order, as blend_wordsum_kernel)
//   O_e  = P_e' V_e
// Numerics equal the per-entry kernel's edit path (cross_attn_kernel in p2p_attn.hip).
#include "p2p_device.h"
#include "p2p_kernels.h"

namespace p2p {
namespace {

typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_t;

#ifdef P2P_EXPERIMENTS
// diagnostic clock stamps (experiments build, P2P_SELF_VARIANT 123): [logical workgroup < 2048]
// [wave < 4][slot < 24]; read back by p2p_diag_group_stamps (tools/group_stamps.py)
__device__ unsigned long long g_group_stamps[2048 * 4 * 24];
#define P2P_GROUP_STAMP(i)                                                                         \
  if (a.variant == 123 && logical < 2048 && wave < 4 && lane == 0 && (i) < 24)                     \
    g_group_stamps[(logical * 4 + wave) * 24 + (i)] = __builtin_amdgcn_s_memtime();
#else
#define P2P_GROUP_STAMP(i) do { } while (0);
#endif

// two workgroups per CU (<= 256 VGPRs) where the state fits without spills: d = 40 unless it both
// edits and stores, d = 80 plain; the others take one (their grids are <= 128 workgroups anyway)
template <int D, int W, bool EDIT, bool STORE>
constexpr int group_occupancy() {
  if (W >= 8) return 1;   // 8 waves: two per SIMD already
  return (D <= 40 && !(EDIT && STORE)) || (D <= 80 && !EDIT && !STORE) ? 2 : 1;
}

template <int D, int W, bool EDIT, bool STORE>
__global__ __launch_bounds__(64 * W, (group_occupancy<D, W, EDIT, STORE>())) void cross_group_kernel(CrossArgs a) {
  constexpr bool kMaskCol = (D + 15) / 16 * 16 > D;   // K column D carries the key mask
  constexpr int DK = (D + 15) / 16 * 16;
  constexpr int DV = (D + 31) / 32 * 32;
  constexpr int NKT = DK / 16;
  constexpr int NDT = DV / 32;
  constexpr int KB = P2P_MAX_KEYS_CROSS / 32;
  constexpr int KR = KB * 32;
  constexpr int KS = KStride<DK, 2>::value;
  constexpr int VS = VStrideBf16<DV>::value;
  constexpr int MD = P2P_PROGRAM_DENSE;
  static_assert(MD == KR, "the mapper tile spans the key blocks");
  constexpr int NT = 64 * W;
  constexpr int CPR = D / 8;                       // 16-byte chunks per K / V row
  constexpr int NCH = (KR * CPR + NT - 1) / NT;    // K (and V) chunks per thread
  constexpr int MCPR = MD / 8;                     // 16-byte chunks per mapper row
  constexpr int NMC = (KR * MCPR + NT - 1) / NT;   // mapper chunks per thread
  __shared__ __attribute__((aligned(16))) uint16_t Ks[KR * KS];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[KR * VS];
  __shared__ __attribute__((aligned(16))) uint16_t Ms[EDIT ? MD * MD : 8];
  __shared__ __attribute__((aligned(16))) float coef[EDIT ? 2 * KR : 4];      // A | B of the entry
  __shared__ __attribute__((aligned(16))) float btab[STORE ? 2 * KR : 4];     // blend alpha | substruct
  extern __shared__ __attribute__((aligned(16))) char cross_dyn[];           // STORE: W x [32][K] f32
  // each wave's output rows on their way out (wave-private: no workgroup barrier)
  // Plain groups only.  Same-box rocprof (profiles/r05/ostore_ab/group/): plain steps 17.23 -> 15.77
  // us, but edit steps 19.29 -> 19.53 (the 12 KiB of rows beside the mapper tile), so the edit
  // instantiations keep the direct row-per-lane store, as does plain + store (at two workgroups
  // per CU the extra addressing spilled 6 VGPRs).
  constexpr bool kLdsOut = !EDIT && !STORE;
  constexpr int OS = D + 8;             // 16-byte aligned rows on distinct banks
  __shared__ __attribute__((aligned(16))) uint16_t Os[kLdsOut ? W * 32 * OS : 8];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int hh = lane >> 5;
  const int qi = lane & 31;

  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  P2P_GROUP_STAMP(0)
  // Work order: query tiles in blocks of 4; inside a block heads fastest (the 8 heads of one query
  // tile side by side on one XCD -- xcd_remap keeps consecutive logical ids together -- so the
  // 640-byte q / o rows they share move as whole lines), then the block's tiles, then the groups,
  // which alternate between the last (edit) and the first (uncond) ones: runs of 4 x H = 32
  // workgroups change group.  With groups slowest (round 3) whole XCDs ran only edit-group
  // workgroups (~20 % longer than plain ones, tools/group_stamps.py) and the others idled at the
  // end; runs of 32 also pair the two workgroups resident on a CU across kinds, as far as the
  // measurement tells: in the pipeline 22.9 -> 20.8 us at G1/G7 (runs of 8 tile-heads: 22.2;
  // profiles/r04/group_order_r04ac/)
  int qt, h, rest;
  {
    const int nfb = a.n_qtiles / 4;             // full blocks of 4 query tiles
    const int per_full = 4 * a.H * a.n_groups;
    if (logical < nfb * per_full) {
      const int t = logical - (logical / per_full) * per_full;
      h = t % a.H;
      const int u = t / a.H;
      qt = (logical / per_full) * 4 + (u & 3);
      rest = u >> 2;
    } else {                                    // the partial last block (n_qtiles % 4 tiles)
      const int r = a.n_qtiles - nfb * 4;
      const int t = logical - nfb * per_full;
      h = t % a.H;
      const int u = t / a.H;
      qt = nfb * 4 + u % r;
      rest = u / r;
    }
  }
  // rest 0, 1, 2, 3, ... -> groups G-1, 0, G-2, 1, ...: edit groups (last in the batch) and plain
  // ones alternate
  const int gi = (rest & 1) == 0 ? a.n_groups - 1 - (rest >> 1) : (rest >> 1);
  const int first = a.grp_first[gi];
  const int count = a.grp_count[gi];
  const char* const prog = static_cast<const char*>(a.grp_prog[gi]);
  const bool edits = EDIT && prog != nullptr && count > 1;
  const int K = a.K;
  const int P = a.P;
  const float c = a.scale_log2;
  // wave-uniform in a scalar register (the running-sum buffer resources built from it stay scalar:
  // from a VGPR each of their loads was a readfirstlane waterfall loop)
  const int p0w = __builtin_amdgcn_readfirstlane(qt * 32 * W + wave * 32);
  const int p = p0w + qi;
  const bool prow = p < P;
  float* const slab = reinterpret_cast<float*>(cross_dyn) + wave * 32 * K;
  const bool blend_on = STORE && a.grp_bsum[gi] != nullptr;
  // p2p_group.flags hints (include/p2p_hip.h), workgroup-uniform:
  //  * R_ONLY: every edit's blend reads only R = P0 M_e this call, so an edit entry needs its V
  //    but not its K and Q -- they are not loaded (a wrong hint reloads them after the entry's
  //    coefficients show it, below);
  //  * SHARED_KV: every entry of the group has the first entry's K and V (the uncond prompts ""):
  //    they are staged once, and a plain group then rewrites no LDS between its entries, so the
  //    barrier pair between entries goes too
  const int gflags = a.grp_flags[gi];
  const bool hint_r = EDIT && edits && (gflags & P2P_GROUP_F_R_ONLY) != 0;
  const bool shared_kv = (gflags & P2P_GROUP_F_SHARED_KV) != 0;
  const bool no_sync = shared_kv && !edits && !blend_on;
  // The mapper tile M_e (source word x target word, f16) is built in LDS from the program's term
  // planes (include/p2p_hip.h: plane t of column w = (source row, value), (0, 0) past the column's
  // last term) instead of copied from its 18 KiB dense image: the tile is zeroed once, then per
  // edit the thread of column w clears the previous edit's terms of its column and writes its own
  // -- the same f16 values at the same places as the dense image (a dense program's values are
  // exact in f16; a column's terms have distinct rows).  Two planes are prefetched with the entry;
  // a program whose columns gather more than two source words (tmax > 2, header int 2) copies the
  // dense image instead, loaded when it is written.
  const int tmax = edits ? __builtin_amdgcn_readfirstlane(reinterpret_cast<const int*>(prog)[2]) : 0;
  const bool terms2 = tmax <= 2;
  int2 tnew[2] = {{0, 0}, {0, 0}}, tprev[2] = {{0, 0}, {0, 0}};

  // ---- padding the MFMAs read and the staging never writes (written once; the staging writes
  // columns < D): K columns D..DK (met by Q's zero columns)
  // K column D carries the key mask: -2^100 (bf16 0xF180) on the rows past K, 0 below, met by a 1 in
  // every Q row's column D, so a masked key's logit leaves the MFMA at -2^100 (below any real logit,
  // exp -> 0 exactly) and no per-register compare is needed (the rows' columns < D are the zeros the
  // staging loads return)
  if constexpr (DK > D) {
    constexpr int PC = (DK - D) / 8;
    for (int i = tid; i < KR * PC; i += NT) {
      const int row = i / PC, j = i % PC;
      *reinterpret_cast<short8_t*>(Ks + row * KS + D + 8 * j) =
          short8_t{(short)(kMaskCol && j == 0 && row >= K ? 0xF180 : 0), 0, 0, 0, 0, 0, 0, 0};
    }
  }
  // (V and mapper rows K..KR: the staging writes the zeros its range-checked loads return; V
  // columns D+1..DV are only read into O^T rows > D, which are never stored).  V column D is 1 on
  // the K key rows and 0 past them, so O^T row D is the row sum of the bf16 weights P V used: the
  // plain entries take that sum instead of an f32 sum and a normalised P (the staging never
  // writes column D, so this holds for every entry)
  if constexpr (EDIT)
    if (edits)
      for (int i = tid; i < MD * MD / 8; i += NT) reinterpret_cast<short8_t*>(Ms)[i] = short8_t{};
  constexpr bool kOnesCol = DV > D;   // (d = 160, experiments builds only: no padding column)
  if constexpr (kOnesCol)
    for (int r = tid; r < KR; r += NT) Vs[r * VS + D] = r < K ? (uint16_t)0x3F80 : (uint16_t)0;

  // ---- the pipelined entry loads: K / V chunks, mapper chunks, coefficients, blend weights, Q
  short8_t kreg[NCH], vreg[NCH];
  float creg[3] = {0.f, 0.f, 0.f}, breg[2] = {0.f, 0.f};   // raw loads, used at LDS-write time
  short8_t qf[NKT];
  // Range-checked buffer loads throughout (zeros past the range): no per-chunk branches, so
  // the whole entry issues as one straight run of loads
  // the entry's K (own softmax), V and Q rows; rows >= K read as zeros (K rows are masked; V rows
  // past K must be zero), Q rows >= P as zeros (columns >= D are zeroed when consumed)
  auto load_k = [&](int e) __attribute__((always_inline)) {
    const char* kp = reinterpret_cast<const char*>(static_cast<const uint16_t*>(a.k) + (int64_t)e * a.bsk + h * D);
    const __amdgpu_buffer_rsrc_t rk = make_rsrc(kp, ((int64_t)(K - 1) * a.ldk + D) * 2);
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int cidx = tid + i * NT;
      const int row = cidx / CPR;
      const int ch = cidx - row * CPR;
      kreg[i] = __builtin_bit_cast(short8_t, __builtin_amdgcn_raw_buffer_load_b128(rk, (row * (int)a.ldk + ch * 8) * 2, 0, 0));
    }
  };
  auto load_q = [&](int e) __attribute__((always_inline)) {
    const char* qp = reinterpret_cast<const char*>(static_cast<const uint16_t*>(a.q) + (int64_t)e * a.bsq + h * D);
    const __amdgpu_buffer_rsrc_t rq = make_rsrc(qp, ((int64_t)(P - 1) * a.ldq + D) * 2);
#pragma unroll
    for (int t = 0; t < NKT; ++t)
      qf[t] = __builtin_bit_cast(short8_t, __builtin_amdgcn_raw_buffer_load_b128(rq, (p * (int)a.ldq + 16 * t + 8 * hh) * 2, 0, 0));
  };
  auto write_k = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int cidx = tid + i * NT;
      const int row = cidx / CPR;
      const int ch = cidx - row * CPR;
      if ((KR * CPR) % NT == 0 || cidx < KR * CPR) *reinterpret_cast<short8_t*>(Ks + row * KS + ch * 8) = kreg[i];
    }
  };
  // which of the entry's rows are staged (workgroup-uniform): K only where the entry's own
  // softmax can run, V unless the group shares the first entry's, Q only with its own softmax
  auto stage_k = [&](int b) { return !(b > 0 && (shared_kv || hint_r)); };
  auto stage_v = [&](int b) { return !(b > 0 && shared_kv); };
  auto stage_q = [&](int b) { return !(b > 0 && hint_r); };
  auto load_entry = [&](int b) __attribute__((always_inline)) {
    const int e = first + b;
    if (stage_k(b)) load_k(e);
    if (stage_v(b)) {
      const char* vp = reinterpret_cast<const char*>(static_cast<const uint16_t*>(a.v) + (int64_t)e * a.bsv + h * D);
      const __amdgpu_buffer_rsrc_t rv = make_rsrc(vp, ((int64_t)(K - 1) * a.ldv + D) * 2);
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        const int cidx = tid + i * NT;
        const int row = cidx / CPR;
        const int ch = cidx - row * CPR;
        vreg[i] = __builtin_bit_cast(short8_t, __builtin_amdgcn_raw_buffer_load_b128(rv, (row * (int)a.ldv + ch * 8) * 2, 0, 0));
      }
    }
    if (stage_q(b)) load_q(e);
    if constexpr (EDIT) {
      if (edits && b > 0) {
        const char* ce = prog + P2P_PROGRAM_HEADER_BYTES + (int64_t)(b - 1) * P2P_PROGRAM_REC_BYTES;
        // term planes 0 and 1 of column tid (columns >= K hold (0, 0); threads past the tile's
        // columns read nothing)
        const __amdgpu_buffer_rsrc_t rt = make_rsrc(ce + 2 * 4 * P2P_PROGRAM_COLS, terms2 ? 2 * 8 * P2P_PROGRAM_COLS : 0);
        const int toff = tid < MD ? tid * 8 : 1 << 30;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const auto v2 = __builtin_amdgcn_raw_buffer_load_b64(rt, toff + t * 8 * P2P_PROGRAM_COLS, 0, 0);
          tnew[t] = int2{(int)v2[0], (int)v2[1]};
        }
        // the column's alpha, c_rep and post (one column per thread, zeros past K); the
        // coefficients are formed at LDS-write time, so nothing here waits for these loads
        const __amdgpu_buffer_rsrc_t ra = make_rsrc(a.grp_alpha[gi] + (int64_t)(b - 1) * K, (int64_t)K * 4);
        const __amdgpu_buffer_rsrc_t rc = make_rsrc(ce, (int64_t)K * 4);
        const __amdgpu_buffer_rsrc_t rp = make_rsrc(ce + 4 * P2P_PROGRAM_COLS, (int64_t)K * 4);
        creg[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ra, tid * 4, 0, 0));
        creg[1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rc, tid * 4, 0, 0));
        creg[2] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rp, tid * 4, 0, 0));
      }
    }
    if constexpr (STORE) {
      if (blend_on) {
        const float* ta = a.grp_balpha[gi] + (int64_t)b * K;
        const float* tsub = a.grp_bsub[gi];
        breg[0] = tid < K ? ta[tid] : 0.f;
        breg[1] = (tid < K && tsub != nullptr) ? tsub[(int64_t)b * K + tid] : 0.f;
      }
    }
  };
  auto write_entry = [&](int b) __attribute__((always_inline)) {
    // every load of the entry (Q included, which is read only in the next iteration) retired
    // HERE: otherwise the loop header merges Q as pending and the next Q K^T waits with a vmcnt
    // that also drains the following entry's prefetch
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    if (stage_k(b)) write_k();   // rows past K are the zeros the loads returned
    if (stage_v(b)) {
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        const int cidx = tid + i * NT;
        const int row = cidx / CPR;
        const int ch = cidx - row * CPR;
        if ((KR * CPR) % NT == 0 || cidx < KR * CPR) *reinterpret_cast<short8_t*>(Vs + row * VS + ch * 8) = vreg[i];
      }
    }
    if constexpr (EDIT) {
      if (edits && b > 0) {
        if (terms2) {
          if (tid < MD) {
#pragma unroll
            for (int t = 0; t < 2; ++t)   // the previous edit's terms of this column
              if (tprev[t].y != 0 && (unsigned)tprev[t].x < (unsigned)MD) Ms[tprev[t].x * MD + tid] = 0;
#pragma unroll
            for (int t = 0; t < 2; ++t)
              if (tnew[t].y != 0 && (unsigned)tnew[t].x < (unsigned)MD)
                Ms[tnew[t].x * MD + tid] = __builtin_bit_cast(uint16_t, (_Float16)__int_as_float(tnew[t].y));
            tprev[0] = tnew[0];
            tprev[1] = tnew[1];
          }
        } else {
          // tmax > 2: the dense image (mapper rows >= K are zero in the program and never staged)
          const __amdgpu_buffer_rsrc_t rm = make_rsrc(static_cast<const uint16_t*>(a.grp_dense[gi]) + (int64_t)(b - 1) * MD * MD,
                                                      (int64_t)K * MCPR * 16);
#pragma unroll
          for (int j = 0; j < NMC; ++j) {
            const int i = tid + j * NT;
            const short8_t mc = __builtin_bit_cast(short8_t, __builtin_amdgcn_raw_buffer_load_b128(rm, i * 16, 0, 0));
            if ((KR * MCPR) % NT == 0 || i < KR * MCPR) reinterpret_cast<short8_t*>(Ms)[i] = mc;
          }
        }
        // P' = alpha post (c_rep P_b + R) + (1 - alpha) P_b = P_b A + R B; columns >= K: A = 1, B = 0
        if (tid < KR) {
          const float aw = creg[0];
          const float ap = aw * creg[2];
          const float A = tid < K ? fmaf(ap, creg[1], 1.f - aw) : 1.f;
          const float B = tid < K ? ap : 0.f;
          coef[tid] = A;
          coef[KR + tid] = B;
        }
      }
    }
    if constexpr (STORE) {
      if (blend_on && tid < KR) {
        btab[tid] = breg[0];
        btab[KR + tid] = breg[1];
      }
    }
  };
  static_assert(KR <= NT, "one column per thread");

  load_entry(0);
  write_entry(0);
  __syncthreads();
  P2P_GROUP_STAMP(1)

  short8_t p0h[EDIT ? KB : 1][2];   // the source's P0 in f16 (the R MFMA's B operand)
  const bool short_tail = K <= (KB - 1) * 32 + 16;   // registers 8..15 of the last block: keys >= 80

  // the blend halves an edit needs (bit 0: some A != 0 -> its own softmax; bit 1: some B != 0 ->
  // R).  A Replace step with alpha = 1 on every word (main.py:189, the first cross_replace_steps)
  // needs only R, one with alpha = 0 only its own P_b: dropping the other half is exact
  // (fma(P, 0, x) = x, fma(P, A, R * 0) = P A)
  int next_flags = 3;
  for (int b = 0; b < count; ++b) {
    const int e = first + b;
    const int eflags = next_flags;   // workgroup-uniform
    short8_t qc[NKT];   // this entry's Q rows (qf is refilled for the next entry below)
#pragma unroll
    for (int t = 0; t < NKT; ++t)   // columns >= D: 0, but column D = 1 (the key-mask column)
      qc[t] = (16 * t + 8 * hh < D) ? qf[t]
                                    : (kMaskCol && 16 * t + 8 * hh == D ? short8_t{0x3F80, 0, 0, 0, 0, 0, 0, 0} : short8_t{});
    const bool more = b + 1 < count;
    if (more) load_entry(b + 1);   // lands while this entry computes
    const bool stored = STORE && a.store_slot[e] >= 0;
    const int slot = stored ? a.store_slot[e] : 0;

    // running sum rows of this wave: touched into L2 now, consumed by the read-add-write below
    float touch0 = 0.f, touch1 = 0.f;
    if (STORE && stored && a.store_accumulate && prow) {
      const int rows = min(32, P - p0w);
      const float* g = a.store + ((int64_t)(slot + h) * P + p0w) * (int64_t)K;
      const int lines = (rows * K * 4 + 127) / 128;
      if (lane < lines) touch0 = g[lane * 32];
      if (lane + 64 < lines) touch1 = g[(lane + 64) * 32];
    }

    const bool is_edit = EDIT && edits && b > 0;
    const bool need_own = !is_edit || (eflags & 1);
    const bool need_r = is_edit && (eflags & 2);
    // a plain entry (no edit, not the source the edits read, maps not kept): unnormalised P
    // through P V, O scaled by 1 / (O^T row D) once (the per-entry kernel's lean path)
    const bool lean = kOnesCol && !is_edit && !(edits && b == 0) && !stored;

    // ---- P_e = softmax(c K_e Q_e^T), exact, f32 (an edit whose blend reads only R skips it)
    float sv[KB][16];
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) sv[kb][r] = 0.f;
    if (need_own) {
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      f32x16_t acc = {};
#pragma unroll
      for (int t = 0; t < NKT; ++t) {
        const short8_t kf = *reinterpret_cast<const short8_t*>(Ks + (kb * 32 + qi) * KS + 16 * t + 8 * hh);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, kf),
                                                      __builtin_bit_cast(bf16x8_t, qc[t]), acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) sv[kb][r] = acc[r];
      if (!kMaskCol && kb * 32 + 32 > K) {   // (no mask column) wave-uniform: only the block past K
        // K made opaque per entry: hoisted out of the entry loop, the 16 per-register lane masks
        // were spilled to VGPR lanes and each restored by two v_readlane (plus a hazard s_nop)
        int Kl = K - kb * 32;
        asm volatile("" : "+s"(Kl));
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (acc_row(r, hh) >= Kl) sv[kb][r] = -INFINITY;
      }
    }
    auto soft = [&](auto tail) __attribute__((always_inline)) {
      constexpr bool kShort = decltype(tail)::value;
      float mx = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (!(kShort && kb == KB - 1 && r >= 8)) mx = fmaxf(mx, sv[kb][r]);
      mx = fmaxf(mx, other_half(mx)) * c;
      if (lean) {
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            sv[kb][r] = (kShort && kb == KB - 1 && r >= 8) ? 0.f : fast_exp2(fmaf(sv[kb][r], c, -mx));
        return;
      }
      float ls = 0.f;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          if (kShort && kb == KB - 1 && r >= 8) {
            sv[kb][r] = 0.f;
          } else {
            const float ex = fast_exp2(fmaf(sv[kb][r], c, -mx));
            sv[kb][r] = ex;
            ls += ex;
          }
        }
      const float inv = 1.f / (ls + other_half(ls));
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (!(kShort && kb == KB - 1 && r >= 8)) sv[kb][r] *= inv;
    };
    if (short_tail) soft(std::true_type{});
    else soft(std::false_type{});
    }
    P2P_GROUP_STAMP(2 + 5 * b)

    if constexpr (EDIT) {
      if (edits && b == 0) {
        // keep the source's probabilities for the edits (f16: <= 2^-12 relative, as the
        // per-entry kernel's dense path rounds them)
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int r = 0; r < 8; ++r)
              p0h[kb][s2][r] = (short)__builtin_bit_cast(uint16_t, (_Float16)sv[kb][8 * s2 + r]);
      }
      if (is_edit && !need_r) {
        // B = 0 on every column: P' = fma(P_b, A, R * 0) = P_b A without R
#pragma unroll
        for (int dt = 0; dt < KB; ++dt)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4_t A4 = *reinterpret_cast<const f32x4_t*>(coef + dt * 32 + 8 * g + 4 * hh);
#pragma unroll
            for (int j = 0; j < 4; ++j) sv[dt][4 * g + j] *= A4[j];
          }
      }
      if (need_r) {
        // R = P0 . M_e on the f16 MFMA: three independent 32-word target blocks, each mapper
        // fragment read once; then P' = P_b A_w + R B_w (a lane's columns come in runs of 4: one
        // 16-byte read each)
        f32x16_t Rd[KB];
#pragma unroll
        for (int dt = 0; dt < KB; ++dt) Rd[dt] = f32x16_t{};
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int dt = 0; dt < KB; ++dt) {
              const MmaBf16::frag af = vt_frag<MD>(Ms, kb * 32, s2, dt * 32, lane);
              Rd[dt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, af.v),
                                                              __builtin_bit_cast(f16x8_t, p0h[kb][s2]), Rd[dt], 0, 0, 0);
            }
#pragma unroll
        for (int dt = 0; dt < KB; ++dt)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int w0 = dt * 32 + 8 * g + 4 * hh;
            const f32x4_t A4 = *reinterpret_cast<const f32x4_t*>(coef + w0);
            const f32x4_t B4 = *reinterpret_cast<const f32x4_t*>(coef + KR + w0);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int r = 4 * g + j;
              sv[dt][r] = fmaf(sv[dt][r], A4[j], Rd[dt][r] * B4[j]);
            }
          }
      }
    }

    P2P_GROUP_STAMP(3 + 5 * b)
    // ---- AttentionStore epilogue: the post-edit rows through this wave's slab (wave-private)
    if constexpr (STORE) {
      if (stored) {
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int w = kb * 32 + acc_row(r, hh);
            if (w < K) slab[qi * K + w] = sv[kb][r];
          }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int rows = min(32, P - p0w);
        if (blend_on && qi < rows) {
          // LocalBlend word sums of this row (lanes 0-31: alpha, 32-63: substruct), words in
          // index order as blend_wordsum_kernel sums them
          float acc = 0.f;
          if ((hh == 0 ? a.grp_balpha[gi] : a.grp_bsub[gi]) != nullptr) {
            const float* tab = btab + hh * KR;
            const float* row = slab + qi * K;
#pragma unroll 8
            for (int w = 0; w < K; ++w) acc += row[w] * tab[w];   // one sequential chain: the reads run ahead
          }
          float* dst = a.grp_bsum[gi] + ((int64_t)(b * 2 + hh) * a.grp_blh[gi] + a.grp_bcol[gi] + h) * P + p0w + qi;
          *dst = a.store_accumulate ? *dst + acc : acc;
        }
        if (rows > 0) {
          float* g = a.store + ((int64_t)(slot + h) * P + p0w) * (int64_t)K;
          const int cnt = rows * K;
          if (((uintptr_t)g & 15) == 0 && (cnt & 3) == 0) {
            store_rows_rmw<32 * KR / 4>(g, slab, cnt, a.store_accumulate != 0, lane);
            if (__builtin_expect(touch0 == -INFINITY || touch1 == -INFINITY, 0)) g[0] = touch0 + touch1;
          } else {
            for (int i = lane; i < cnt; i += 64) g[i] = a.store_accumulate ? g[i] + slab[i] : slab[i];
          }
        }
        // the slab is rewritten by the next stored entry: every lane's reads come first
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    }

    P2P_GROUP_STAMP(4 + 5 * b)
    // ---- O_e = P_e' V_e
    f32x16_t O[NDT];
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) O[dt] = f32x16_t{};
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) pv_block<VS, NDT>(MmaBf16{}, O, Vs, kb * 32, sv[kb], lane);
    // O^T row D (d tile D / 32, register kLr of lane half kLh): the row sum of a lean entry
    constexpr int kLrr = D % 32;
    constexpr int kLh = (kLrr >> 2) & 1;
    constexpr int kLr = (kLrr & 3) + 4 * (kLrr >> 3);
    const float inv = lean ? 1.f / __shfl(O[kOnesCol ? D / 32 : 0][kLr], (lane & 31) + 32 * kLh) : 1.f;
    // O out: the accumulator puts the query on the lane, so a direct store writes 32 rows x 8 bytes
    // per instruction; the wave's 32 rows go through its LDS rows instead and leave as whole
    // 16-byte row chunks, consecutive lanes along a row (the per-entry kernel's epilogue)
    const bool o16 = kLdsOut && (a.ldo & 7) == 0 && (a.bso & 7) == 0 && ((uintptr_t)a.o & 15) == 0;
    if (o16) {
      uint16_t* const orow = Os + wave * 32 * OS;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int dd = dt * 32 + 8 * g + 4 * hh;
          if (dd < D)
            store4(orow + qi * OS + dd, O[dt][4 * g] * inv, O[dt][4 * g + 1] * inv, O[dt][4 * g + 2] * inv,
                   O[dt][4 * g + 3] * inv);
        }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      uint16_t* const ob = static_cast<uint16_t*>(a.o) + (int64_t)e * a.bso + h * D;
#pragma unroll
      for (int c0 = 0; c0 < 32 * CPR; c0 += 64) {
        const int cidx = c0 + lane;
        const int row = cidx / CPR, ch = cidx - row * CPR;
        if (((32 * CPR) % 64 == 0 || cidx < 32 * CPR) && p0w + row < P)
          *reinterpret_cast<short8_t*>(ob + (int64_t)(p0w + row) * a.ldo + ch * 8) =
              *reinterpret_cast<const short8_t*>(orow + row * OS + ch * 8);
      }
      // the next entry rewrites these rows: every lane's reads first
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else if (prow) {
      uint16_t* const op = static_cast<uint16_t*>(a.o) + (int64_t)e * a.bso + h * D + (int64_t)p * a.ldo;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int dd = dt * 32 + 8 * g + 4 * hh;
          if (dd < D)
            store4(op + dd, O[dt][4 * g] * inv, O[dt][4 * g + 1] * inv, O[dt][4 * g + 2] * inv, O[dt][4 * g + 3] * inv);
        }
    }
    P2P_GROUP_STAMP(5 + 5 * b)
    if (more && no_sync) {
      // shared K / V, no program, no blend table: nothing in LDS changes for the next entry; its Q
      // rows retire here (as in write_entry), not in the next entry's first Q K^T
      __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    } else if (more) {
      __syncthreads();   // every wave is done with this entry's K, V, mapper and coefficients
      if (b == 1) {
        P2P_GROUP_STAMP(22)
      }
      write_entry(b + 1);
      if (b == 1) {
        P2P_GROUP_STAMP(23)
      }
      __syncthreads();
      if constexpr (EDIT) {
        // the blend halves the next edit uses, from its coefficients (every wave scans the row
        // itself: no extra barrier)
        if (edits) {
          const int c0 = lane, c1 = lane + 64;
          const bool a0 = c0 < K && coef[c0] != 0.f, a1 = c1 < K && coef[c1] != 0.f;
          const bool b0 = c0 < K && coef[KR + c0] != 0.f, b1 = c1 < K && coef[KR + c1] != 0.f;
          next_flags = (__any(a0 || a1) ? 1 : 0) | (__any(b0 || b1) ? 2 : 0);
          if (hint_r && (next_flags & 1)) {
            // a wrong R_ONLY hint (some A != 0): the next edit runs its own softmax after all, so
            // its K and Q rows come now (every wave reads the same coefficients: uniform branch)
            load_k(first + b + 1);
            load_q(first + b + 1);
            __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
            write_k();
            __syncthreads();
          }
        }
      }
    }
    P2P_GROUP_STAMP(6 + 5 * b)
  }
}

template <int D, int W>
hipError_t launch_group(const CrossArgs& a, hipStream_t st) {
  CrossArgs b = a;
  b.n_qtiles = (a.P + 32 * W - 1) / (32 * W);
  const bool edit = a.edit_dense != 0;
  const bool store = a.any_store != 0;
  const size_t dyn = store ? (size_t)W * 32 * a.K * sizeof(float) : 0;
  dim3 grid(b.n_qtiles * a.H * a.n_groups), block(64 * W);
  if (edit && store) launch_kernel((cross_group_kernel<D, W, true, true>), grid, block, dyn, st, b);
  else if (edit) launch_kernel((cross_group_kernel<D, W, true, false>), grid, block, dyn, st, b);
  else if (store) launch_kernel((cross_group_kernel<D, W, false, true>), grid, block, dyn, st, b);
  else launch_kernel((cross_group_kernel<D, W, false, false>), grid, block, dyn, st, b);
  return hipGetLastError();
}

}  // namespace

// bf16 inputs and compute (the caller checks), no term-plane (non-dense) programs, a compiled
// head dim; anything else -- or an experiments-build A/B selecting the per-entry kernel --
// launches cross_attn_kernel instead
// The workgroup walks the group's entries one after another, so it only pays where the grid
// still fills the chip: >= 2 workgroups per CU (G1/G7: 2 groups x 8 heads x 32 query tiles).
// Smaller grids (the 32x32 / 16x16 / 8x8 layers) keep the per-entry kernel's parallelism, and so
// do d = 80 / 160 at any size: with eight groups per U-Net call (configs[3], 1024 workgroups at
// G2/G6) the group kernel -- four entries with their map stores walked in sequence -- measured
// 228.5 us per launch against the per-entry kernel's 131.4 (profiles/r04/group_vs_entry_r04aj/);
// at d = 40 it stays ahead (146.9 vs 215.0 us).  (The d = 80 / 160 instantiations remain in the
// experiments build, variants 122 / 123.)
bool cross_group_eligible(const CrossArgs& a, int d) {
  if (a.edit_terms || a.K > P2P_MAX_KEYS_CROSS) return false;
  const int wgs = a.n_groups * a.H * ((a.P + 127) / 128);
#ifdef P2P_EXPERIMENTS
  if (a.variant == 123) return d == 40 || d == 80 || d == 160;   // clock stamps (tools/group_stamps.py)
#endif
  return d == 40 && wgs >= 512;
}

int run_cross_group(const CrossArgs& a, int d, hipStream_t st) {
  switch (d) {
#ifdef P2P_EXPERIMENTS
    case 40: return (int)launch_group<40, 4>(a, st);
    case 80: return (int)launch_group<80, 4>(a, st);
    case 160: return (int)launch_group<160, 4>(a, st);
#else
    case 40: return (int)launch_group<40, 4>(a, st);
#endif
    default: return P2P_E_HEAD_DIM;
  }
}

}  // namespace p2p

#ifdef P2P_EXPERIMENTS
// dst == nullptr: clear the stamps
extern "C" int p2p_diag_group_stamps(void* dst, int64_t bytes) {
  const int64_t n = (int64_t)sizeof(p2p::g_group_stamps);
  if (dst == nullptr) {
    void* p = nullptr;
    hipError_t e = hipGetSymbolAddress(&p, HIP_SYMBOL(p2p::g_group_stamps));
    return e != hipSuccess ? (int)e : (int)hipMemset(p, 0, n);
  }
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(p2p::g_group_stamps), bytes < n ? bytes : n, 0, hipMemcpyDeviceToHost);
}
#endif
