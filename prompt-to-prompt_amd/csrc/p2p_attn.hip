// Fused Prompt-to-Prompt attention kernels for MI355X (gfx950).
//
// self_attn_kernel  : flash-style self-attention (ptp_utils.py:183-208, context=None) with the
//                     source-map injection of AttentionControlEdit.replace_self_attention
//                     (main.py:169-174 / null_text.py:224-230) as a batch index remap, and the
//                     AttentionStore epilogue (main.py:129-142) for layers whose maps are kept.
// cross_attn_kernel : cross-attention over the 77 text tokens with the P2P cross edit
//                     (AttentionControlEdit.forward, main.py:180-197) applied in registers
//                     between the exact softmax and PV, for every prompt group.
//
// Both kernels follow the transposed-fragment convention of p2p_device.h: S^T = K Q^T and
// O^T = V^T P^T, query on the lane.
#include "p2p_device.h"
#include "p2p_kernels.h"

namespace p2p {

// ====================================================================== self attention
// MODE_FUSED : one online-softmax pass, O = softmax(S) V                        (no map kept)
// MODE_STORE : pass 1 row max/sum, pass 2 exact P -> store + PV                 (maps kept)
// MODE_PROBS : pass 1 + pass 2 writing P only                                   (materialise)
// MODE_PV    : O = P V with P read from HBM                                     (materialise)
enum { MODE_FUSED = 0, MODE_STORE = 1, MODE_PROBS = 2, MODE_PV = 3 };

template <typename IO, typename M, int D, int BK, int WAVES, int MODE>
__global__ __launch_bounds__(64 * WAVES) void self_attn_kernel(SelfArgs a) {
  using E = typename M::elem;
  constexpr int DK = (D + 15) / 16 * 16;
  constexpr int DV = (D + 31) / 32 * 32;
  constexpr int NKT = DK / 16;
  constexpr int NDT = DV / 32;
  constexpr int NSB = BK / 32;
  constexpr int KS = KStride<DK, M::kElemBytes>::value;
  constexpr int VS = (M::kElemBytes == 2) ? VStrideBf16<DV>::value : DV;
  constexpr int NT = 64 * WAVES;
  constexpr int CPR = D / 8;
  constexpr int NCH = (BK * CPR + NT - 1) / NT;
  constexpr bool kNeedK = MODE != MODE_PV;
  constexpr bool kNeedV = MODE == MODE_FUSED || MODE == MODE_STORE || MODE == MODE_PV;
  constexpr int KBUF = kNeedK ? 2 * BK * KS : 0;
  constexpr int VBUF = kNeedV ? 2 * BK * VS : 0;
  __shared__ __attribute__((aligned(16))) E smem[KBUF + VBUF + 8];
  E* const Ks = smem;
  E* const Vs = smem + KBUF;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int hh = lane >> 5;
  const int qi = lane & 31;

  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int qt = logical % a.n_qtiles;
  const int nh = logical / a.n_qtiles;
  const int h = nh % a.H;
  const int n = nh / a.H;
  const int src = a.qk_src[n];
  const int p = qt * 32 * WAVES + wave * 32 + qi;
  const bool prow = p < a.P;
  const int K = a.K;
  const float c = a.scale_log2;

  const IO* const qp = static_cast<const IO*>(a.q) + (int64_t)src * a.bsq + h * D;
  const IO* const kp = static_cast<const IO*>(a.k) + (int64_t)src * a.bsk + h * D;
  const IO* const vp = static_cast<const IO*>(a.v) + (int64_t)n * a.bsv + h * D;
  IO* const op = static_cast<IO*>(a.o) + (int64_t)n * a.bso + h * D;

  // zero the LDS image once: pad columns [D, DK) / [D, DV) and rows >= K stay zero.
  for (int i = tid; i < KBUF + VBUF; i += NT) smem[i] = E(0);

  // Q fragments stay in registers for the whole key loop.
  typename M::frag qf[NKT];
  if constexpr (kNeedK) {
#pragma unroll
    for (int t = 0; t < NKT; ++t) {
      const int col = 16 * t + 8 * hh;
      if (prow && col < D) {
        E tmp[8] __attribute__((aligned(16)));
        load8_global<IO, M>(qp + (int64_t)p * a.ldq + col, tmp);
        qf[t] = M::load8(tmp);
      } else {
        qf[t] = M::zero();
      }
    }
  }

  Chunk8<IO> kreg[NCH], vreg[NCH];
  auto stage_load = [&](int kt, bool withK, bool withV) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int cidx = tid + i * NT;
      const int row = cidx / CPR;
      const int ch = cidx - row * CPR;
      const int key = kt * BK + row;
      const bool ok = cidx < BK * CPR && key < K;
      if (withK) {
        if (ok) kreg[i].load(kp + (int64_t)key * a.ldk + ch * 8); else kreg[i].clear();
      }
      if (withV) {
        if (ok) vreg[i].load(vp + (int64_t)key * a.ldv + ch * 8); else vreg[i].clear();
      }
    }
  };
  auto stage_write = [&](int buf, bool withK, bool withV) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int cidx = tid + i * NT;
      if (cidx < BK * CPR) {
        const int row = cidx / CPR;
        const int ch = cidx - row * CPR;
        if (withK) kreg[i].store(Ks + buf * BK * KS + row * KS + ch * 8);
        if (withV) vreg[i].store(Vs + buf * BK * VS + row * VS + ch * 8);
      }
    }
  };

  // S^T block sb of the tile in buffer buf, masked beyond K (and by the optional key mask).
  auto scores = [&](int buf, int kt, float (&sv)[NSB][16]) {
    const E* Kb = Ks + buf * BK * KS;
#pragma unroll
    for (int sb = 0; sb < NSB; ++sb) {
      f32x16_t acc = {};
#pragma unroll
      for (int t = 0; t < NKT; ++t) {
        const typename M::frag fa = M::load8(Kb + (sb * 32 + qi) * KS + 16 * t + 8 * hh);
        M::mma(acc, fa, qf[t]);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) sv[sb][r] = acc[r];
    }
    if ((kt + 1) * BK > K || a.key_mask) {
#pragma unroll
      for (int sb = 0; sb < NSB; ++sb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kt * BK + sb * 32 + acc_row(r, hh);
          if (key >= K) sv[sb][r] = -INFINITY;
          else if (a.key_mask && !a.key_mask[(int64_t)((n * a.H + h) % a.N) * K + key])
            sv[sb][r] = -3.402823466e38f;
        }
    }
  };

  const int ntiles = (K + BK - 1) / BK;
  f32x16_t O[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) O[dt] = f32x16_t{};

  float m_run = -INFINITY, l_run = 0.f;

  if constexpr (MODE == MODE_FUSED) {
    __syncthreads();
    stage_load(0, true, true);
    stage_write(0, true, true);
    __syncthreads();
    for (int kt = 0; kt < ntiles; ++kt) {
      const int buf = kt & 1;
      if (kt + 1 < ntiles) stage_load(kt + 1, true, true);
      float sv[NSB][16];
      scores(buf, kt, sv);
      float mx = -INFINITY;
#pragma unroll
      for (int sb = 0; sb < NSB; ++sb)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sv[sb][r]);
      mx = fmaxf(mx, __shfl_xor(mx, 32));
      const float mnew = fmaxf(m_run, mx * c);
      const float alpha = fast_exp2(m_run - mnew);
      float ls = 0.f;
#pragma unroll
      for (int sb = 0; sb < NSB; ++sb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = fast_exp2(fmaf(sv[sb][r], c, -mnew));
          sv[sb][r] = e;
          ls += e;
        }
      l_run = fmaf(l_run, alpha, ls);
      m_run = mnew;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) O[dt][r] *= alpha;
      const E* Vb = Vs + buf * BK * VS;
#pragma unroll
      for (int sb = 0; sb < NSB; ++sb) pv_block<VS, NDT>(M{}, O, Vb, sb * 32, sv[sb], lane);
      if (kt + 1 < ntiles) stage_write(buf ^ 1, true, true);
      __syncthreads();
    }
    const float l = l_run + __shfl_xor(l_run, 32);
    const float inv = 1.f / l;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) O[dt][r] *= inv;
  } else if constexpr (MODE == MODE_STORE || MODE == MODE_PROBS) {
    // ---- pass 1: exact row max and row sum
    __syncthreads();
    stage_load(0, true, false);
    stage_write(0, true, false);
    __syncthreads();
    for (int kt = 0; kt < ntiles; ++kt) {
      const int buf = kt & 1;
      if (kt + 1 < ntiles) stage_load(kt + 1, true, false);
      float sv[NSB][16];
      scores(buf, kt, sv);
      float mx = -INFINITY;
#pragma unroll
      for (int sb = 0; sb < NSB; ++sb)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sv[sb][r]);
      mx = fmaxf(mx, __shfl_xor(mx, 32));
      const float mnew = fmaxf(m_run, mx * c);
      float ls = 0.f;
#pragma unroll
      for (int sb = 0; sb < NSB; ++sb)
#pragma unroll
        for (int r = 0; r < 16; ++r) ls += fast_exp2(fmaf(sv[sb][r], c, -mnew));
      l_run = fmaf(l_run, fast_exp2(m_run - mnew), ls);
      m_run = mnew;
      if (kt + 1 < ntiles) stage_write(buf ^ 1, true, false);
      __syncthreads();
    }
    const float inv = 1.f / (l_run + __shfl_xor(l_run, 32));
    // ---- pass 2: exact probabilities -> store (+ PV)
    constexpr bool kPV = MODE == MODE_STORE;
    const int slot = a.store_slot[n];
    float* const mp = (a.store && slot >= 0 && prow)
                          ? a.store + ((int64_t)(slot + h) * a.P + p) * (int64_t)K
                          : nullptr;
    const bool vec4 = (K & 3) == 0;
    stage_load(0, true, kPV);
    stage_write(0, true, kPV);
    __syncthreads();
    for (int kt = 0; kt < ntiles; ++kt) {
      const int buf = kt & 1;
      if (kt + 1 < ntiles) stage_load(kt + 1, true, kPV);
      float sv[NSB][16];
      scores(buf, kt, sv);
#pragma unroll
      for (int sb = 0; sb < NSB; ++sb)
#pragma unroll
        for (int r = 0; r < 16; ++r) sv[sb][r] = fast_exp2(fmaf(sv[sb][r], c, -m_run)) * inv;
      if (mp) {
#pragma unroll
        for (int sb = 0; sb < NSB; ++sb)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int key = kt * BK + sb * 32 + 8 * g + 4 * hh;
            if (vec4) {
              if (key < K) {
                f32x4_t v = {sv[sb][4 * g], sv[sb][4 * g + 1], sv[sb][4 * g + 2], sv[sb][4 * g + 3]};
                f32x4_t* dst = reinterpret_cast<f32x4_t*>(mp + key);
                if (a.store_accumulate) v += *dst;
                *dst = v;
              }
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e)
                if (key + e < K) {
                  const float v = sv[sb][4 * g + e];
                  mp[key + e] = a.store_accumulate ? mp[key + e] + v : v;
                }
            }
          }
      }
      if constexpr (kPV) {
        const E* Vb = Vs + buf * BK * VS;
#pragma unroll
        for (int sb = 0; sb < NSB; ++sb) pv_block<VS, NDT>(M{}, O, Vb, sb * 32, sv[sb], lane);
      }
      if (kt + 1 < ntiles) stage_write(buf ^ 1, true, kPV);
      __syncthreads();
    }
  } else {  // MODE_PV: O = P V with P from HBM (materialise mode)
    const float* const pp = a.probs + ((int64_t)(n * a.H + h) * a.P + (prow ? p : 0)) * (int64_t)K;
    __syncthreads();
    stage_load(0, false, true);
    stage_write(0, false, true);
    __syncthreads();
    for (int kt = 0; kt < ntiles; ++kt) {
      const int buf = kt & 1;
      if (kt + 1 < ntiles) stage_load(kt + 1, false, true);
      float sv[NSB][16];
#pragma unroll
      for (int sb = 0; sb < NSB; ++sb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kt * BK + sb * 32 + acc_row(r, hh);
          sv[sb][r] = (prow && key < K) ? pp[key] : 0.f;
        }
      const E* Vb = Vs + buf * BK * VS;
#pragma unroll
      for (int sb = 0; sb < NSB; ++sb) pv_block<VS, NDT>(M{}, O, Vb, sb * 32, sv[sb], lane);
      if (kt + 1 < ntiles) stage_write(buf ^ 1, false, true);
      __syncthreads();
    }
  }

  if constexpr (MODE != MODE_PROBS) {
    if (prow) {
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int dd = dt * 32 + 8 * g + 4 * hh;
          if (dd < D)
            store4(op + (int64_t)p * a.ldo + dd, O[dt][4 * g], O[dt][4 * g + 1], O[dt][4 * g + 2],
                   O[dt][4 * g + 3]);
        }
    }
  }
}

// ====================================================================== cross attention
// One workgroup = one head x one tile of 32*WAVES queries x one prompt group.  The group's
// prompts are processed in order; the source prompt's probabilities P0 are parked in LDS
// (one 32-row slab per wave) so each edit can gather from them:
//   R[w]  = post[w] * ( c_rep[w] * P_b[w] + sum_t val[t] * P0[rowidx[t]] ),  t in column w
//   P_b'  = alpha[w] * R[w] + (1 - alpha[w]) * P_b[w]
// which is AttentionReplace (c_rep 0, mapper column w), AttentionRefine (c_rep 1-a, one term
// mapper[w] with weight a), AttentionReweight (c_rep 0, term (w, eq[w])), and Reweight
// chained on either (post = eq) -- host side: p2p_amd/programs.py.
template <typename IO, typename M, int D, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void cross_attn_kernel(CrossArgs a) {
  using E = typename M::elem;
  constexpr int DK = (D + 15) / 16 * 16;
  constexpr int DV = (D + 31) / 32 * 32;
  constexpr int NKT = DK / 16;
  constexpr int NDT = DV / 32;
  constexpr int KB = P2P_MAX_KEYS_CROSS / 32;
  constexpr int KR = KB * 32;
  constexpr int KS = KStride<DK, M::kElemBytes>::value;
  constexpr int VS = (M::kElemBytes == 2) ? VStrideBf16<DV>::value : DV;
  constexpr int NT = 64 * WAVES;
  constexpr int CPR = D / 8;
  constexpr int P0S = KR + 1;  // odd f32 stride: 32 rows reading one column hit 32 banks
  constexpr int KBYTES = KR * KS * (int)sizeof(E);
  constexpr int VBYTES = KR * VS * (int)sizeof(E);
  constexpr int PBYTES = WAVES * 32 * P0S * 4;
  __shared__ __attribute__((aligned(16))) char smem[KBYTES + VBYTES + PBYTES];
  E* const Ks = reinterpret_cast<E*>(smem);
  E* const Vs = reinterpret_cast<E*>(smem + KBYTES);
  float* const P0 = reinterpret_cast<float*>(smem + KBYTES + VBYTES);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int hh = lane >> 5;
  const int qi = lane & 31;

  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int qt = logical % a.n_qtiles;
  const int rest = logical / a.n_qtiles;
  const int h = rest % a.H;
  const int gi = rest / a.H;
  const int first = a.grp_first[gi];
  const int count = a.grp_count[gi];
  const char* const prog = static_cast<const char*>(a.grp_prog[gi]);
  const float* const alpha = a.grp_alpha[gi];
  const int p = qt * 32 * WAVES + wave * 32 + qi;
  const bool prow = p < a.P;
  const int K = a.K;
  const float c = a.scale_log2;
  float* const P0w = P0 + wave * 32 * P0S + qi * P0S;

  for (int i = tid; i < (KBYTES + VBYTES) / 4; i += NT) reinterpret_cast<float*>(smem)[i] = 0.f;

  // edit program tables (P2P_PROGRAM_COLS-strided; see p2p_amd/programs.py)
  int n_edits = 0, nnz = 0;
  const float* crep = nullptr;
  const float* post = nullptr;
  const int* colptr = nullptr;
  const int* rowidx = nullptr;
  const float* val = nullptr;
  if (prog) {
    const int* hdr = reinterpret_cast<const int*>(prog);
    n_edits = hdr[0];
    nnz = hdr[2];
    crep = reinterpret_cast<const float*>(prog + 16);
    post = crep + n_edits * P2P_PROGRAM_COLS;
    colptr = reinterpret_cast<const int*>(post + n_edits * P2P_PROGRAM_COLS);
    rowidx = colptr + n_edits * P2P_PROGRAM_COLS;
    val = reinterpret_cast<const float*>(rowidx + nnz);
  }

  for (int b = 0; b < count; ++b) {
    const int n = first + b;
    const IO* const qp = static_cast<const IO*>(a.q) + (int64_t)n * a.bsq + h * D;
    const IO* const kp = static_cast<const IO*>(a.k) + (int64_t)n * a.bsk + h * D;
    const IO* const vp = static_cast<const IO*>(a.v) + (int64_t)n * a.bsv + h * D;
    IO* const op = static_cast<IO*>(a.o) + (int64_t)n * a.bso + h * D;

    __syncthreads();  // previous prompt's LDS reads are done
    for (int cidx = tid; cidx < K * CPR; cidx += NT) {
      const int row = cidx / CPR;
      const int ch = cidx - row * CPR;
      Chunk8<IO> kc, vc;
      kc.load(kp + (int64_t)row * a.ldk + ch * 8);
      vc.load(vp + (int64_t)row * a.ldv + ch * 8);
      kc.store(Ks + row * KS + ch * 8);
      vc.store(Vs + row * VS + ch * 8);
    }
    typename M::frag qf[NKT];
#pragma unroll
    for (int t = 0; t < NKT; ++t) {
      const int col = 16 * t + 8 * hh;
      if (prow && col < D) {
        E tmp[8] __attribute__((aligned(16)));
        load8_global<IO, M>(qp + (int64_t)p * a.ldq + col, tmp);
        qf[t] = M::load8(tmp);
      } else {
        qf[t] = M::zero();
      }
    }
    __syncthreads();

    // ---- S^T and the exact softmax over the K keys
    float sv[KB][16];
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      f32x16_t acc = {};
#pragma unroll
      for (int t = 0; t < NKT; ++t) {
        const typename M::frag fa = M::load8(Ks + (kb * 32 + qi) * KS + 16 * t + 8 * hh);
        M::mma(acc, fa, qf[t]);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) sv[kb][r] = (kb * 32 + acc_row(r, hh) < K) ? acc[r] : -INFINITY;
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sv[kb][r]);
    mx = fmaxf(mx, __shfl_xor(mx, 32)) * c;
    float ls = 0.f;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = fast_exp2(fmaf(sv[kb][r], c, -mx));
        sv[kb][r] = e;
        ls += e;
      }
    const float inv = 1.f / (ls + __shfl_xor(ls, 32));
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) sv[kb][r] *= inv;

    // ---- P2P cross edit (cond groups only)
    if (prog && count > 1) {
      if (b == 0) {
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int w = kb * 32 + acc_row(r, hh);
            if (w < K) P0w[w] = sv[kb][r];
          }
        __syncthreads();
      } else {
        const int e = b - 1;
        const float* ce = crep + e * P2P_PROGRAM_COLS;
        const float* pe = post + e * P2P_PROGRAM_COLS;
        const int* cp = colptr + e * P2P_PROGRAM_COLS;
        const float* al = alpha + e * K;
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int w = kb * 32 + acc_row(r, hh);
            if (w < K) {
#pragma clang fp contract(off)
              const float pb = sv[kb][r];
              float acc = ce[w] * pb;
              const int t1 = cp[w + 1];
              for (int t = cp[w]; t < t1; ++t) acc = acc + val[t] * P0w[rowidx[t]];
              const float R = pe[w] * acc;
              const float aw = al[w];
              sv[kb][r] = aw * R + (1.f - aw) * pb;
            }
          }
      }
    }

    // ---- AttentionStore epilogue (post-edit maps)
    const int slot = a.store_slot[n];
    if (a.store && slot >= 0 && prow) {
      float* mp = a.store + ((int64_t)(slot + h) * a.P + p) * (int64_t)K;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int w = kb * 32 + acc_row(r, hh);
          if (w < K) mp[w] = a.store_accumulate ? mp[w] + sv[kb][r] : sv[kb][r];
        }
    }

    // ---- O = P' V
    f32x16_t O[NDT];
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) O[dt] = f32x16_t{};
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) pv_block<VS, NDT>(M{}, O, Vs, kb * 32, sv[kb], lane);
    if (prow) {
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int dd = dt * 32 + 8 * g + 4 * hh;
          if (dd < D)
            store4(op + (int64_t)p * a.ldo + dd, O[dt][4 * g], O[dt][4 * g + 1], O[dt][4 * g + 2],
                   O[dt][4 * g + 3]);
        }
    }
  }
}

// ====================================================================== launchers
template <typename IO, typename M, int D>
static hipError_t launch_self_d(const SelfArgs& a, int mode, hipStream_t st) {
  constexpr int BK = (D >= 128 || M::kElemBytes == 4) ? 32 : 64;
  const bool small = a.P <= 64;
  SelfArgs b = a;
  if (small) {
    constexpr int W = 2;
    b.n_qtiles = (a.P + 32 * W - 1) / (32 * W);
    dim3 grid(b.n_qtiles * a.H * a.N), block(64 * W);
    switch (mode) {
      case MODE_FUSED: hipLaunchKernelGGL((self_attn_kernel<IO, M, D, BK, W, MODE_FUSED>), grid, block, 0, st, b); break;
      case MODE_STORE: hipLaunchKernelGGL((self_attn_kernel<IO, M, D, BK, W, MODE_STORE>), grid, block, 0, st, b); break;
      case MODE_PROBS: hipLaunchKernelGGL((self_attn_kernel<IO, M, D, BK, W, MODE_PROBS>), grid, block, 0, st, b); break;
      default: hipLaunchKernelGGL((self_attn_kernel<IO, M, D, BK, W, MODE_PV>), grid, block, 0, st, b); break;
    }
  } else {
    constexpr int W = 4;
    b.n_qtiles = (a.P + 32 * W - 1) / (32 * W);
    dim3 grid(b.n_qtiles * a.H * a.N), block(64 * W);
    switch (mode) {
      case MODE_FUSED: hipLaunchKernelGGL((self_attn_kernel<IO, M, D, BK, W, MODE_FUSED>), grid, block, 0, st, b); break;
      case MODE_STORE: hipLaunchKernelGGL((self_attn_kernel<IO, M, D, BK, W, MODE_STORE>), grid, block, 0, st, b); break;
      case MODE_PROBS: hipLaunchKernelGGL((self_attn_kernel<IO, M, D, BK, W, MODE_PROBS>), grid, block, 0, st, b); break;
      default: hipLaunchKernelGGL((self_attn_kernel<IO, M, D, BK, W, MODE_PV>), grid, block, 0, st, b); break;
    }
  }
  return hipGetLastError();
}

template <typename IO, typename M, int D>
static hipError_t launch_cross_d(const CrossArgs& a, int n_groups, hipStream_t st) {
  constexpr int W = (M::kElemBytes == 4 && D >= 128) ? 2 : 4;
  CrossArgs b = a;
  b.n_qtiles = (a.P + 32 * W - 1) / (32 * W);
  dim3 grid(b.n_qtiles * a.H * n_groups), block(64 * W);
  hipLaunchKernelGGL((cross_attn_kernel<IO, M, D, W>), grid, block, 0, st, b);
  return hipGetLastError();
}

#define P2P_FOR_EACH_D(X) X(8) X(16) X(32) X(40) X(64) X(80) X(128) X(160)

template <typename IO, typename M>
static int dispatch_self(const SelfArgs& a, int d, int mode, hipStream_t st) {
  switch (d) {
#define P2P_CASE(DD) case DD: return (int)launch_self_d<IO, M, DD>(a, mode, st);
    P2P_FOR_EACH_D(P2P_CASE)
#undef P2P_CASE
    default: return P2P_E_HEAD_DIM;
  }
}

template <typename IO, typename M>
static int dispatch_cross(const CrossArgs& a, int d, int n_groups, hipStream_t st) {
  switch (d) {
#define P2P_CASE(DD) case DD: return (int)launch_cross_d<IO, M, DD>(a, n_groups, st);
    P2P_FOR_EACH_D(P2P_CASE)
#undef P2P_CASE
    default: return P2P_E_HEAD_DIM;
  }
}

int run_self(const SelfArgs& a, int io_dtype, int compute, int d, int mode, hipStream_t st) {
  if (compute == P2P_COMPUTE_F32) {
    if (io_dtype != P2P_DTYPE_F32) return P2P_E_DTYPE;
    return dispatch_self<float, MmaF32>(a, d, mode, st);
  }
  if (io_dtype == P2P_DTYPE_F32) return dispatch_self<float, MmaBf16>(a, d, mode, st);
  return dispatch_self<uint16_t, MmaBf16>(a, d, mode, st);
}

int run_cross(const CrossArgs& a, int io_dtype, int compute, int d, int n_groups, hipStream_t st) {
  if (compute == P2P_COMPUTE_F32) {
    if (io_dtype != P2P_DTYPE_F32) return P2P_E_DTYPE;
    return dispatch_cross<float, MmaF32>(a, d, n_groups, st);
  }
  if (io_dtype == P2P_DTYPE_F32) return dispatch_cross<float, MmaBf16>(a, d, n_groups, st);
  return dispatch_cross<uint16_t, MmaBf16>(a, d, n_groups, st);
}

}  // namespace p2p
