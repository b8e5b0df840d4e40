// Fused Prompt-to-Prompt attention kernels for MI355X (gfx950).
//
// self_attn_fused_kernel : flash-style self-attention (ptp_utils.py:183-208, context=None) with
//                     the source-map injection of AttentionControlEdit.replace_self_attention
//                     (main.py:169-174 / null_text.py:224-230) as a batch index remap.
// self_maps_kernel  : the AttentionStore epilogue (main.py:129-142) for self layers whose maps
//                     are kept, from the fused kernel's row log-sum-exp.
// self_probs_kernel / self_pv_kernel : the materialise protocol (probabilities to HBM, then P V).
// cross_attn_kernel : cross-attention over the 77 text tokens with the P2P cross edit
//                     (AttentionControlEdit.forward, main.py:180-197) applied in registers
//                     between the exact softmax and PV, for every prompt group.
//
// Both kernels follow the transposed-fragment convention of p2p_device.h: S^T = K Q^T and
// O^T = V^T P^T, query on the lane.
#include <type_traits>

#include "p2p_device.h"
#include "p2p_kernels.h"

namespace p2p {

template <typename E>
__device__ __forceinline__ E one_elem();
template <>
__device__ __forceinline__ float one_elem<float>() { return 1.0f; }
template <>
__device__ __forceinline__ uint16_t one_elem<uint16_t>() { return 0x3F80; }  // bf16 1.0

// ====================================================================== self attention
enum { MODE_FUSED = 0, MODE_PV = 3 };

// The materialise protocol's second half (ptp_utils.py:206-207 after a controller rewrote attn):
// O[n] = probs[n*H + h] V[n] with the probabilities read from HBM.  Same Oᵀ = Vᵀ Pᵀ form as the
// fused kernel: the lane (query) reads its row's keys in the Sᵀ accumulator order, 4 consecutive
// keys per 16-byte load (keys (r&3) + 8(r>>2) + 4h), so a half-wave covers 32 bytes of each of its
// 32 rows per instruction and four instructions a 128-byte segment; V tiles are staged in LDS.
template <typename IO, typename MP, int D, int BK, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void self_pv_kernel(SelfArgs a) {
  using EV = typename MP::elem;
  constexpr int DV = (D + 31) / 32 * 32;
  constexpr int NDT = DV / 32;
  constexpr int NSB = BK / 32;
  constexpr int VS = (MP::kElemBytes == 2) ? VStrideBf16<DV>::value : DV;
  constexpr int NT = 64 * WAVES;
  constexpr int CPR = D / 8;
  constexpr int NCH = (BK * CPR + NT - 1) / NT;
  constexpr int VBUF = BK * VS;
  constexpr int VBYTES = 2 * VBUF * (int)sizeof(EV);
  __shared__ __attribute__((aligned(16))) char smem[VBYTES + 16];
  EV* const Vs = reinterpret_cast<EV*>(smem);

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
  const int p = qt * 32 * WAVES + wave * 32 + qi;
  const bool prow = p < a.P;
  const int K = a.K;
  const IO* const vp = static_cast<const IO*>(a.v) + (int64_t)n * a.bsv + h * D;
  IO* const op = static_cast<IO*>(a.o) + (int64_t)n * a.bso + h * D;
  const float* const pp = a.probs + ((int64_t)(n * a.H + h) * a.P + (prow ? p : 0)) * (int64_t)K;
  const bool vec4 = (K & 3) == 0;

  // zero the LDS image once: pad columns [D, DV) and rows >= K stay zero
  for (int i = tid; i < VBYTES / 4; i += NT) reinterpret_cast<float*>(smem)[i] = 0.f;

  Chunk8<IO> vreg[NCH];
  auto stage_load = [&](int kt) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int cidx = tid + i * NT;
      const int row = cidx / CPR;
      const int ch = cidx - row * CPR;
      const int key = kt * BK + row;
      if (cidx < BK * CPR && key < K) vreg[i].load(vp + (int64_t)key * a.ldv + ch * 8); else vreg[i].clear();
    }
  };
  auto stage_write = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int cidx = tid + i * NT;
      if (cidx < BK * CPR) {
        const int row = cidx / CPR;
        const int ch = cidx - row * CPR;
        vreg[i].store(Vs + buf * VBUF + row * VS + ch * 8);
      }
    }
  };

  const int ntiles = (K + BK - 1) / BK;
  f32x16_t O[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) O[dt] = f32x16_t{};
  __syncthreads();
  stage_load(0);
  stage_write(0);
  __syncthreads();
  for (int kt = 0; kt < ntiles; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < ntiles) stage_load(kt + 1);
    float sv[NSB][16];
#pragma unroll
    for (int sb = 0; sb < NSB; ++sb)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int key = kt * BK + sb * 32 + 8 * g + 4 * hh;
        if (vec4 && prow && key < K) {  // K % 4 == 0: the 4 keys are all in range together
          const f32x4_t x = *reinterpret_cast<const f32x4_t*>(pp + key);
          sv[sb][4 * g] = x[0];
          sv[sb][4 * g + 1] = x[1];
          sv[sb][4 * g + 2] = x[2];
          sv[sb][4 * g + 3] = x[3];
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) sv[sb][4 * g + e] = (prow && key + e < K) ? pp[key + e] : 0.f;
        }
      }
    const EV* Vb = Vs + buf * VBUF;
#pragma unroll
    for (int sb = 0; sb < NSB; ++sb) pv_block<VS, NDT>(MP{}, O, Vb, sb * 32, sv[sb], lane);
    if (kt + 1 < ntiles) stage_write(buf ^ 1);
    __syncthreads();
  }
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

// ====================================================================== fused self attention
// The hot kernel (G1/G7: P = K = 4096, d = 40).  Beyond a plain online-softmax (flash) loop:
//  * row sums come out of the PV MFMA: V's first padding column (d..DV) is set to 1 in LDS, so
//    O^T row d accumulates sum_k bf16(p_k) -- the same weights the PV uses -- with no VALU adds
//    (only when DV > D; otherwise the sum is a per-lane VALU sum as before);
//  * lazy rescale (defer-max): the running max only moves -- and O is only rescaled -- when a
//    tile's max exceeds it by more than kRescaleThr (log2 units), so p stays <= 2^kRescaleThr;
//    the decision precedes the tile's exponentiation (the safe order), wave-uniform;
//  * no key-mask support (materialise mode only) and masking code only for a partial last tile.
//  * EXACT (launches that keep maps): the row sum is the f32 sum of the exponentials (VALU adds),
//    not the MFMA sum of their bf16 roundings, so the lse that self_maps_kernel normalises the
//    stored maps with is f32-exact (a peaky row's bf16 rounding would otherwise be ~2e-3).
//  * NOMAX (launches that want O only): no per-tile row max at all.  The first tile sets the
//    reference point from its exact max; later tiles exponentiate against it directly and the
//    row sum that the PV MFMA leaves in the ones column is checked once per tile: a row whose sum
//    passes 2^64 is rescaled by 2^-64 (its reference moves up by 64).  bf16 P has the f32
//    exponent range, so p may grow far past 1 without any loss of relative precision; only a
//    logit jumping more than ~115 (log2 units) above the running reference within one tile could
//    overflow -- that shows as a non-finite row sum, and then the whole workgroup recomputes
//    its tiles with the max-tracking loop.  Saves the 8 v_max3 + reduction + decision of every
//    32 x 32 block (the kernel is VALU-issue-bound at d = 40).
template <typename IO, typename MQ, typename MP, int D, int BK, int WAVES, bool EXACT = false, bool NOMAX = false>
__global__ __launch_bounds__(64 * WAVES) void self_attn_fused_kernel(SelfArgs a) {
  using EK = typename MQ::elem;
  using EV = typename MP::elem;
  constexpr int DK = (D + 15) / 16 * 16;
  constexpr int DV = (D + 31) / 32 * 32;
  constexpr int NKT = DK / 16;
  constexpr int NDT = DV / 32;
  constexpr int NSB = BK / 32;
  constexpr int KS = KStride<DK, MQ::kElemBytes>::value;
  constexpr int VS = (MP::kElemBytes == 2) ? VStrideBf16<DV>::value : DV;
  constexpr int NT = 64 * WAVES;
  constexpr int CPR = D / 8;
  constexpr int NCH = (BK * CPR + NT - 1) / NT;
  constexpr int KPLANE = BK * KS;
  constexpr int KBUF = KPLANE * MQ::planes;
  constexpr int VBUF = BK * VS;
  constexpr int KBYTES = 2 * KBUF * (int)sizeof(EK);
  constexpr int VBYTES = 2 * VBUF * (int)sizeof(EV);
  constexpr bool kOnes = DV > D && !EXACT;       // row sum through the PV MFMA
  constexpr int kLdt = D / 32;                   // O^T tile / register / lane-half holding row D
  constexpr int kLrr = D % 32;
  constexpr int kLh = (kLrr >> 2) & 1;
  constexpr int kLr = (kLrr & 3) + 4 * (kLrr >> 3);
  constexpr float kRescaleThr = 8.0f;
  __shared__ __attribute__((aligned(16))) char smem[KBYTES + VBYTES + 16];
  EK* const Ks = reinterpret_cast<EK*>(smem);
  EV* const Vs = reinterpret_cast<EV*>(smem + KBYTES);

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

  // LDS image: zero pads; V column D = 1 in every row of both buffers (the row-sum column)
  for (int i = tid; i < (KBYTES + VBYTES) / 4; i += NT) reinterpret_cast<float*>(smem)[i] = 0.f;
  __syncthreads();
  if constexpr (kOnes) {
    for (int r = tid; r < 2 * BK; r += NT) Vs[r * VS + D] = one_elem<EV>();
  }

  typename MQ::frag qf[NKT];
#pragma unroll
  for (int t = 0; t < NKT; ++t) {
    const int col = 16 * t + 8 * hh;
    qf[t] = (prow && col < D) ? MQ::load_q(qp + (int64_t)p * a.ldq + col) : MQ::zero();
  }

  Chunk8<IO> kreg[NCH], vreg[NCH];
  // Per-lane element offsets inside a tile are loop-invariant (the tile base advances by a
  // wave-uniform stride), so no address VGPR is rewritten inside the loop.  Rows past K load
  // row K-1 instead of a divergent clear path: those keys are masked to -inf, p = 0, and the
  // duplicated K/V rows never contribute.  Chunk slots past the tile are wave-uniform when
  // BK*CPR % 64 == 0.
  // K/V tiles are fetched with range-checked buffer loads: the descriptor spans this (entry,
  // head)'s rows [tile start, K), so chunks of rows past K read as zeros with no tail logic,
  // and the per-lane byte offsets stay loop-invariant (a VMEM address VGPR rewritten inside
  // the loop makes the compiler drain the prefetch with vmcnt(0)).  Chunk slots past the tile
  // are wave-uniform when BK*CPR % 64 == 0.
  uint32_t koff[NCH], voff[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int cidx = tid + i * NT;
    const int row = min(cidx / CPR, BK - 1);
    const int ch = cidx - (cidx / CPR) * CPR;
    koff[i] = (uint32_t)((row * (int)a.ldk + ch * 8) * (int)sizeof(IO));
    voff[i] = (uint32_t)((row * (int)a.ldv + ch * 8) * (int)sizeof(IO));
  }
  const int64_t kbytes = ((int64_t)(K - 1) * a.ldk + D) * (int64_t)sizeof(IO);
  const int64_t vbytes = ((int64_t)(K - 1) * a.ldv + D) * (int64_t)sizeof(IO);
  const int64_t kstep = (int64_t)BK * a.ldk * (int64_t)sizeof(IO);
  const int64_t vstep = (int64_t)BK * a.ldv * (int64_t)sizeof(IO);
  auto stage_load = [&](int kt) {
    const __amdgpu_buffer_rsrc_t rk =
        make_rsrc(reinterpret_cast<const char*>(kp) + kt * kstep, kbytes - kt * kstep);
    const __amdgpu_buffer_rsrc_t rv =
        make_rsrc(reinterpret_cast<const char*>(vp) + kt * vstep, vbytes - kt * vstep);
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int cidx = tid + i * NT;
      if ((BK * CPR) % NT == 0 || cidx < BK * CPR) {
        kreg[i].load_buf(rk, koff[i]);
        vreg[i].load_buf(rv, voff[i]);
      }
    }
  };
  auto stage_write = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int cidx = tid + i * NT;
      if ((BK * CPR) % NT == 0 || cidx < BK * CPR) {
        const int row = cidx / CPR;
        const int ch = cidx - row * CPR;
        MQ::stage(kreg[i], Ks + buf * KBUF + row * KS + ch * 8, KPLANE);
        vreg[i].store(Vs + buf * VBUF + row * VS + ch * 8);
      }
    }
  };

  const int ntiles = (K + BK - 1) / BK;
  f32x16_t O[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) O[dt] = f32x16_t{};
  float m_run = -INFINITY;  // log2-domain running max (scaled), lagging by < kRescaleThr
  float l_run = 0.f;        // per-lane partial row sum (only when !kOnes)

  stage_load(0);
  stage_write(0);
  // retire every prologue load (Q fragments included) before the loop: otherwise the loop
  // header merge leaves Q "possibly pending" and the first QK^T waits vmcnt(0), draining the
  // tile prefetch on every iteration
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  __syncthreads();
  // one K/V tile; the key mask exists only in the instantiation for a partial last tile (as a
  // runtime branch the compiler if-converted it: ~100 extra VALU per tile on every tile)
  bool bad = false;  // NOMAX: some row sum of this lane went non-finite
  auto tile = [&](int kt, auto masked, auto fast) {
    const int buf = kt & 1;
    if (kt + 1 < ntiles) stage_load(kt + 1);
    float sv[NSB][16];
    const EK* Kb = Ks + buf * KBUF;
#pragma unroll
    for (int sb = 0; sb < NSB; ++sb) {
      f32x16_t acc = {};
#pragma unroll
      for (int t = 0; t < NKT; ++t) {
        const typename MQ::frag fa = MQ::load_k(Kb + (sb * 32 + qi) * KS + 16 * t + 8 * hh, KPLANE);
        MQ::mma(acc, fa, qf[t]);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) sv[sb][r] = acc[r];
    }
    if constexpr (decltype(masked)::value) {
#pragma unroll
      for (int sb = 0; sb < NSB; ++sb)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (kt * BK + sb * 32 + acc_row(r, hh) >= K) sv[sb][r] = -INFINITY;
    }
    if constexpr (!decltype(fast)::value) {
      float mx = -INFINITY;
#pragma unroll
      for (int sb = 0; sb < NSB; ++sb)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sv[sb][r]);
      mx = fmaxf(mx, other_half(mx)) * c;
      // defer-max: move the reference point only when this tile overshoots it by > thr
      if (__builtin_expect(!__all(mx <= m_run + kRescaleThr), 0)) {
        const float mnew = fmaxf(m_run, mx);
        const float alpha = fast_exp2(m_run - mnew);
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
          for (int r = 0; r < 16; ++r) O[dt][r] *= alpha;
        l_run *= alpha;
        m_run = mnew;
      }
    }
    float ls = 0.f;
#pragma unroll
    for (int sb = 0; sb < NSB; ++sb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = fast_exp2(fmaf(sv[sb][r], c, -m_run));
        sv[sb][r] = e;
        if constexpr (!kOnes) ls += e;
      }
    if constexpr (!kOnes) l_run += ls;
    const EV* Vb = Vs + buf * VBUF;
#pragma unroll
    for (int sb = 0; sb < NSB; ++sb) pv_block<VS, NDT>(MP{}, O, Vb, sb * 32, sv[sb], lane);
    if constexpr (decltype(fast)::value) {
      // the row sum so far (ones column; lanes kLh of the pair hold it, the other half a zero
      // pad column): rescale rows past 2^64, flag non-finite ones
      const float own = O[kLdt][kLr];
      const float lsum = own + other_half(own);
      bad |= !(lsum < INFINITY);
      if (__builtin_expect(__any(lsum > 0x1p64f), 0)) {
        if (lsum > 0x1p64f) {
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
            for (int r = 0; r < 16; ++r) O[dt][r] *= 0x1p-64f;
          m_run += 64.f;
        }
      }
    }
    if (kt + 1 < ntiles) stage_write(buf ^ 1);
    __syncthreads();
  };
  const int nfull = K / BK;
  if constexpr (NOMAX) {
    static_assert(kOnes, "NOMAX reads the row sum from the ones column");
    __shared__ int wg_bad;
    if (tid == 0) wg_bad = 0;
    // tile 0 sets every row's reference point from its exact max
    if (nfull == 0) tile(0, std::true_type{}, std::false_type{});
    else tile(0, std::false_type{}, std::false_type{});
    for (int kt = 1; kt < nfull; ++kt) tile(kt, std::false_type{}, std::true_type{});
    if (nfull < ntiles && nfull > 0) tile(nfull, std::true_type{}, std::true_type{});
    if (__any(bad) && lane == 0) wg_bad = 1;
    __syncthreads();
    if (__builtin_expect(wg_bad != 0, 0)) {
      // some row overflowed: the whole workgroup recomputes with the max-tracking loop
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) O[dt] = f32x16_t{};
      m_run = -INFINITY;
      stage_load(0);
      stage_write(0);
      __builtin_amdgcn_s_waitcnt(0x0F70);
      __syncthreads();
      for (int kt = 0; kt < nfull; ++kt) tile(kt, std::false_type{}, std::false_type{});
      if (nfull < ntiles) tile(nfull, std::true_type{}, std::false_type{});
    }
  } else {
    for (int kt = 0; kt < nfull; ++kt) tile(kt, std::false_type{}, std::false_type{});
    if (nfull < ntiles) tile(nfull, std::true_type{}, std::false_type{});
  }
  float l;
  if constexpr (kOnes) l = __shfl(O[kLdt][kLr], (lane & 31) + 32 * kLh);
  else l = l_run + __shfl_xor(l_run, 32);
  const float inv = 1.f / l;
  if (prow) {
    IO* const op = static_cast<IO*>(a.o) + (int64_t)n * a.bso + h * D + (int64_t)p * a.ldo;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int dd = dt * 32 + 8 * g + 4 * hh;
        if (dd < D)
          store4(op + dd, O[dt][4 * g] * inv, O[dt][4 * g + 1] * inv, O[dt][4 * g + 2] * inv,
                 O[dt][4 * g + 3] * inv);
      }
    // row log-sum-exp for the backward pass (log2 domain, scale folded: p = exp2(c s - lse))
    if (a.lse && hh == 0) a.lse[(int64_t)(n * a.H + h) * a.P + p] = m_run + __log2f(l);
  }
}

// ====================================================================== fused self attention, QB rows/wave
// The production d = 40 kernel (G1/G7 without kept maps or autograd): the NOMAX loop above with
// QB 32-row query blocks per wave.  Every K fragment and V fragment read from LDS feeds QB MFMAs
// (half the LDS reads per FLOP at QB = 2), the QB blocks are independent instruction streams in
// the wave, and a tile runs sub-block by sub-block (Q K^T, [max decision], exp, P V) so only one
// 32-key sub-block of scores per block is live; 128-key tiles halve the barriers.  Slow tiles
// (the first one, and the overflow recompute) move the reference point per sub-block with the
// defer-max rule -- the sub-block's P V follows at once, so no P is pending at a rescale.
// Measured at G1 (N = 8, H = 8, bf16; tools/g1_ab.py, profiles/r02): 0.239 ms (64-key tiles with
// the per-tile max, one block per wave) -> 0.233 (NOMAX) -> 0.217 (this, QB = 2, BK = 128).
//
// F16 (bf16 inputs, d = 40): the MFMA itself emits the exponent c*s - m, so a score costs one
// v_exp and half a v_cvt_pk on the VALU instead of v_fma + v_exp + half a cvt:
//   * Q is prescaled by c = scale*log2(e) once, at load, and rounded to f16 (2^-12 relative,
//     8x finer than bf16); K is staged as f16 -- exact, a bf16 value has 8 significant bits --
//     so the QK^T products stay exact in the f32 accumulator;
//   * d = 40 pads to 48 for the MFMA: K column 40 is 1 and Q column 40 holds -m (the row's
//     reference point, an f16 value), so S^T = c s - m comes out of the MFMA;
//   * values outside the f16 range (|k| >= 65520, |c q| >= 65520, |m| >= 65504) set a flag and
//     the workgroup recomputes on the exact bf16 path (K restaged as bf16, fma with c), like the
//     NOMAX overflow recompute.
template <typename IO, typename MQ, int D, int BK, int WAVES, int QB, bool F16 = false, bool PIPE = false,
          bool PRIO = false>
__global__ __launch_bounds__(64 * WAVES) void self_attn_multi_kernel(SelfArgs a) {
  using EK = typename MQ::elem;
  constexpr int DK = (D + 15) / 16 * 16;
  constexpr int DV = (D + 31) / 32 * 32;
  static_assert(DV > D, "needs the ones column");
  static_assert(!F16 || (DK > D && MQ::planes == 1 && sizeof(IO) == 2), "F16: bf16 inputs, a padding column");
  constexpr int NKT = DK / 16;
  constexpr int NDT = DV / 32;
  constexpr int NSB = BK / 32;
  constexpr int KS = KStride<DK, MQ::kElemBytes>::value;
  constexpr int VS = VStrideBf16<DV>::value;
  constexpr int NT = 64 * WAVES;
  constexpr int CPR = D / 8;
  constexpr int NCH = (BK * CPR + NT - 1) / NT;
  constexpr int KPLANE = BK * KS;
  constexpr int KBUF = KPLANE * MQ::planes;
  constexpr int VBUF = BK * VS;
  constexpr int KBYTES = 2 * KBUF * (int)sizeof(EK);
  constexpr int VBYTES = 2 * VBUF * 2;
  constexpr int kLdt = D / 32;
  constexpr int kLrr = D % 32;
  constexpr int kLh = (kLrr >> 2) & 1;
  constexpr int kLr = (kLrr & 3) + 4 * (kLrr >> 3);
  // F16: Q column D (the -m slot) = element (D % 16) % 8 of k-step D / 16, lane half (D % 16) / 8
  constexpr int kMt = D / 16;
  constexpr int kMh = (D % 16) / 8;
  constexpr int kMj = D % 8;
  constexpr float kRescaleThr = 8.0f;
  __shared__ __attribute__((aligned(16))) char smem[KBYTES + VBYTES + 16];
  __shared__ int wg_bad;
  EK* const Ks = reinterpret_cast<EK*>(smem);
  uint16_t* const Vs = reinterpret_cast<uint16_t*>(smem + KBYTES);

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
  const int pw = (qt * WAVES + wave) * 32 * QB;   // first query of this wave
  const int K = a.K;
  const float c = a.scale_log2;

  const IO* const qp = static_cast<const IO*>(a.q) + (int64_t)src * a.bsq + h * D;
  const IO* const kp = static_cast<const IO*>(a.k) + (int64_t)src * a.bsk + h * D;
  const IO* const vp = static_cast<const IO*>(a.v) + (int64_t)n * a.bsv + h * D;

  for (int i = tid; i < (KBYTES + VBYTES) / 4; i += NT) reinterpret_cast<float*>(smem)[i] = 0.f;
  if (tid == 0) wg_bad = 0;
  __syncthreads();
  for (int r = tid; r < 2 * BK; r += NT) {
    Vs[r * VS + D] = 0x3F80;
    if constexpr (F16) Ks[r * KS + D] = 0x3C00;   // f16 1.0: the -m column of Q K^T
  }

  // F16 state: the exact bf16 path is taken by the recompute only (ex), after an f16 range miss
  bool ovf = false;
  typename MQ::frag qf[QB][NKT];
  auto load_qf = [&](auto ex) __attribute__((always_inline)) {
#pragma unroll
    for (int b = 0; b < QB; ++b)
#pragma unroll
      for (int t = 0; t < NKT; ++t) {
        const int col = 16 * t + 8 * hh;
        const int p = pw + 32 * b + qi;
        qf[b][t] = (p < a.P && col < D) ? MQ::load_q(qp + (int64_t)p * a.ldq + col) : MQ::zero();
        if constexpr (F16) if constexpr (!decltype(ex)::value) {
          float mx = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float x = bf2f((uint16_t)qf[b][t].h[j]) * c;
            mx = fmaxf(mx, fabsf(x));
            qf[b][t].h[j] = (short)__builtin_bit_cast(uint16_t, (_Float16)x);
          }
          ovf |= !(mx < 65520.f);
        }
      }
  };
  load_qf(std::false_type{});

  Chunk8<IO> kreg[NCH], vreg[NCH];
  uint32_t koff[NCH], voff[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int cidx = tid + i * NT;
    const int row = min(cidx / CPR, BK - 1);
    const int ch = cidx - (cidx / CPR) * CPR;
    koff[i] = (uint32_t)((row * (int)a.ldk + ch * 8) * (int)sizeof(IO));
    voff[i] = (uint32_t)((row * (int)a.ldv + ch * 8) * (int)sizeof(IO));
  }
  const int64_t kbytes = ((int64_t)(K - 1) * a.ldk + D) * (int64_t)sizeof(IO);
  const int64_t vbytes = ((int64_t)(K - 1) * a.ldv + D) * (int64_t)sizeof(IO);
  const int64_t kstep = (int64_t)BK * a.ldk * (int64_t)sizeof(IO);
  const int64_t vstep = (int64_t)BK * a.ldv * (int64_t)sizeof(IO);
  auto stage_load = [&](int kt) __attribute__((always_inline)) {
    const __amdgpu_buffer_rsrc_t rk =
        make_rsrc(reinterpret_cast<const char*>(kp) + kt * kstep, kbytes - kt * kstep);
    const __amdgpu_buffer_rsrc_t rv =
        make_rsrc(reinterpret_cast<const char*>(vp) + kt * vstep, vbytes - kt * vstep);
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      if ((BK * CPR) % NT == 0 || tid + i * NT < BK * CPR) {
        kreg[i].load_buf(rk, koff[i]);
        vreg[i].load_buf(rv, voff[i]);
      }
    }
  };
  auto stage_write = [&](int buf, auto ex) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int cidx = tid + i * NT;
      if ((BK * CPR) % NT == 0 || cidx < BK * CPR) {
        const int row = cidx / CPR;
        const int ch = cidx - row * CPR;
        EK* const kd = Ks + buf * KBUF + row * KS + ch * 8;
        bool staged = false;
        if constexpr (F16) if constexpr (!decltype(ex)::value) {
          staged = true;
          // bf16 -> f16 is exact for magnitudes in [2^-14, 65504] (8 significant bits); below
          // 2^-14 f16 subnormals keep fewer bits (absolute error < 2^-25, flush to 0 under 2^-25),
          // negligible beside the logits.  RTZ packing would clamp past 65504 silently: the range
          // is checked instead
          short8_t hv;
          float mx = 0.f;
#pragma unroll
          for (int j = 0; j < 8; j += 2) {
            const float x0 = bf2f((uint16_t)kreg[i].v[j]), x1 = bf2f((uint16_t)kreg[i].v[j + 1]);
            mx = fmaxf(mx, fmaxf(fabsf(x0), fabsf(x1)));
            const auto pk = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(x0, x1));
            hv[j] = (short)(pk & 0xffff);
            hv[j + 1] = (short)(pk >> 16);
          }
          ovf |= !(mx < 65504.f);
          *reinterpret_cast<short8_t*>(kd) = hv;
        }
        if (!staged) MQ::stage(kreg[i], kd, KPLANE);
        vreg[i].store(Vs + buf * VBUF + row * VS + ch * 8);
      }
    }
  };

  const int ntiles = (K + BK - 1) / BK;
  f32x16_t O[QB][NDT];
  float m_run[QB];
  float m_q[QB];   // F16: the reference point currently held in Q column D (as -m)
#pragma unroll
  for (int b = 0; b < QB; ++b) {
    m_run[b] = -INFINITY;
    m_q[b] = 0.f;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) O[b][dt] = f32x16_t{};
  }
  auto set_mcol = [&](int b, float m) __attribute__((always_inline)) {   // F16: Q column D := -m (lanes of half kMh)
    m_q[b] = m;
    if constexpr (F16)
      if (hh == kMh) qf[b][kMt].h[kMj] = (short)__builtin_bit_cast(uint16_t, (_Float16)(-m));
  };
  auto mma_qk = [&](f32x16_t& acc, const typename MQ::frag& k, const typename MQ::frag& q, auto ex)
      __attribute__((always_inline)) {
    bool done = false;
    if constexpr (F16) if constexpr (!decltype(ex)::value) {
      done = true;
      typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_t;
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, k.h),
                                                   __builtin_bit_cast(f16x8_t, q.h), acc, 0, 0, 0);
    }
    if (!done) MQ::mma(acc, k, q);
  };

  stage_load(0);
  stage_write(0, std::false_type{});
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  __syncthreads();
  // PRIO (experiment): static priority 1 for the second-dispatched half of the waves
  if constexpr (PRIO)
    if (wave >= WAVES / 2) __builtin_amdgcn_s_setprio(1);
  bool bad = false;
  // One tile, sub-block by sub-block (Q K^T, [max decision], exp, P V): only one sub-block's scores
  // per query block are live.  Slow tiles (the first one, and the overflow recompute) move the
  // reference point per 32-key sub-block with the defer-max rule; fast tiles (NOMAX) do not.
  // ex: the exact bf16 path (F16 recompute after a range miss; the only path without F16).
  auto tile = [&](int kt, auto masked, auto fast, auto ex) __attribute__((always_inline)) {
    constexpr bool kF16 = F16 && !decltype(ex)::value;
    const int buf = kt & 1;
    if (kt + 1 < ntiles) stage_load(kt + 1);
    const EK* Kb = Ks + buf * KBUF;
    const uint16_t* Vb = Vs + buf * VBUF;
    auto qk = [&](int sb, f32x16_t (&acc)[QB]) __attribute__((always_inline)) {
#pragma unroll
      for (int b = 0; b < QB; ++b) acc[b] = f32x16_t{};
#pragma unroll
      for (int t = 0; t < NKT; ++t) {
        const typename MQ::frag fa = MQ::load_k(Kb + (sb * 32 + qi) * KS + 16 * t + 8 * hh, KPLANE);
#pragma unroll
        for (int b = 0; b < QB; ++b) mma_qk(acc[b], fa, qf[b][t], ex);
      }
    };
    // PIPE (fast F16 tiles, where the reference point is fixed for the whole tile): sub-block
    // sb+1's Q K^T is issued before sub-block sb's exponentials, so they can overlap it
    constexpr bool kPipe = PIPE && kF16 && decltype(fast)::value;
    f32x16_t accs[2][QB];
    if constexpr (kPipe) qk(0, accs[0]);
#pragma unroll
    for (int sb = 0; sb < NSB; ++sb) {
      f32x16_t acc[QB];
      if constexpr (kPipe) {
#pragma unroll
        for (int b = 0; b < QB; ++b) acc[b] = accs[sb & 1][b];
        if (sb + 1 < NSB) qk(sb + 1, accs[(sb + 1) & 1]);
      } else {
        qk(sb, acc);
      }
      float sv[QB][16];
#pragma unroll
      for (int b = 0; b < QB; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          sv[b][r] = acc[b][r];
          if constexpr (decltype(masked)::value)
            if (kt * BK + sb * 32 + acc_row(r, hh) >= K) sv[b][r] = -INFINITY;
        }
      if constexpr (!decltype(fast)::value) {
#pragma unroll
        for (int b = 0; b < QB; ++b) {
          float mx = -INFINITY;
#pragma unroll
          for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sv[b][r]);
          mx = fmaxf(mx, other_half(mx));
          mx = kF16 ? mx + m_q[b] : mx * c;   // the sub-block's max, log2 units
          if (__builtin_expect(!__all(mx <= m_run[b] + kRescaleThr), 0)) {
            float mnew = fmaxf(m_run[b], mx);
            if constexpr (kF16) {
              mnew = (float)(_Float16)mnew;   // representable in Q's f16 column
              ovf |= !(fabsf(mnew) < 65504.f);
            }
            const float alpha = fast_exp2(m_run[b] - mnew);
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
              for (int r = 0; r < 16; ++r) O[b][dt][r] *= alpha;
            m_run[b] = mnew;
          }
        }
      }
#pragma unroll
      for (int b = 0; b < QB; ++b) {
        if constexpr (kF16) {
          if constexpr (decltype(fast)::value) {
#pragma unroll
            for (int r = 0; r < 16; ++r) sv[b][r] = fast_exp2(sv[b][r]);
          } else {
            const float dm = m_run[b] - m_q[b];
#pragma unroll
            for (int r = 0; r < 16; ++r) sv[b][r] = fast_exp2(sv[b][r] - dm);
            set_mcol(b, m_run[b]);
          }
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) sv[b][r] = fast_exp2(fmaf(sv[b][r], c, -m_run[b]));
        }
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        MmaBf16::frag pb[QB];
#pragma unroll
        for (int b = 0; b < QB; ++b) pb[b] = MmaBf16::pack_p(sv[b] + 8 * s2);
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const MmaBf16::frag af = vt_frag<VS>(Vb, sb * 32, s2, dt * 32, lane);
#pragma unroll
          for (int b = 0; b < QB; ++b) MmaBf16::mma(O[b][dt], af, pb[b]);
        }
      }
    }
    if constexpr (decltype(fast)::value) {
#pragma unroll
      for (int b = 0; b < QB; ++b) {
        const float own = O[b][kLdt][kLr];
        const float lsum = own + other_half(own);
        bad |= !(lsum < INFINITY);
        if (__builtin_expect(__any(lsum > 0x1p64f), 0)) {
          if (lsum > 0x1p64f) {
            // the new reference is rounded first (F16: it must be exact in Q's f16 column) and
            // O rescaled by the exact factor between the two, so old and new tiles stay consistent
            const float mnew = kF16 ? (float)(_Float16)(m_run[b] + 64.f) : m_run[b] + 64.f;
            const float f = fast_exp2(m_run[b] - mnew);
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
              for (int r = 0; r < 16; ++r) O[b][dt][r] *= f;
            m_run[b] = mnew;
            if constexpr (kF16) {
              ovf |= !(fabsf(mnew) < 65504.f);
              set_mcol(b, mnew);
            }
          }
        }
      }
    }
    if (kt + 1 < ntiles) stage_write(buf ^ 1, ex);
    __syncthreads();
  };
  const int nfull = K / BK;
  constexpr std::false_type kNo{};
  constexpr std::true_type kYes{};
  if (nfull == 0) tile(0, kYes, kNo, kNo);
  else tile(0, kNo, kNo, kNo);
  for (int kt = 1; kt < nfull; ++kt) tile(kt, kNo, kYes, kNo);
  if (nfull < ntiles && nfull > 0) tile(nfull, kYes, kYes, kNo);
  {
    const bool any_bad = __any(bad), any_ovf = __any(ovf);
    if (lane == 0 && (any_bad || any_ovf)) atomicOr(&wg_bad, any_ovf ? 2 : 1);
  }
  __syncthreads();
  if (__builtin_expect(wg_bad != 0, 0)) {
#pragma unroll
    for (int b = 0; b < QB; ++b) {
      m_run[b] = -INFINITY;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) O[b][dt] = f32x16_t{};
    }
    auto redo = [&](auto ex) __attribute__((always_inline)) {
      if constexpr (decltype(ex)::value) {
        load_qf(ex);   // unscaled bf16 Q, column D zero
      } else if constexpr (F16) {
#pragma unroll
        for (int b = 0; b < QB; ++b) set_mcol(b, 0.f);
      }
      stage_load(0);
      stage_write(0, ex);
      __builtin_amdgcn_s_waitcnt(0x0F70);
      __syncthreads();
      for (int kt = 0; kt < nfull; ++kt) tile(kt, kNo, kNo, ex);
      if (nfull < ntiles) tile(nfull, kYes, kNo, ex);
    };
    // F16: every recompute (a range miss or a non-finite row sum) takes the exact bf16 path; a
    // row-sum recompute on the F16 slow path could meet |m| >= 65504 on a later tile with nothing
    // left to catch it
    if constexpr (F16) redo(kYes);
    else redo(kNo);
  }
#pragma unroll
  for (int b = 0; b < QB; ++b) {
    const float l = __shfl(O[b][kLdt][kLr], (lane & 31) + 32 * kLh);
    const float inv = 1.f / l;
    const int p = pw + 32 * b + qi;
    if (p < a.P) {
      IO* const op = static_cast<IO*>(a.o) + (int64_t)n * a.bso + h * D + (int64_t)p * a.ldo;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int dd = dt * 32 + 8 * g + 4 * hh;
          if (dd < D)
            store4(op + dd, O[b][dt][4 * g] * inv, O[b][dt][4 * g + 1] * inv, O[b][dt][4 * g + 2] * inv,
                   O[b][dt][4 * g + 3] * inv);
        }
    }
  }
}

// ====================================================================== stored self maps
// AttentionStore epilogue of the self layers whose maps are kept (main.py:129-142, P <= 32^2;
// the stored tensor is the post-injection map, main.py:181-195).  The fused kernel above has
// produced O and every row's log-sum-exp (log2 domain, scale folded); this kernel recomputes
// S = Q K^T in the NON-transposed orientation -- key on the lane, query on the accumulator
// row -- so p = exp2(c s - lse) leaves as 128-byte row segments per half-wave: the read-add-
// write of the running sum is the whole cost of the layer and is HBM-bound.  With the softmax
// statistics known, keys split freely: one wave = 32 queries x kw keys, one workgroup = four
// consecutive key chunks, so the grid is as wide as the map.  K fragments come straight from
// global memory (a [K, d] head slice is L2-resident); no LDS, no barrier.
template <typename IO, typename MQ, int D, int NB, bool NT>
__global__ __launch_bounds__(256) void self_maps_kernel(SelfArgs a, int kw, int n_kgroups) {
  constexpr int DK = (D + 15) / 16 * 16;
  constexpr int NKT = DK / 16;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int hh = lane >> 5;
  const int li = lane & 31;

  int rest = xcd_remap(blockIdx.x, gridDim.x);
  const int kg = rest % n_kgroups;
  rest /= n_kgroups;
  const int qb = rest % a.n_qtiles;
  rest /= a.n_qtiles;
  const int h = rest % a.H;
  const int n = a.map_entry[rest / a.H];
  const int src = a.qk_src[n];
  const int P = a.P;
  const int K = a.K;
  const int k0 = (kg * 4 + wave) * kw;
  if (k0 >= K) return;  // wave-uniform: no barrier in this kernel
  const int k1 = min(K, k0 + kw);
  const int p0 = qb * 32;
  const float c = a.scale_log2;

  const IO* const qp = static_cast<const IO*>(a.q) + (int64_t)src * a.bsq + h * D;
  const IO* const kp = static_cast<const IO*>(a.k) + (int64_t)src * a.bsk + h * D;
  typename MQ::frag qf[NKT];
#pragma unroll
  for (int t = 0; t < NKT; ++t) {
    const int col = 16 * t + 8 * hh;
    qf[t] = (p0 + li < P && col < D) ? MQ::load_q(qp + (int64_t)(p0 + li) * a.ldq + col) : MQ::zero();
  }
  // per accumulator register r: query row p0 + acc_row(r, hh), its lse and map row
  const float* const lse = a.lse + (int64_t)(n * a.H + h) * P;
  float* const mp = a.store + (int64_t)(a.store_slot[n] + h) * P * (int64_t)K;
  float lr[16];
  bool rok[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = p0 + acc_row(r, hh);
    rok[r] = row < P;
    lr[r] = rok[r] ? lse[row] : 0.f;
  }
  const bool acc_on = a.store_accumulate != 0;
  // NB key blocks per step: all their running-sum reads are issued before the first write (the
  // compiler cannot hoist a later block's loads over stores to the same map)
  for (int kb = k0; kb < k1; kb += 32 * NB) {
    float old[NB][16];
    if (acc_on) {
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int key = kb + 32 * j + li;
#pragma unroll
        for (int r = 0; r < 16; ++r)
          old[j][r] = (key < k1 && rok[r])
                          ? (NT ? __builtin_nontemporal_load(mp + (int64_t)(p0 + acc_row(r, hh)) * K + key)
                                : mp[(int64_t)(p0 + acc_row(r, hh)) * K + key])
                          : 0.f;
      }
    }
    f32x16_t acc[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const IO* const krow = kp + (int64_t)min(kb + 32 * j + li, K - 1) * a.ldk;
      acc[j] = f32x16_t{};
#pragma unroll
      for (int t = 0; t < NKT; ++t) {
        const int col = 16 * t + 8 * hh;
        const typename MQ::frag kf = col < D ? MQ::load_q(krow + col) : MQ::zero();
        MQ::mma(acc[j], qf[t], kf);  // A = Q rows, B = K rows: S (query x key), key on the lane
      }
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int key = kb + 32 * j + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (key < k1 && rok[r]) {
          float v = fast_exp2(fmaf(acc[j][r], c, -lr[r]));
          if (acc_on) v += old[j][r];
          if constexpr (NT) __builtin_nontemporal_store(v, mp + (int64_t)(p0 + acc_row(r, hh)) * K + key);
          else mp[(int64_t)(p0 + acc_row(r, hh)) * K + key] = v;
        }
      }
    }
  }
}

// ====================================================================== materialised probabilities
// The materialise protocol's first half (controllers that override forward(attn, ...),
// main.py:85-98): probs[n*H + h] = softmax(Q K^T * scale), f32 [N*H, P, K] (ptp_utils.py:195-204,
// with the optional key mask of :197-201 and its head-major repeat of the mask rows).  HBM-bound
// (G1: 4.3 GB written per layer), so the store side follows self_maps_kernel: one workgroup = 32
// queries x all keys, the four waves split the keys.  Pass 1 (S^T, query on the lane: reductions
// stay in the lane) gives each wave's partial row max / sum, combined across the waves in LDS;
// pass 2 recomputes S with the key on the lane and writes p = exp2(t - M) / L as 128-byte row
// segments per half-wave.  A masked key scores -FLT_MAX after the scale (the reference fills the
// scaled logits with -finfo.max): p = 0 beside any unmasked key, 1/K on a fully masked row.
template <typename IO, typename MQ, int D, bool NT>
__global__ __launch_bounds__(256) void self_probs_kernel(SelfArgs a, int kw) {
  constexpr int DK = (D + 15) / 16 * 16;
  constexpr int NKT = DK / 16;
  constexpr float kNeg = -3.402823466e38f;
  __shared__ float sm[4][32], sl[4][32];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int hh = lane >> 5;
  const int li = lane & 31;

  int rest = xcd_remap(blockIdx.x, gridDim.x);
  const int qb = rest % a.n_qtiles;
  rest /= a.n_qtiles;
  const int h = rest % a.H;
  const int n = rest / a.H;
  const int P = a.P;
  const int K = a.K;
  const int k0 = wave * kw;
  const int k1 = min(K, k0 + kw);  // empty for trailing waves when K < 4 kw: they still sync
  const int p0 = qb * 32;
  const float c = a.scale_log2;
  const uint8_t* const km = a.key_mask ? a.key_mask + (int64_t)((n * a.H + h) % a.N) * K : nullptr;

  const IO* const qp = static_cast<const IO*>(a.q) + (int64_t)n * a.bsq + h * D;
  const IO* const kp = static_cast<const IO*>(a.k) + (int64_t)n * a.bsk + h * D;
  typename MQ::frag qf[NKT];
#pragma unroll
  for (int t = 0; t < NKT; ++t) {
    const int col = 16 * t + 8 * hh;
    qf[t] = (p0 + li < P && col < D) ? MQ::load_q(qp + (int64_t)(p0 + li) * a.ldq + col) : MQ::zero();
  }
  auto scores = [&](int kb, bool transposed, f32x16_t& acc) {
    const IO* const krow = kp + (int64_t)min(kb + li, K - 1) * a.ldk;
    acc = f32x16_t{};
#pragma unroll
    for (int t = 0; t < NKT; ++t) {
      const int col = 16 * t + 8 * hh;
      const typename MQ::frag kf = col < D ? MQ::load_q(krow + col) : MQ::zero();
      if (transposed) MQ::mma(acc, kf, qf[t]);  // S^T: key on the accumulator row, query on the lane
      else MQ::mma(acc, qf[t], kf);             // S:   query on the accumulator row, key on the lane
    }
  };

  // ---- pass 1: this wave's row max / sum over its keys (t = s * c, or kNeg when masked)
  float m = -INFINITY, l = 0.f;
#pragma unroll 4
  for (int kb = k0; kb < k1; kb += 32) {
    f32x16_t acc;
    scores(kb, true, acc);
    float tv[16];
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = kb + acc_row(r, hh);
      tv[r] = key >= k1 ? -INFINITY : (km && !km[key]) ? kNeg : acc[r] * c;
      mx = fmaxf(mx, tv[r]);
    }
    const float mnew = fmaxf(m, mx);
    if (mnew != -INFINITY) {
      float ls = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) ls += fast_exp2(tv[r] - mnew);
      l = fmaf(l, fast_exp2(m - mnew), ls);
      m = mnew;
    }
  }
  {  // the other half-wave holds the other keys of the same query
    const float m2 = __shfl_xor(m, 32), l2 = __shfl_xor(l, 32);
    const float M = fmaxf(m, m2);
    if (M != -INFINITY) {
      l = (m == -INFINITY ? 0.f : l * fast_exp2(m - M)) + (m2 == -INFINITY ? 0.f : l2 * fast_exp2(m2 - M));
      m = M;
    }
  }
  if (hh == 0) {
    sm[wave][li] = m;
    sl[wave][li] = l;
  }
  __syncthreads();
  // per accumulator register r of the S orientation: query row p0 + acc_row(r, hh)
  float Mr[16], Ir[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = acc_row(r, hh);
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < 4; ++w) M = fmaxf(M, sm[w][row]);
    float L = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) L += sm[w][row] == -INFINITY ? 0.f : sl[w][row] * fast_exp2(sm[w][row] - M);
    Mr[r] = M;
    Ir[r] = 1.f / L;
  }

  // ---- pass 2: exact probabilities, key on the lane
  float* const pp = a.store + (int64_t)(n * a.H + h) * P * (int64_t)K;
#pragma unroll 2
  for (int kb = k0; kb < k1; kb += 32) {
    f32x16_t acc;
    scores(kb, false, acc);
    const int key = kb + li;
    if (key < k1) {
      const bool masked = km && !km[key];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = p0 + acc_row(r, hh);
        if (row < P) {
          const float x = masked ? kNeg - Mr[r] : fmaf(acc[r], c, -Mr[r]);
          if constexpr (NT) __builtin_nontemporal_store(fast_exp2(x) * Ir[r], pp + (int64_t)row * K + key);
          else pp[(int64_t)row * K + key] = fast_exp2(x) * Ir[r];
        }
      }
    }
  }
}

// ====================================================================== cross attention
// One workgroup = one head x one tile of 32*WAVES queries x one batch entry n.  An edit entry
// (position b > 0 of a prompt group that carries an edit program) first recomputes the
// source prompt's probabilities P0 for the same rows (the K = 77 cross product is cheap) and
// parks them in LDS, one 32-row slab per wave, so the edit can gather from them:
//   R[w]  = post[w] * ( c_rep[w] * P_b[w] + sum_{t < tmax} val[t][w] * P0[row[t][w]] )
//   P_b'  = alpha[w] * R[w] + (1 - alpha[w]) * P_b[w]
// which is AttentionReplace (c_rep 0, mapper column w), AttentionRefine (c_rep 1-a, one term
// mapper[w] with weight a), AttentionReweight (c_rep 0, term (w, eq[w])), and Reweight
// chained on either (post = eq) -- host side: p2p_amd/programs.py.  The term planes make the
// gather a wave-uniform loop whose loads are independent across the lane's 48 columns.
// Stored maps leave through the same slab as whole contiguous rows (one [32, K] block per
// wave).  The slab is dynamic LDS, allocated only by launches with an edit or a store, so a
// plain launch runs at the occupancy of its K/V tiles alone.
#ifdef P2P_EXPERIMENTS
// diagnostic clock stamps of the cross kernel (experiments build, P2P_SELF_VARIANT 90):
// [logical workgroup < 4096][wave < 4][slot < 24]; read back by p2p_diag_cross_stamps
__device__ unsigned long long g_cross_stamps[4096 * 4 * 24];
#define P2P_CROSS_STAMP(i)                                                                              \
  if (a.variant == 90 && logical < 4096 && wave < 4 && lane == 0)                                       \
    g_cross_stamps[(logical * 4 + wave) * 24 + (i)] = __builtin_amdgcn_s_memtime();
#else
#define P2P_CROSS_STAMP(i) do { } while (0);
#endif

template <typename IO, typename MQ, typename MP, int D, int WAVES, bool DENSE>
__global__ __launch_bounds__(64 * WAVES, (DENSE && D <= 80) ? 2 : 1) void cross_attn_kernel(CrossArgs a) {
  using EK = typename MQ::elem;
  using EV = typename MP::elem;
  constexpr int DK = (D + 15) / 16 * 16;
  constexpr int DV = (D + 31) / 32 * 32;
  constexpr int NKT = DK / 16;
  constexpr int NDT = DV / 32;
  constexpr int KB = P2P_MAX_KEYS_CROSS / 32;
  constexpr int KR = KB * 32;
  constexpr int KS = KStride<DK, MQ::kElemBytes>::value;
  constexpr int VS = (MP::kElemBytes == 2) ? VStrideBf16<DV>::value : DV;
  constexpr int NT = 64 * WAVES;
  constexpr int CPR = D / 8;
  constexpr int NCH = (KR * CPR + NT - 1) / NT;
  constexpr int KPLANE = KR * KS;
  constexpr int KBYTES = KPLANE * MQ::planes * (int)sizeof(EK);
  constexpr int VBYTES = KR * VS * (int)sizeof(EV);
  __shared__ __attribute__((aligned(16))) char smem[KBYTES + VBYTES];
  extern __shared__ __attribute__((aligned(16))) char cross_dyn[];  // slab: WAVES * 32 * P0S f32
  EK* const Ks = reinterpret_cast<EK*>(smem);
  EV* const Vs = reinterpret_cast<EV*>(smem + KBYTES);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int hh = lane >> 5;
  const int qi = lane & 31;

  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  P2P_CROSS_STAMP(0)
  // Kernel arguments live in memory: every a.field is a scalar load, and a chain of dependent
  // ones costs a round trip each at the start of every workgroup.  Everything the lean path reads
  // that does not depend on the entry is pinned here, so it all arrives in ONE round trip; the
  // entry's packed info is the one dependent load after it.
  asm volatile("" ::"s"(a.n_qtiles), "s"(a.H), "s"(a.N), "s"(a.P), "s"(a.K), "s"(a.q), "s"(a.k), "s"(a.v),
               "s"(a.o), "s"(a.ldq), "s"(a.ldk), "s"(a.ldv), "s"(a.ldo), "s"(a.bsq), "s"(a.bsk), "s"(a.bsv),
               "s"(a.bso), "s"(a.scale_log2));
  // Entries fastest (rotated, below), then heads -- xcd_remap keeps consecutive ids on one XCD, so the source's Q
  // rows that a tile's three edit workgroups re-read (for P0) and the tile's q / o lines stay in
  // that XCD's L2 (in the pipeline, rocprof: G2/G6 21.4 -> 20.1 us, d = 160 21.7 -> 20.9 us;
  // profiles/r04/cross_order_r04p/)
  // (every launch size: with eight groups per call, N = 64, entries fastest also took G2/G6 134 ->
  // 115 us and d = 160 84 -> 72 us against heads fastest, profiles/r04/cross_order_large_r04am/)
  // The second 32 of every 64 ids rotate the entries by N/2, so the two workgroups a CU holds
  // (ids i and i + 32 of an XCD's chunk, as the group kernel's order measured) pair an edit or
  // source entry with an uncond one instead of two edits: G2/G6 19.8 -> 18.5 us in the pipeline
  // (profiles/r04/cross_pairing_r04ae/).  The rotation is constant over each run of N ids only
  // when N divides 32 -- otherwise (N = 64: eight groups per call) two runs would map onto the
  // same entries -- so only then
  const int rot = (32 % a.N == 0) ? ((logical >> 5) & 1) * (a.N >> 1) : 0;
  const int rest = (logical % a.N + rot) % a.N;
  const int h = (logical / a.N) % a.H;
  const int qt = logical / a.N / a.H;
  const int n = a.N - 1 - rest;  // the edits sit last in the batch: dispatch them first
  // one dependent kernel-argument load decides the path (every a.field read is a scalar memory
  // round trip; chains of them cost ~1 us at the start of every workgroup)
  const int info = a.ent_info[n];
  asm volatile("" ::"s"(info));
  const int gi = info & 0xff;
  const int b = (info >> 8) & 0xff;
  const int first = n - b;
  const bool edit = (info >> 16) & 1;
  const bool stored = (info >> 17) & 1;
  // p2p_group.flags P2P_GROUP_F_R_ONLY (dense edits): this call's alpha makes every blend
  // coefficient A = alpha post c_rep + 1 - alpha zero (a Replace / Reweight step inside
  // cross_replace_steps, main.py:189), so P' = R B: the entry's own Q K^T softmax is not needed and
  // neither are its Q and K -- only its V (checked again from the coefficients below)
  const bool r_only = (info >> 18) & 1;
  // wave-uniform in a scalar register: the buffer resources built from it (Q rows, the running-sum
  // rows) stay scalar -- from a VGPR every such load became a readfirstlane waterfall loop
  const int p0w = __builtin_amdgcn_readfirstlane(qt * 32 * WAVES + wave * 32);
  const int p = p0w + qi;
  const bool prow = p < a.P;
  const int K = a.K;
  const float c = a.scale_log2;
  const int P0S = a.slab_stride;
  float* const slab = reinterpret_cast<float*>(cross_dyn) + wave * 32 * P0S;
  // O out.  The accumulator puts the query on the lane, so a direct store writes 32 rows x 8 bytes
  // per instruction.  bf16 outputs with 16-byte rows instead go through LDS (the self kernels'
  // epilogue): after a workgroup barrier (every wave is done with K / V) each wave writes its 32
  // rows into the dead K / V image and stores them back as whole 16-byte row chunks, consecutive
  // lanes along a row -- half the store instructions, whole lines.
  // Same-box rocprof (profiles/r05/ostore_ab/): d = 80 edit steps 16.43 -> 14.90 us, d = 160 17.44 ->
  // 16.56; the 8x8 layers (P = 64: half of every 128-query workgroup's rows past P) ran 2 % slower
  // and keep the direct store
  const bool o16 = std::is_same<IO, uint16_t>::value && a.P >= 256 && (a.ldo & 7) == 0 &&
                   (a.bso & 7) == 0 && ((uintptr_t)a.o & 15) == 0;
  auto store_o = [&](const f32x16_t (&O)[NDT], float inv) __attribute__((always_inline)) {
    if constexpr (std::is_same<IO, uint16_t>::value) {
      if (o16) {
        constexpr int OS = D + 8;   // 16-byte aligned rows on distinct banks
        static_assert(WAVES * 32 * OS * 2 <= KBYTES + VBYTES, "the output rows fit the K / V image");
        __syncthreads();
        uint16_t* const orow = reinterpret_cast<uint16_t*>(smem) + wave * 32 * OS;
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
        uint16_t* const ob = static_cast<uint16_t*>(a.o) + (int64_t)n * a.bso + h * D;
#pragma unroll
        for (int c0 = 0; c0 < 32 * CPR; c0 += 64) {
          const int cidx = c0 + lane;
          const int row = cidx / CPR, ch = cidx - row * CPR;
          if (((32 * CPR) % 64 == 0 || cidx < 32 * CPR) && p0w + row < a.P)
            *reinterpret_cast<short8_t*>(ob + (int64_t)(p0w + row) * a.ldo + ch * 8) =
                *reinterpret_cast<const short8_t*>(orow + row * OS + ch * 8);
        }
        return;
      }
    }
    if (prow) {
      IO* const op = static_cast<IO*>(a.o) + (int64_t)n * a.bso + h * D + (int64_t)p * a.ldo;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int dd = dt * 32 + 8 * g + 4 * hh;
          if (dd < D)
            store4(op + dd, O[dt][4 * g] * inv, O[dt][4 * g + 1] * inv, O[dt][4 * g + 2] * inv, O[dt][4 * g + 3] * inv);
        }
    }
  };

  // ---- plain entries (no edit program, maps not kept): the lean path.  Every global load is
  // issued first (Q fragments, this thread's K and V chunks) and the padding is written while they
  // fly; V's column D is 1, so the P V MFMA's row D is the row sum of the bf16 weights it used
  // (no per-element sum, no normalised P: O is scaled once); only a key block that runs past K
  // is masked.  (Measured at G1, N = 8, H = 8: tools/cross_bench.py, profiles/r02.)
  if constexpr (MP::kElemBytes == 2 && DV > D) {
    if (!edit && !stored) {
      constexpr int kLdt = D / 32;
      constexpr int kLrr = D % 32;
      constexpr int kLh = (kLrr >> 2) & 1;
      constexpr int kLr = (kLrr & 3) + 4 * (kLrr >> 3);
      typename MQ::frag qf[NKT];
      {
        const IO* qp = static_cast<const IO*>(a.q) + (int64_t)n * a.bsq + h * D + (int64_t)p * a.ldq;
#pragma unroll
        for (int t = 0; t < NKT; ++t) {
          const int col = 16 * t + 8 * hh;
          qf[t] = (prow && col < D) ? MQ::load_q(qp + col) : MQ::zero();
        }
      }
      const IO* kp = static_cast<const IO*>(a.k) + (int64_t)n * a.bsk + h * D;
      const IO* vp = static_cast<const IO*>(a.v) + (int64_t)n * a.bsv + h * D;
      Chunk8<IO> kc[NCH], vc[NCH];
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        const int cidx = tid + i * NT;
        const int row = cidx / CPR;
        const int ch = cidx - row * CPR;
        if (cidx < K * CPR) {
          kc[i].load(kp + (int64_t)row * a.ldk + ch * 8);
          vc[i].load(vp + (int64_t)row * a.ldv + ch * 8);
        }
      }
      P2P_CROSS_STAMP(1)
      if constexpr (DK > D) {   // K columns D..DK of every row: Q's zero columns meet zeros, not stale LDS
        constexpr int PC = (DK - D) / 8;
        for (int i = tid; i < KR * PC * MQ::planes; i += NT) {
          const int pl = i / (KR * PC);
          const int j = i - pl * KR * PC;
          *reinterpret_cast<short8_t*>(Ks + pl * KPLANE + (j / PC) * KS + D + 8 * (j % PC)) = short8_t{};
        }
      }
      for (int i = tid; i < (KR - K) * VS / 8; i += NT)   // V rows K..KR (weighted by p = 0)
        *reinterpret_cast<short8_t*>(Vs + K * VS + 8 * i) = short8_t{};
      for (int r = tid; r < K; r += NT) Vs[r * VS + D] = 0x3F80;   // bf16 1.0: the row-sum column
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        const int cidx = tid + i * NT;
        const int row = cidx / CPR;
        const int ch = cidx - row * CPR;
        if (cidx < K * CPR) {
          MQ::stage(kc[i], Ks + row * KS + ch * 8, KPLANE);
          vc[i].store(Vs + row * VS + ch * 8);
        }
      }
      __syncthreads();
      P2P_CROSS_STAMP(2)
      float sv[KB][16];
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        f32x16_t acc = {};
#pragma unroll
        for (int t = 0; t < NKT; ++t) {
          const typename MQ::frag fa = MQ::load_k(Ks + (kb * 32 + qi) * KS + 16 * t + 8 * hh, KPLANE);
          MQ::mma(acc, fa, qf[t]);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) sv[kb][r] = acc[r];
        if (kb * 32 + 32 > K) {   // wave-uniform: only the block that runs past K
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (kb * 32 + acc_row(r, hh) >= K) sv[kb][r] = -INFINITY;
        }
      }
      // K <= (KB-1)*32 + 16 (the 77 text tokens): registers 8..15 of the last block are all masked
      auto soft = [&](auto tail) {
        constexpr bool kShort = decltype(tail)::value;
        float mx = -INFINITY;
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (!(kShort && kb == KB - 1 && r >= 8)) mx = fmaxf(mx, sv[kb][r]);
        mx = fmaxf(mx, other_half(mx)) * c;
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            sv[kb][r] = (kShort && kb == KB - 1 && r >= 8) ? 0.f : fast_exp2(fmaf(sv[kb][r], c, -mx));
      };
      if (K <= (KB - 1) * 32 + 16) soft(std::true_type{});
      else soft(std::false_type{});
      P2P_CROSS_STAMP(3)
      f32x16_t O[NDT];
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) O[dt] = f32x16_t{};
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) pv_block<VS, NDT>(MP{}, O, Vs, kb * 32, sv[kb], lane);
      P2P_CROSS_STAMP(4)
      const float inv = 1.f / __shfl(O[kLdt][kLr], (lane & 31) + 32 * kLh);
      store_o(O, inv);
      P2P_CROSS_STAMP(5)
      return;
    }
  }

  const char* const prog = static_cast<const char*>(a.grp_prog[gi]);
  const int slot = a.store_slot[n];
  // maps kept and accumulated: touch this wave's rows of the running sum now (32 x K f32,
  // contiguous), so the read-add-write of the store epilogue finds them in this XCD's L2 instead of
  // paying an HBM round trip at the end of the workgroup
  // (two loads per lane cover 32 rows of up to 96 keys; their values are only consumed at the very
  // end, so nothing waits for them)
  float touch0 = 0.f, touch1 = 0.f;
  // LocalBlend word weights of this entry (lanes 0-31: alpha, 32-63: substruct) for LDS: loaded now
  // (unconditionally, from valid addresses: a load inside a branch gets its own wait), written to
  // LDS once the prologue's loads are in flight; the store epilogue's per-row word sums then read
  // them from LDS, not global memory
  __shared__ __attribute__((aligned(16))) float btab[2][P2P_MAX_KEYS_CROSS];
  const bool blend_on = stored && a.grp_bsum[gi] != nullptr;
  float bw0 = 0.f, bw1 = 0.f;
  if (blend_on) {
    const float* const ta = a.grp_balpha[gi] + (int64_t)b * K;
    const float* const tsub = a.grp_bsub[gi];
    static_assert(2 * P2P_MAX_KEYS_CROSS <= 2 * NT, "two weights per thread");
    const int i1 = tid + NT;
    const float* s0 = tid < K ? ta + tid : (tid < 2 * K && tsub != nullptr) ? tsub + (int64_t)b * K + tid - K : ta;
    const float* s1 = i1 < K ? ta + i1 : (i1 < 2 * K && tsub != nullptr) ? tsub + (int64_t)b * K + i1 - K : ta;
    bw0 = *s0;
    bw1 = *s1;
    if (!(tid < K || (tid < 2 * K && tsub != nullptr))) bw0 = 0.f;
    if (!(i1 < K || (i1 < 2 * K && tsub != nullptr))) bw1 = 0.f;
  }
  // once the prologue's loads are issued: the blend weights into LDS; this wave's rows of the
  // running sum are touched into this XCD's L2 (32 x K f32, contiguous; two loads per lane cover 32
  // rows of up to 96 keys) so the store epilogue's read-add-write finds them there.  The touches
  // go after every other load: they miss to HBM, and a wait for any load issued after them would
  // wait for them too
  // The touches are issued after the workgroup's first barrier, not with the prologue: the whole
  // launch issues its prologue loads at once, and 10 MB of touches (G2/G6) in that burst delayed
  // every workgroup's first round trip (in the pipeline, rocprof: G2/G6 20.0 -> 19.1 us, d = 160
  // 20.7 -> 20.4; no touches at all: 19.8 / 20.6; profiles/r04/cross_touch_r04r/).  Experiments:
  // Mode 3 goes further: after the first barrier the wave reads its rows of the running sum (and
  // its LocalBlend word-sum entries) into registers, so the store epilogue only adds and writes.
  // (bf16 inputs only: the f32-input instantiations have no registers to spare for the rows)
  // 1: touches after the first barrier, 3: the values themselves
  constexpr int touch_when = std::is_same<IO, uint16_t>::value ? 3 : 1;
  constexpr int kRmwF4 = 32 * KR / 4;
  f32x4_t rmwbuf[(kRmwF4 + 63) / 64];
  float bsum_old = 0.f;
  const int srows = min(32, a.P - p0w);
  float* const sg = stored ? a.store + ((int64_t)(slot + h) * a.P + p0w) * (int64_t)K : nullptr;
  const bool rmw_vec = stored && srows > 0 && ((uintptr_t)sg & 15) == 0 && ((srows * K) & 3) == 0;
  float* const bdst = blend_on ? a.grp_bsum[gi] + ((int64_t)(b * 2 + hh) * a.grp_blh[gi] + a.grp_bcol[gi] + h) * a.P +
                                     p0w + qi
                               : nullptr;
  auto touch = [&]() __attribute__((always_inline)) {
    if (touch_when == 3) {
      // issued unconditionally (zero-size buffer resources when nothing is kept: no traffic), so
      // every path issues the same number of loads here -- a branch-skipped load makes hipcc's waits
      // for the prologue's loads count on the path without it (the dense prologue below)
      const bool acc = stored && a.store_accumulate;
      rmw_load<kRmwF4>(sg, (acc && rmw_vec) ? srows * K : 0, lane, rmwbuf);
      // the lane's LocalBlend word-sum entry: (b * 2 + hh)'s plane, query p0w + qi (lanes past the
      // rows read a neighbour or zero, and keep 0)
      const bool bl = acc && blend_on;
      const float* const bb = bl ? a.grp_bsum[gi] + ((int64_t)(b * 2) * a.grp_blh[gi] + a.grp_bcol[gi] + h) * a.P + p0w : nullptr;
      const __amdgpu_buffer_rsrc_t rb = make_rsrc(bb, bl ? ((int64_t)a.grp_blh[gi] * a.P + srows) * 4 : 0);
      const float v = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rb, (hh * a.grp_blh[gi] * a.P + qi) * 4, 0, 0));
      bsum_old = qi < srows ? v : 0.f;
    } else if (stored && a.store_accumulate) {
      const int rows = min(32, a.P - p0w);
      const float* g = a.store + ((int64_t)(slot + h) * a.P + p0w) * (int64_t)K;
      const int lines = (rows * K * 4 + 127) / 128;
      static_assert(32 * P2P_MAX_KEYS_CROSS * 4 / 128 <= 128, "two touches per lane");
      if (lane < lines) touch0 = g[lane * 32];
      if (lane + 64 < lines) touch1 = g[(lane + 64) * 32];
    }
  };
  auto finish_prologue = [&]() __attribute__((always_inline)) {
    if (blend_on) {
      const int i1 = tid + NT;
      if (tid < 2 * K) btab[tid < K ? 0 : 1][tid < K ? tid : tid - K] = bw0;
      if (i1 < 2 * K) btab[i1 < K ? 0 : 1][i1 < K ? i1 : i1 - K] = bw1;
      // columns K.. of both tables are zero (the 16-byte weight reads of the register sums)
      static_assert(P2P_MAX_KEYS_CROSS <= NT, "one padding column per thread");
      if (tid < P2P_MAX_KEYS_CROSS - K) btab[0][K + tid] = btab[1][K + tid] = 0.f;
    }
    if (touch_when == 0) touch();
  };

  // padding the MFMAs read but the staging never writes (disjoint from it: no extra barrier):
  // K columns D..DK (multiplied by Q's zero columns) and V rows K..KR (weighted by p = 0)
  if constexpr (DK > D) {
    for (int i = tid; i < MQ::planes * KR * (DK - D); i += NT) {
      const int pl = i / (KR * (DK - D));
      const int j = i - pl * KR * (DK - D);
      const int row = j / (DK - D);
      Ks[pl * KPLANE + row * KS + D + (j - row * (DK - D))] = EK(0);
    }
  }
  for (int i = tid; i < (KR - K) * VS; i += NT) Vs[K * VS + i] = EV(0);

  // bf16 inputs: Q rows and K / V chunks by range-checked buffer loads issued unconditionally
  // (rows >= P / >= K read as zeros).  Loads inside a branch per fragment or chunk made hipcc
  // re-load kernel arguments and drain the earlier loads with vmcnt(0) between them: the stored
  // source / plain entries' staging ran as a chain of round trips
  constexpr bool kBufIO = std::is_same<IO, uint16_t>::value && std::is_same<MQ, QkBf16<uint16_t>>::value;
  auto load_q = [&](int e, typename MQ::frag (&qf)[NKT]) {
    const IO* qp = static_cast<const IO*>(a.q) + (int64_t)e * a.bsq + h * D;
    if constexpr (kBufIO) {
      const __amdgpu_buffer_rsrc_t rq = make_rsrc(qp + (int64_t)p0w * a.ldq, ((int64_t)(a.P - 1 - p0w) * a.ldq + D) * 2);
#pragma unroll
      for (int t = 0; t < NKT; ++t) {
        const int col = 16 * t + 8 * hh;
        qf[t].h = __builtin_bit_cast(short8_t, __builtin_amdgcn_raw_buffer_load_b128(rq, (qi * (int)a.ldq + col) * 2, 0, 0));
        if (col >= D) qf[t] = MQ::zero();
      }
    } else {
#pragma unroll
      for (int t = 0; t < NKT; ++t) {
        const int col = 16 * t + 8 * hh;
        qf[t] = (prow && col < D) ? MQ::load_q(qp + (int64_t)p * a.ldq + col) : MQ::zero();
      }
    }
  };

  // K (and V) of entry e: global -> registers (load_kv), registers -> LDS (store_kv); withK = false:
  // V only (an R_ONLY edit)
  auto load_kv = [&](int e, Chunk8<IO> (&kc)[NCH], Chunk8<IO> (&vc)[NCH], bool withV, bool withK = true) {
    const IO* kp = static_cast<const IO*>(a.k) + (int64_t)e * a.bsk + h * D;
    const IO* vp = static_cast<const IO*>(a.v) + (int64_t)e * a.bsv + h * D;
    if constexpr (kBufIO) {
      const __amdgpu_buffer_rsrc_t rk = make_rsrc(kp, ((int64_t)(K - 1) * a.ldk + D) * 2);
      const __amdgpu_buffer_rsrc_t rv = make_rsrc(vp, ((int64_t)(K - 1) * a.ldv + D) * 2);
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        const int cidx = tid + i * NT;
        const int row = cidx / CPR;
        const int ch = cidx - row * CPR;
        if (withK) kc[i].load_buf(rk, (uint32_t)((row * (int)a.ldk + ch * 8) * 2));
        if (withV) vc[i].load_buf(rv, (uint32_t)((row * (int)a.ldv + ch * 8) * 2));
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int cidx = tid + i * NT;
      const int row = cidx / CPR;
      const int ch = cidx - row * CPR;
      if (cidx < K * CPR) {
        if (withK) kc[i].load(kp + (int64_t)row * a.ldk + ch * 8);
        if (withV) vc[i].load(vp + (int64_t)row * a.ldv + ch * 8);
      }
    }
  };
  auto store_kv = [&](const Chunk8<IO> (&kc)[NCH], const Chunk8<IO> (&vc)[NCH], bool withV, bool withK = true) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int cidx = tid + i * NT;
      const int row = cidx / CPR;
      const int ch = cidx - row * CPR;
      if (cidx < K * CPR) {   // (V rows K..KR are zeroed with the padding; K rows past K are masked)
        if (withK) MQ::stage(kc[i], Ks + row * KS + ch * 8, KPLANE);
        if (withV) vc[i].store(Vs + row * VS + ch * 8);
      }
    }
  };
  // exact softmax of S^T = K_e Q_e^T over the K keys for this lane's query row (K rows past
  // K hold stale LDS: their accumulator rows are replaced by -inf, never used)
  // kShort (K <= (KB-1)*32 + 16, e.g. the 77 text tokens): registers 8..15 of the last key block
  // hold keys >= 80, all masked -- their exponentials, sums and scalings are skipped
  const bool short_tail = K <= (KB - 1) * 32 + 16;
  auto probs_t = [&](const typename MQ::frag (&qf)[NKT], float (&sv)[KB][16], auto tail) {
    constexpr bool kShort = decltype(tail)::value;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      f32x16_t acc = {};
#pragma unroll
      for (int t = 0; t < NKT; ++t) {
        const typename MQ::frag fa = MQ::load_k(Ks + (kb * 32 + qi) * KS + 16 * t + 8 * hh, KPLANE);
        MQ::mma(acc, fa, qf[t]);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) sv[kb][r] = acc[r];
      if (kb * 32 + 32 > K) {   // wave-uniform: only the block that runs past K is masked
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (kb * 32 + acc_row(r, hh) >= K) sv[kb][r] = -INFINITY;
      }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (!(kShort && kb == KB - 1 && r >= 8)) mx = fmaxf(mx, sv[kb][r]);
    mx = fmaxf(mx, other_half(mx)) * c;
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
  auto probs = [&](const typename MQ::frag (&qf)[NKT], float (&sv)[KB][16]) {
    if (short_tail) probs_t(qf, sv, std::true_type{});
    else probs_t(qf, sv, std::false_type{});
  };

  typename MQ::frag qf[NKT];
  float sv[KB][16];
  // dense edit (bf16 PV path, program carries the f16 mapper tile): R = P0 . M_e on the MFMA
  constexpr bool kDenseOk = DENSE && MP::kElemBytes == 2;  // separate instantiation: its VGPRs
  // the dense edit's per-column blend coefficients A | B: static LDS, so the store epilogue's
  // per-wave slab (which overlays the dead mapper tile) never overlaps them
  __shared__ __attribute__((aligned(16))) float dcol[kDenseOk ? 2 * KR : 4];
  const bool dense = kDenseOk && edit;   // the launcher picks DENSE only if every edit group is
  f32x16_t Rd[KB];
  int dense_flags = 3;   // dense edits: the blend halves in use (set from the coefficients)
  // dense edits: this entry's own K / V are loaded together with the source's prologue loads, so
  // the workgroup waits one memory round trip instead of two (measured against staging them
  // after the R phase: profiles/r03/cross_store/cross_bench_own_kv_*.log)
  Chunk8<IO> kc1[kDenseOk ? NCH : 1], vc1[kDenseOk ? NCH : 1];
  typename MQ::frag qf1[kDenseOk ? NKT : 1];   // (and its own Q rows)
  bool own_early = false;
  if constexpr (kDenseOk) {
   if (dense) {
    const uint16_t* mg = static_cast<const uint16_t*>(a.grp_dense[gi]) +
                         (int64_t)(b - 1) * P2P_PROGRAM_DENSE * P2P_PROGRAM_DENSE;
    EV* const Ms = reinterpret_cast<EV*>(cross_dyn);  // [96 source words][96 target words]
    // every global load of the prologue is issued at once (one memory round trip), in the order
    // of use: the coefficients and the source's K and Q (P0), then the mapper tile (R) and this
    // entry's own rows.  Each is waited for only where it is used, so the in-order counter lets
    // P0 start once the source's bytes have landed while the tile and the own V land behind it:
    // the launch-wide prologue burst, not the latency, sets the first round trip.
    // d = 160 only: at d <= 80 (two workgroups per CU, 256 VGPRs) the tile and the own V held in
    // registers across P0 spill 56 VGPRs
    constexpr bool late = D > 80;
    constexpr int kMCh = P2P_PROGRAM_DENSE * P2P_PROGRAM_DENSE / 8;   // 16-byte chunks of the tile
    constexpr int kMPer = (kMCh + NT - 1) / NT;
    const float* ce = reinterpret_cast<const float*>(prog + P2P_PROGRAM_HEADER_BYTES +
                                                     (int64_t)(b - 1) * P2P_PROGRAM_REC_BYTES);
    const float* al = a.grp_alpha[gi] + (b - 1) * K;
    static_assert(KR <= NT, "one column per thread");
    const int w = tid;
    float aw = 0.f, cw = 0.f, pw = 0.f;
    if (w < K) {
      aw = al[w];
      cw = ce[w];
      pw = ce[P2P_PROGRAM_COLS + w];
    }
    Chunk8<IO> kc0[NCH], vc0[NCH];
    load_kv(first, kc0, vc0, false);
    load_q(first, qf);
    // (the scheduler would otherwise issue the Q loads last, and every wait for Q would then wait
    // for the tile and the own rows as well)
    __builtin_amdgcn_sched_barrier(0);
    // the tile by range-checked buffer loads (chunks past it read as zeros), the own V on both
    // paths, and only then the path-dependent own K and Q: hipcc's wait for a load counts the
    // loads issued after it on the path that issued the FEWEST, so a branch-skipped load between
    // Q and its use would make the R_ONLY path wait for the tile and the own V before P0
    short8_t mreg[kMPer];
    {
      // rows >= K are zero in the program: past the resource, so they read as zeros without a fetch
      const __amdgpu_buffer_rsrc_t rm = make_rsrc(mg, (int64_t)K * P2P_PROGRAM_DENSE * 2);
#pragma unroll
      for (int j = 0; j < kMPer; ++j)
        mreg[j] = __builtin_bit_cast(short8_t, __builtin_amdgcn_raw_buffer_load_b128(rm, (tid + j * NT) * 16, 0, 0));
    }
    __builtin_amdgcn_sched_barrier(0);
    own_early = !r_only;
    load_kv(n, kc1, vc1, true, false);   // own V
    __builtin_amdgcn_sched_barrier(0);
    if (own_early) {
      load_kv(n, kc1, vc1, false, true);   // own K
      load_q(n, qf1);
    }
    auto store_tile = [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < kMPer; ++j) {
        const int i = tid + j * NT;
        if (i < kMCh) reinterpret_cast<short8_t*>(Ms)[i] = mreg[j];
      }
    };
    finish_prologue();
    P2P_CROSS_STAMP(19)
    if (!late) store_tile();
    P2P_CROSS_STAMP(20)
    {  // per-column coefficients next to the tile, read back after the barriers:
      // P' = alpha*post*(c_rep*P_b + R) + (1-alpha)*P_b = P_b*A + R*B
      float* col = dcol;
      if (w < KR) {
        const float ap = aw * pw;
        col[w] = fmaf(ap, cw, 1.f - aw);
        col[KR + w] = ap;
      }
    }
    P2P_CROSS_STAMP(21)
    store_kv(kc0, vc0, false);
    // R_ONLY: the own V goes to its LDS image in this phase (the P0 / R phase reads only K and the
    // mapper), so no second staging phase follows
    if (r_only && !late) store_kv(kc1, vc1, true, false);
    P2P_CROSS_STAMP(22)
    __syncthreads();
    if (touch_when == 1 || touch_when == 3) touch();
    P2P_CROSS_STAMP(8)
    {
      // which blend halves the row uses (every wave scans the coefficients itself): bit 0 some
      // A != 0 -> this edit's own softmax, bit 1 some B != 0 -> P0 and R.  A Replace step with
      // alpha = 1 on every word (main.py:189) needs only R, one with alpha = 0 only its own P_b;
      // dropping the other half is exact (fma(P, 0, x) = x, fma(P, A, R * 0) = P A)
      const float* col = dcol;
      const int c0 = lane, c1 = lane + 64;
      const bool a0 = c0 < K && col[c0] != 0.f, a1 = c1 < K && col[c1] != 0.f;
      const bool b0 = c0 < K && col[KR + c0] != 0.f, b1 = c1 < K && col[KR + c1] != 0.f;
      dense_flags = (__any(a0 || a1) ? 1 : 0) | (__any(b0 || b1) ? 2 : 0);
    }
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) Rd[kb] = f32x16_t{};
    if (dense_flags & 2) {
    float p0[KB][16];
    probs(qf, p0);
    if (late) {
      store_tile();      // (workgroup-uniform branch: every wave reads the same coefficients)
      __syncthreads();
    }
    P2P_CROSS_STAMP(9)
    // R = M^T P0 on the f16 MFMA: the mapper weights (1, 1/2, 1/4, ...) are exact in f16 and P0 in
    // [0, 1] rounds to 11 significant bits (|dR| <= 2^-12 R, inside the 2e-3 bar); every mapper
    // fragment read once; one 32-key block at a time (the scheduler would otherwise hoist all 18
    // fragment reads)
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        short8_t ph;
#pragma unroll
        for (int r = 0; r < 8; ++r) ph[r] = (short)__builtin_bit_cast(uint16_t, (_Float16)p0[kb][8 * s2 + r]);
#pragma unroll
        for (int dt = 0; dt < KB; ++dt) {
          const MmaBf16::frag af =
              vt_frag<P2P_PROGRAM_DENSE>(reinterpret_cast<const uint16_t*>(Ms), kb * 32, s2, dt * 32, lane);
          typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_t;
          Rd[dt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, af.v),
                                                          __builtin_bit_cast(f16x8_t, ph), Rd[dt], 0, 0, 0);
        }
      }
    }
    }
    if (own_early) {
#pragma unroll
      for (int t = 0; t < NKT; ++t) qf[t] = qf1[t];
    } else if (!r_only || (dense_flags & 1)) {
      load_q(n, qf);
    }
    if (r_only && late) store_kv(kc1, vc1, true, false);   // (V is read only after the barrier below)
    __syncthreads();  // every wave is done with the source K tile and the mapper tile
    P2P_CROSS_STAMP(10)
   }
  }
  if (edit && !dense) {
    // ---- source probabilities P0 for these rows -> this wave's LDS slab
    load_q(first, qf);
    {
      Chunk8<IO> kc[NCH], vc[NCH];
      load_kv(first, kc, vc, false);
      finish_prologue();
      store_kv(kc, vc, false);
    }
    __syncthreads();
    if (touch_when == 1 || touch_when == 3) touch();
    probs(qf, sv);
    load_q(n, qf);
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int w = kb * 32 + acc_row(r, hh);
        if (w < K) slab[qi * P0S + w] = sv[kb][r];
      }
    __syncthreads();  // slab written; every wave is done reading the source K tile
  } else if (!edit) {
    load_q(n, qf);
  }
  auto stage_own = [&]() __attribute__((always_inline)) {
    Chunk8<IO> kc[NCH], vc[NCH];
    load_kv(n, kc, vc, true);
    if (!edit) finish_prologue();   // (the edit paths called it with their first loads)
    store_kv(kc, vc, true);
  };
  bool own_staged = true;
  if constexpr (kDenseOk) {
    if (own_early) {
      store_kv(kc1, vc1, true);
    } else if (r_only) {
      // own V is in LDS already; own K only if the coefficients contradict the host's flag
      own_staged = (dense_flags & 1) != 0;
      if (own_staged) {
        Chunk8<IO> kc[NCH], vc[NCH];
        load_kv(n, kc, vc, false);
        store_kv(kc, vc, false);
      }
    } else {
      stage_own();
    }
  } else {
    stage_own();
  }
  if (own_staged) __syncthreads();   // (workgroup-uniform: every wave reads the same coefficients)
  if (!edit && (touch_when == 1 || touch_when == 3)) touch();
  P2P_CROSS_STAMP(11)
  if (!dense || (dense_flags & 1)) {
    probs(qf, sv);
  } else {
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) sv[kb][r] = 0.f;   // A = 0 on every column: P' = R B
  }
  P2P_CROSS_STAMP(12)

  if (dense) {
    // a lane's columns come in runs of 4 (r & 3): one 16-byte LDS read per run and table;
    // one 32-column block at a time (hoisting every read costs ~150 VGPRs)
    const float* const col = dcol;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int w0 = kb * 32 + 8 * g + 4 * hh;
        const f32x4_t A4 = *reinterpret_cast<const f32x4_t*>(col + w0);
        const f32x4_t B4 = *reinterpret_cast<const f32x4_t*>(col + KR + w0);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = 4 * g + j;
          sv[kb][r] = fmaf(sv[kb][r], A4[j], Rd[kb][r] * B4[j]);   // columns >= K: A = 1, B = 0
        }
      }
    }
  } else if (edit) {
#pragma clang fp contract(off)
    const int tmax = reinterpret_cast<const int*>(prog)[2];
    const char* const rec = prog + P2P_PROGRAM_HEADER_BYTES + (int64_t)(b - 1) * P2P_PROGRAM_REC_BYTES;
    const float* const ce = reinterpret_cast<const float*>(rec);
    const float* const pe = ce + P2P_PROGRAM_COLS;
    const int2* const terms = reinterpret_cast<const int2*>(pe + P2P_PROGRAM_COLS);
    const float* const al = a.grp_alpha[gi] + (b - 1) * K;
    const float* const P0 = slab + qi * P0S;
    float acc[KB][16];
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[kb][r] = ce[kb * 32 + acc_row(r, hh)] * sv[kb][r];
    for (int t = 0; t < tmax; ++t) {  // wave-uniform; padding terms add +0
      const int2* const plane = terms + t * P2P_PROGRAM_COLS;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int2 tm = plane[kb * 32 + acc_row(r, hh)];
          acc[kb][r] = acc[kb][r] + __int_as_float(tm.y) * P0[tm.x];
        }
    }
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int w = kb * 32 + acc_row(r, hh);
        if (w < K) {
          const float pb = sv[kb][r];
          const float R = pe[w] * acc[kb][r];
          const float aw = al[w];
          sv[kb][r] = aw * R + (1.f - aw) * pb;
        }
      }
  }

  P2P_CROSS_STAMP(13)
  // ---- AttentionStore epilogue: post-edit maps, whole rows through the wave's slab
  if (stored) {
    // the slab is this wave's own region: wave-level ordering suffices (the dense tile under it
    // died at the post-R barrier; the term-plane path's P0 gather reads only this wave's slab)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // key blocks wholly below K write every register (one branch per block, wave-uniform); only
    // the block that crosses K checks its keys (a per-element check costs a compare and two exec
    // updates around every LDS write)
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      if (kb * 32 + 32 <= K) {
#pragma unroll
        for (int r = 0; r < 16; ++r) slab[qi * K + kb * 32 + acc_row(r, hh)] = sv[kb][r];
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int w = kb * 32 + acc_row(r, hh);
          if (w < K) slab[qi * K + w] = sv[kb][r];
        }
      }
    }
    P2P_CROSS_STAMP(16)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    P2P_CROSS_STAMP(17)
    const int rows = min(32, a.P - p0w);
    // LocalBlend's word sums of these rows (alpha- and substruct-weighted), folded here so the
    // blend never re-reads the maps: each lane sums the words it holds in registers (runs of four
    // consecutive words, weights read 16 bytes at a time), the two lane halves of a row add, and
    // lanes 0-31 write the alpha sum, 32-63 the substruct sum.  (A pairwise order instead of
    // blend_wordsum_kernel's sequential one: the fold is already a measured summation-order
    // deviation from the map path; the sequential chain cost ~3k cycles per workgroup.)
    if (blend_on) {
      const bool has_sub = a.grp_bsub[gi] != nullptr;
      // (no key checks: past K both the probabilities -- masked to exact zeros by every path --
      // and the weights are 0, so those terms add +0; runs past the short tail are skipped)
      float sa = 0.f, ss = 0.f;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          if (kb == KB - 1 && g4 >= 2 && short_tail) continue;   // registers 8..15: keys >= 80
          const int w0 = kb * 32 + 8 * g4 + 4 * hh;
          const f32x4_t ta = *reinterpret_cast<const f32x4_t*>(&btab[0][w0]);
          const f32x4_t ts = *reinterpret_cast<const f32x4_t*>(&btab[1][w0]);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            sa = fmaf(sv[kb][4 * g4 + j], ta[j], sa);
            ss = fmaf(sv[kb][4 * g4 + j], ts[j], ss);
          }
        }
      sa += other_half(sa);
      ss += other_half(ss);
      if (qi < rows) {
        const float acc = hh == 0 ? sa : (has_sub ? ss : 0.f);
        *bdst = a.store_accumulate ? (touch_when == 3 ? bsum_old : *bdst) + acc : acc;
      }
    }
    P2P_CROSS_STAMP(18)
    if (rows > 0) {
      float* g = a.store + ((int64_t)(slot + h) * a.P + p0w) * (int64_t)K;
      const int count = rows * K;
      if (touch_when == 3 && rmw_vec && a.store_accumulate) {
        rmw_add_store<kRmwF4>(g, slab, count, lane, rmwbuf);
      } else if (((uintptr_t)g & 15) == 0 && (count & 3) == 0) {
        store_rows_rmw<32 * KR / 4>(g, slab, count, a.store_accumulate != 0, lane);
        // keeps the prefetch touches alive (never true: a running sum of probabilities is finite)
        if (__builtin_expect(touch0 == -INFINITY || touch1 == -INFINITY, 0)) g[0] = touch0 + touch1;
      } else {
        for (int i = lane; i < count; i += 64) g[i] = a.store_accumulate ? g[i] + slab[i] : slab[i];
      }
    }
  }

  P2P_CROSS_STAMP(14)
  // ---- O = P' V
  f32x16_t O[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) O[dt] = f32x16_t{};
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) pv_block<VS, NDT>(MP{}, O, Vs, kb * 32, sv[kb], lane);
  P2P_CROSS_STAMP(15)
  store_o(O, 1.f);
}

// ====================================================================== launchers
template <typename IO, typename MQ, typename MP, int D, int BK, int W>
static void launch_fused(const SelfArgs& a, hipStream_t st) {
  SelfArgs b = a;
  b.n_qtiles = (a.P + 32 * W - 1) / (32 * W);
  dim3 grid(b.n_qtiles * a.H * a.N), block(64 * W);
  constexpr bool kOnes = ((D + 31) / 32 * 32) > D;
  if (a.n_maps > 0)  // the lse feeds stored maps: exact f32 row sums
    launch_kernel((self_attn_fused_kernel<IO, MQ, MP, D, BK, W, true>), grid, block, 0, st, b);
  else if constexpr (kOnes && MP::kElemBytes == 2) {
    // O only (no lse): no per-tile max
    if (a.lse == nullptr)
      launch_kernel((self_attn_fused_kernel<IO, MQ, MP, D, BK, W, false, true>), grid, block, 0, st, b);
    else
      launch_kernel((self_attn_fused_kernel<IO, MQ, MP, D, BK, W>), grid, block, 0, st, b);
  } else
    launch_kernel((self_attn_fused_kernel<IO, MQ, MP, D, BK, W>), grid, block, 0, st, b);
}

template <typename IO, typename MQ, int D, int BK, int W, int QB, bool F16 = false, bool PIPE = false,
          bool PRIO = false>
static void launch_multi(const SelfArgs& a, hipStream_t st) {
  SelfArgs b = a;
  b.n_qtiles = (a.P + 32 * W * QB - 1) / (32 * W * QB);
  dim3 grid(b.n_qtiles * a.H * a.N), block(64 * W);
  launch_kernel((self_attn_multi_kernel<IO, MQ, D, BK, W, QB, F16, PIPE, PRIO>), grid, block, 0, st, b);
}

template <typename IO, typename MQ, typename MP, int D>
static hipError_t launch_self_d(const SelfArgs& a, int mode, hipStream_t st) {
  constexpr int BK = (D >= 128 || MP::kElemBytes == 4) ? 32 : 64;
  if constexpr (MP::kElemBytes == 2 && D == 40) {
    // d = 40 on the bf16 pipe, nothing but O wanted (G1/G7 without kept maps or autograd)
    if (mode == MODE_FUSED && a.lse == nullptr && a.n_maps == 0 && a.P > 64) {
      constexpr bool kF16 = MQ::planes == 1 && sizeof(IO) == 2;
      // bf16 inputs: the software-pipelined F16-form kernel (p2p_self40.hip)
      if constexpr (kF16)
        if (self40_eligible(a, 40)) return (hipError_t)run_self40(a, 40, st);
      if (a.P >= 2048) {
        // f32 inputs (split-bf16 Q K^T, two K planes): the multi-block kernel, 128-key tiles;
        // bf16 inputs with K < 256: the same with the F16 form
        if constexpr (MQ::planes == 1) launch_multi<IO, MQ, D, 256, 8, 2, kF16, true>(a, st);
        else launch_multi<IO, MQ, D, 128, 8, 2, kF16>(a, st);
        return hipGetLastError();
      }
    }
  }
  if constexpr (MP::kElemBytes == 2 && D == 80 && MQ::planes == 1 && sizeof(IO) == 2) {
    // d = 80, bf16 inputs, nothing but O wanted (G2/G6 without kept maps or autograd): the
    // software-pipelined kernel of p2p_self40.hip in its bf16 form
    if (mode == MODE_FUSED && a.lse == nullptr && a.n_maps == 0 && self40_eligible(a, 80))
      return (hipError_t)run_self40(a, 80, st);
  }
  if constexpr (MP::kElemBytes == 2 && D == 160 && MQ::planes == 1 && sizeof(IO) == 2) {
    // d = 160, bf16 inputs, O only (the 16x16 / 8x8 layers without kept maps or autograd): the
    // waves of a 32-query workgroup split the keys (p2p_selfsplit.hip, K <= 128), or the per-tile
    // kernel with its 4-stage DMA ring (K = 256)
    if (mode == MODE_FUSED && self_split_eligible(a, D)) return (hipError_t)run_self_split(a, D, st);
    if (mode == MODE_FUSED && self_ring_eligible(a, D)) return (hipError_t)run_self_ring(a, D, st);
  }
  if (mode == MODE_FUSED) {
    if constexpr (BK == 64 && (D == 40 || D == 80)) {
      if (a.P > 64) {
        // 8 waves x 32 query rows per workgroup, 64-key tiles (measured best at d = 40 and within
        // 2 % of best at d = 80: tools/attn_bench.py, profiles/)
        launch_fused<IO, MQ, MP, D, 64, 8>(a, st);
        return hipGetLastError();
      }
    }
    if (a.P <= 64) launch_fused<IO, MQ, MP, D, BK, 2>(a, st);
    else launch_fused<IO, MQ, MP, D, BK, 4>(a, st);
    return hipGetLastError();
  }
  // MODE_PV: the materialise protocol's P V
  SelfArgs b = a;
  constexpr int W = 4;
  b.n_qtiles = (a.P + 32 * W - 1) / (32 * W);
  dim3 grid(b.n_qtiles * a.H * a.N), block(64 * W);
  launch_kernel((self_pv_kernel<IO, MP, D, BK, W>), grid, block, 0, st, b);
  return hipGetLastError();
}

template <typename IO, typename MQ, typename MP, int D, int W>
static hipError_t launch_cross_w(const CrossArgs& a, hipStream_t st) {
  CrossArgs b = a;
  b.n_qtiles = (a.P + 32 * W - 1) / (32 * W);
  // the slab holds a [32, K] f32 block per wave: stride K | 1 (odd, so the 32 rows of one
  // column hit distinct banks) for the edit gather, K for the store rows
  b.slab_stride = a.K | 1;
  // the dense path (bf16 PV only) stages the mapper tile in the same dynamic region the slab
  // uses later (the tile is dead before any store)
  constexpr bool kDense = MP::kElemBytes == 2;
  const bool dense = kDense && a.edit_dense && !a.edit_terms;
  b.slab = (a.any_store || ((a.edit_terms || a.edit_dense) && !dense)) ? 1 : 0;
  size_t dyn = b.slab ? (size_t)W * 32 * b.slab_stride * sizeof(float) : 0;
  const size_t tile = (size_t)P2P_PROGRAM_DENSE * P2P_PROGRAM_DENSE * sizeof(uint16_t);
  if (dense && dyn < tile) dyn = tile;
  dim3 grid(b.n_qtiles * a.H * a.N), block(64 * W);
  if (dense)
    launch_kernel((cross_attn_kernel<IO, MQ, MP, D, W, kDense>), grid, block, dyn, st, b);
  else
    launch_kernel((cross_attn_kernel<IO, MQ, MP, D, W, false>), grid, block, dyn, st, b);
  return hipGetLastError();
}

template <typename IO, typename MQ, typename MP, int D>
static hipError_t launch_cross_d(const CrossArgs& a, hipStream_t st) {
  return launch_cross_w<IO, MQ, MP, D, (MP::kElemBytes == 4 && D >= 128) ? 2 : 4>(a, st);
}

#define P2P_FOR_EACH_D(X) X(8) X(16) X(32) X(40) X(64) X(80) X(128) X(160)

template <typename IO, typename MQ, typename MP>
static int dispatch_self(const SelfArgs& a, int d, int mode, hipStream_t st) {
  switch (d) {
#define P2P_CASE(DD) case DD: return (int)launch_self_d<IO, MQ, MP, DD>(a, mode, st);
    P2P_FOR_EACH_D(P2P_CASE)
#undef P2P_CASE
    default: return P2P_E_HEAD_DIM;
  }
}

template <typename IO, typename MQ, int D>
static hipError_t launch_self_maps_d(const SelfArgs& a, hipStream_t st) {
  SelfArgs b = a;
  // keys per wave: a quarter of the row (whole 32-key blocks), at most 256 -> a workgroup
  // spans up to 1024 keys; wider rows take more key groups
  const int kw = min(256, ((a.K + 3) / 4 + 31) / 32 * 32);
  const int n_kgroups = (a.K + 4 * kw - 1) / (4 * kw);
  b.n_qtiles = (a.P + 31) / 32;
  dim3 grid(n_kgroups * b.n_qtiles * a.H * a.n_maps), block(256);
  // non-temporal running-sum accesses (the map streams through once per step: -7.5 % at G2 with
  // the maps HBM-resident; two key blocks per step measured +2 %, not instantiated)
  launch_kernel((self_maps_kernel<IO, MQ, D, 1, true>), grid, block, 0, st, b, kw, n_kgroups);
  return hipGetLastError();
}

template <typename IO, typename MQ, int D>
static hipError_t launch_self_probs_d(const SelfArgs& a, hipStream_t st) {
  SelfArgs b = a;
  const int kw = ((a.K + 3) / 4 + 31) / 32 * 32;  // keys per wave: a quarter of the row
  b.n_qtiles = (a.P + 31) / 32;
  dim3 grid(b.n_qtiles * a.H * a.N), block(256);
  // non-temporal probability stores (a write-once stream: G1 1.33 -> 1.04 ms, G2 118 -> 104 us)
  launch_kernel((self_probs_kernel<IO, MQ, D, true>), grid, block, 0, st, b, kw);
  return hipGetLastError();
}

template <typename IO, typename MQ>
static int dispatch_self_probs(const SelfArgs& a, int d, hipStream_t st) {
  switch (d) {
#define P2P_CASE(DD) case DD: return (int)launch_self_probs_d<IO, MQ, DD>(a, st);
    P2P_FOR_EACH_D(P2P_CASE)
#undef P2P_CASE
    default: return P2P_E_HEAD_DIM;
  }
}

template <typename IO, typename MQ>
static int dispatch_self_maps(const SelfArgs& a, int d, hipStream_t st) {
  switch (d) {
#define P2P_CASE(DD) case DD: return (int)launch_self_maps_d<IO, MQ, DD>(a, st);
    P2P_FOR_EACH_D(P2P_CASE)
#undef P2P_CASE
    default: return P2P_E_HEAD_DIM;
  }
}

template <typename IO, typename MQ, typename MP>
static int dispatch_cross(const CrossArgs& a, int d, hipStream_t st) {
  switch (d) {
#define P2P_CASE(DD) case DD: return (int)launch_cross_d<IO, MQ, MP, DD>(a, st);
    P2P_FOR_EACH_D(P2P_CASE)
#undef P2P_CASE
    default: return P2P_E_HEAD_DIM;
  }
}

// Precision selection: exact-f32 check mode; bf16 pipe on f32 inputs (split-bf16 QK^T so the
// logits keep f32 grade, bf16 PV); bf16 inputs (one bf16 MFMA per step, exact products).
int run_self(const SelfArgs& a, int io_dtype, int compute, int d, int mode, hipStream_t st) {
  if (compute == P2P_COMPUTE_F32) {
    if (io_dtype != P2P_DTYPE_F32) return P2P_E_DTYPE;
    return dispatch_self<float, QkF32, MmaF32>(a, d, mode, st);
  }
  if (io_dtype == P2P_DTYPE_F32) return dispatch_self<float, QkSplit, MmaBf16>(a, d, mode, st);
  return dispatch_self<uint16_t, QkBf16<uint16_t>, MmaBf16>(a, d, mode, st);
}

int run_self_probs(const SelfArgs& a, int io_dtype, int compute, int d, hipStream_t st) {
  if (compute == P2P_COMPUTE_F32) {
    if (io_dtype != P2P_DTYPE_F32) return P2P_E_DTYPE;
    return dispatch_self_probs<float, QkF32>(a, d, st);
  }
  if (io_dtype == P2P_DTYPE_F32) return dispatch_self_probs<float, QkSplit>(a, d, st);
  return dispatch_self_probs<uint16_t, QkBf16<uint16_t>>(a, d, st);
}

int run_self_maps(const SelfArgs& a, int io_dtype, int compute, int d, hipStream_t st) {
  if (a.n_maps < 1) return 0;
  if (compute == P2P_COMPUTE_F32) {
    if (io_dtype != P2P_DTYPE_F32) return P2P_E_DTYPE;
    return dispatch_self_maps<float, QkF32>(a, d, st);
  }
  if (io_dtype == P2P_DTYPE_F32) return dispatch_self_maps<float, QkSplit>(a, d, st);
  return dispatch_self_maps<uint16_t, QkBf16<uint16_t>>(a, d, st);
}

int run_cross(const CrossArgs& a, int io_dtype, int compute, int d, hipStream_t st) {
  if (compute == P2P_COMPUTE_F32) {
    if (io_dtype != P2P_DTYPE_F32) return P2P_E_DTYPE;
    return dispatch_cross<float, QkF32, MmaF32>(a, d, st);
  }
  if (io_dtype == P2P_DTYPE_F32) return dispatch_cross<float, QkSplit, MmaBf16>(a, d, st);
  if (cross_group_eligible(a, d)) return run_cross_group(a, d, st);
  return dispatch_cross<uint16_t, QkBf16<uint16_t>, MmaBf16>(a, d, st);
}

}  // namespace p2p

#ifdef P2P_EXPERIMENTS
// dst == nullptr: clear the stamps
extern "C" int p2p_diag_cross_stamps(void* dst, int64_t bytes) {
  const int64_t n = (int64_t)sizeof(p2p::g_cross_stamps);
  if (dst == nullptr) {
    void* p = nullptr;
    hipError_t e = hipGetSymbolAddress(&p, HIP_SYMBOL(p2p::g_cross_stamps));
    return e != hipSuccess ? (int)e : (int)hipMemset(p, 0, n);
  }
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(p2p::g_cross_stamps), bytes < n ? bytes : n, 0, hipMemcpyDeviceToHost);
}
#endif
