// Attention backward for null-text inversion (null_text.py:574-606: every Adam step on the null
// embedding back-propagates through all 32 patched attentions of the U-Net, ptp_utils.py:183-208).
//
//   P = exp2(c S - lse)              (recomputed; lse from the forward, c = scale * log2 e)
//   dV = P^T dO,  dP = dO V^T,  dS = P o (dP - delta),  delta = rowsum(dO o O)
//   dQ = scale dS K,  dK = scale dS^T Q
//
// Two passes, no atomics on dQ:
//   bwd_dq_kernel  -- one wave per 32 queries (query on the lane, as the forward): S^T = K Q^T and
//                     dP^T = V dO^T on 32x32x16 MFMAs, then dQ^T += K^T dS^T with the dS^T
//                     accumulator as the B operand and K^T from a transposable LDS image;
//   bwd_dkv_kernel -- one wave per 32 keys (key on the lane): S = Q K^T, dP = dO V^T, then
//                     dV^T += dO^T P and dK^T += Q^T dS with P / dS as B operands.
// Cross-attention (77 keys) and small batches have too few key tiles to fill the chip, so the
// key/value pass splits the queries over workgroups: each split stores its partial dK/dV (f32)
// into a workspace and bwd_kv_reduce_kernel adds them in split order (deterministic; the f32
// atomics this replaced serialised on the shared rows: 3-4x slower).
#include <cstdlib>

#include "p2p_device.h"
#include "p2p_kernels.h"

namespace p2p {

// delta[n*H + h][p] = sum_d dO[n, p, h*D + d] O[n, p, h*D + d]
template <typename IO, int D>
__global__ __launch_bounds__(256) void bwd_delta_kernel(BwdArgs a) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)a.N * a.H * a.P) return;
  const int p = (int)(idx % a.P);
  const int nh = (int)(idx / a.P);
  const int h = nh % a.H, n = nh / a.H;
  const IO* o = static_cast<const IO*>(a.o) + (int64_t)n * a.bso + (int64_t)p * a.ldo + h * D;
  const IO* g = static_cast<const IO*>(a.dout) + (int64_t)n * a.bsdo + (int64_t)p * a.lddo + h * D;
  float acc = 0.f;
#pragma unroll
  for (int c = 0; c < D / 8; ++c) {
    Chunk8<IO> x, y;
    x.load(o + 8 * c);
    y.load(g + 8 * c);
    float tx[8], ty[8];
    x.store(tx);
    y.store(ty);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = fmaf(tx[j], ty[j], acc);
  }
  a.delta[idx] = acc;
}

// 8 consecutive elements of a row as a bf16 fragment (zeros past D or for rows out of range)
template <typename IO, int D>
__device__ __forceinline__ short8_t row_frag(const IO* row, int col, bool ok) {
  if (!ok || col >= D) return short8_t{0, 0, 0, 0, 0, 0, 0, 0};
  Chunk8<IO> c;
  c.load(row + col);
  uint16_t t[8] __attribute__((aligned(16)));
  c.store(t);
  return *reinterpret_cast<const short8_t*>(t);
}

// Tile staging shared by both passes: `rows` rows of two [*, H*D] tensors (X, Y) into a row
// image [T][KS] (ds_read_b128 reads) and a transposable image [T][VS] (ds_read_b64_tr_b16),
// both bf16; rows past `limit` are zeros.
template <typename IO, int D, int T, int NT>
struct TileStage {
  static constexpr int DK = (D + 15) / 16 * 16;
  static constexpr int DV = (D + 31) / 32 * 32;
  static constexpr int KS = KStride<DK, 2>::value;
  static constexpr int VS = VStrideBf16<DV>::value;
  static constexpr int CPR = D / 8;
  static constexpr int NCH = (T * CPR + NT - 1) / NT;
  Chunk8<IO> xr[NCH], yr[NCH];
  __device__ __forceinline__ void load(const IO* x, int64_t ldx, const IO* y, int64_t ldy, int row0, int limit,
                                       int tid) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = tid + i * NT;
      const int r = c / CPR, ch = c - r * CPR;
      if (c < T * CPR && row0 + r < limit) {
        xr[i].load(x + (int64_t)(row0 + r) * ldx + ch * 8);
        yr[i].load(y + (int64_t)(row0 + r) * ldy + ch * 8);
      } else {
        xr[i].clear();
        yr[i].clear();
      }
    }
  }
  // images: xrow [T][KS], xtr [T][VS], yrow [T][KS], ytr [T][VS] (any may be null)
  __device__ __forceinline__ void write(uint16_t* xrow, uint16_t* xtr, uint16_t* yrow, uint16_t* ytr, int tid) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = tid + i * NT;
      if (c < T * CPR) {
        const int r = c / CPR, ch = c - r * CPR;
        if (xrow) xr[i].store(xrow + r * KS + ch * 8);
        if (xtr) xr[i].store(xtr + r * VS + ch * 8);
        if (yrow) yr[i].store(yrow + r * KS + ch * 8);
        if (ytr) yr[i].store(ytr + r * VS + ch * 8);
      }
    }
  }
};

// ---------------------------------------------------------------------------- dQ pass
template <typename IO, int D, int T, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void bwd_dq_kernel(BwdArgs a) {
  using St = TileStage<IO, D, T, 64 * WAVES>;
  constexpr int NKT = St::DK / 16;
  constexpr int NDT = St::DV / 32;
  constexpr int KS = St::KS, VS = St::VS;
  constexpr int NSB = T / 32;
  constexpr int IMG = T * (2 * KS + VS);          // Krow, Vrow, Ktr per buffer (elements)
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * IMG];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hh = lane >> 5, qi = lane & 31;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int qt = logical % a.n_tiles;
  const int nh = logical / a.n_tiles;
  const int h = nh % a.H, n = nh / a.H;
  const int p = qt * 32 * WAVES + wave * 32 + qi;
  const bool prow = p < a.P;
  const float c = a.scale_log2;

  const IO* qp = static_cast<const IO*>(a.q) + (int64_t)n * a.bsq + h * D;
  const IO* gp = static_cast<const IO*>(a.dout) + (int64_t)n * a.bsdo + h * D;
  const IO* kp = static_cast<const IO*>(a.k) + (int64_t)n * a.bsk + h * D;
  const IO* vp = static_cast<const IO*>(a.v) + (int64_t)n * a.bsv + h * D;

  for (int i = tid; i < IMG; i += 64 * WAVES) reinterpret_cast<uint32_t*>(smem)[i] = 0u;  // both buffers

  short8_t qf[NKT], gf[NKT];
#pragma unroll
  for (int t = 0; t < NKT; ++t) {
    qf[t] = row_frag<IO, D>(qp + (int64_t)p * a.ldq, 16 * t + 8 * hh, prow);
    gf[t] = row_frag<IO, D>(gp + (int64_t)p * a.lddo, 16 * t + 8 * hh, prow);
  }
  const float lse = prow ? a.lse[(int64_t)nh * a.P + p] : INFINITY;
  const float dlt = prow ? a.delta[(int64_t)nh * a.P + p] : 0.f;

  f32x16_t dQ[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) dQ[dt] = f32x16_t{};

  St st;
  const int ntiles = (a.K + T - 1) / T;
  __syncthreads();
  st.load(kp, a.ldk, vp, a.ldv, 0, a.K, tid);
  st.write(smem, smem + 2 * T * KS, smem + T * KS, nullptr, tid);
  __syncthreads();
  for (int kt = 0; kt < ntiles; ++kt) {
    uint16_t* buf = smem + (kt & 1) * IMG;
    const uint16_t* Krow = buf;
    const uint16_t* Vrow = buf + T * KS;
    const uint16_t* Ktr = buf + 2 * T * KS;
    if (kt + 1 < ntiles) st.load(kp, a.ldk, vp, a.ldv, (kt + 1) * T, a.K, tid);
#pragma unroll
    for (int sb = 0; sb < NSB; ++sb) {
      f32x16_t S = {}, dP = {};
#pragma unroll
      for (int t = 0; t < NKT; ++t) {
        const short8_t kf = *reinterpret_cast<const short8_t*>(Krow + (sb * 32 + qi) * KS + 16 * t + 8 * hh);
        const short8_t vf = *reinterpret_cast<const short8_t*>(Vrow + (sb * 32 + qi) * KS + 16 * t + 8 * hh);
        S = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, kf),
                                                    __builtin_bit_cast(bf16x8_t, qf[t]), S, 0, 0, 0);
        dP = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, vf),
                                                     __builtin_bit_cast(bf16x8_t, gf[t]), dP, 0, 0, 0);
      }
      float ds[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kt * T + sb * 32 + acc_row(r, hh);
        const float pr = key < a.K ? fast_exp2(fmaf(S[r], c, -lse)) : 0.f;
        ds[r] = pr * (dP[r] - dlt);
      }
      pv_block<VS, NDT>(MmaBf16{}, dQ, Ktr, sb * 32, ds, lane);
    }
    if (kt + 1 < ntiles) {
      uint16_t* nb = smem + ((kt + 1) & 1) * IMG;
      st.write(nb, nb + 2 * T * KS, nb + T * KS, nullptr, tid);
    }
    __syncthreads();
  }
  if (prow) {
    IO* dq = static_cast<IO*>(a.dq) + (int64_t)n * a.bsdq + (int64_t)p * a.lddq + h * D;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int dd = dt * 32 + 8 * g + 4 * hh;
        if (dd < D)
          store4(dq + dd, dQ[dt][4 * g] * a.scale, dQ[dt][4 * g + 1] * a.scale, dQ[dt][4 * g + 2] * a.scale,
                 dQ[dt][4 * g + 3] * a.scale);
      }
  }
}

// ---------------------------------------------------------------------------- dK / dV pass
// WANT: 1 = dV, 2 = dK, 3 = both.  OUT: element type of dk/dv (IO or float); with a query split
// the partials go to the f32 workspace instead.
template <typename IO, typename OUT, int D, int T, int WAVES, int WANT>
__global__ __launch_bounds__(64 * WAVES) void bwd_dkv_kernel(BwdArgs a) {
  using St = TileStage<IO, D, T, 64 * WAVES>;
  constexpr int NKT = St::DK / 16;
  constexpr int NDT = St::DV / 32;
  constexpr int KS = St::KS, VS = St::VS;
  constexpr int NSB = T / 32;
  constexpr bool kDV = WANT & 1, kDK = WANT & 2;
  constexpr int IMG = T * (2 * KS + 2 * VS) + 2 * T * 2;   // Qrow, dOrow, Qtr, dOtr + lse/delta (f32)
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * IMG];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hh = lane >> 5, ki = lane & 31;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int split = logical % a.kv_split;
  const int rest = logical / a.kv_split;
  const int kt0 = rest % a.n_tiles;
  const int nh = rest / a.n_tiles;
  const int h = nh % a.H, n = nh / a.H;
  const int key = kt0 * 32 * WAVES + wave * 32 + ki;
  const bool krow = key < a.K;
  const float c = a.scale_log2;

  const IO* qp = static_cast<const IO*>(a.q) + (int64_t)n * a.bsq + h * D;
  const IO* gp = static_cast<const IO*>(a.dout) + (int64_t)n * a.bsdo + h * D;
  const IO* kp = static_cast<const IO*>(a.k) + (int64_t)n * a.bsk + h * D;
  const IO* vp = static_cast<const IO*>(a.v) + (int64_t)n * a.bsv + h * D;
  const float* lsep = a.lse + (int64_t)nh * a.P;
  const float* dltp = a.delta + (int64_t)nh * a.P;

  for (int i = tid; i < IMG; i += 64 * WAVES) reinterpret_cast<uint32_t*>(smem)[i] = 0u;

  short8_t kf[NKT], vf[NKT];
#pragma unroll
  for (int t = 0; t < NKT; ++t) {
    kf[t] = row_frag<IO, D>(kp + (int64_t)key * a.ldk, 16 * t + 8 * hh, krow);
    if constexpr (kDK) vf[t] = row_frag<IO, D>(vp + (int64_t)key * a.ldv, 16 * t + 8 * hh, krow);
  }
  f32x16_t dV[kDV ? NDT : 1], dK[kDK ? NDT : 1];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) {
    if constexpr (kDV) dV[dt] = f32x16_t{};
    if constexpr (kDK) dK[dt] = f32x16_t{};
  }

  // this workgroup's query range
  const int per = ((a.P + a.kv_split - 1) / a.kv_split + T - 1) / T * T;
  const int q_begin = split * per;
  const int q_end = min(a.P, q_begin + per);
  const int ntiles = q_end > q_begin ? (q_end - q_begin + T - 1) / T : 0;

  St st;
  auto stage_rows = [&](int qt, uint16_t* b) {
    const int row0 = q_begin + qt * T;
    st.write(b, b + 2 * T * KS, b + T * KS, b + 2 * T * KS + T * VS, tid);
    float* lb = reinterpret_cast<float*>(b + T * (2 * KS + 2 * VS));
    for (int i = tid; i < T; i += 64 * WAVES) {
      const int q = row0 + i;
      lb[i] = q < q_end ? lsep[q] : INFINITY;       // rows past the range: p = 0
      lb[T + i] = q < q_end ? dltp[q] : 0.f;
    }
  };
  __syncthreads();
  if (ntiles > 0) {
    st.load(qp, a.ldq, gp, a.lddo, q_begin, q_end, tid);
    stage_rows(0, smem);
  }
  __syncthreads();
  for (int qt = 0; qt < ntiles; ++qt) {
    uint16_t* buf = smem + (qt & 1) * IMG;
    const uint16_t* Qrow = buf;
    const uint16_t* Grow = buf + T * KS;
    const uint16_t* Qtr = buf + 2 * T * KS;
    const uint16_t* Gtr = buf + 2 * T * KS + T * VS;
    const float* lb = reinterpret_cast<const float*>(buf + T * (2 * KS + 2 * VS));
    if (qt + 1 < ntiles) st.load(qp, a.ldq, gp, a.lddo, q_begin + (qt + 1) * T, q_end, tid);
#pragma unroll
    for (int sb = 0; sb < NSB; ++sb) {
      f32x16_t S = {}, dP = {};
#pragma unroll
      for (int t = 0; t < NKT; ++t) {
        const short8_t qa = *reinterpret_cast<const short8_t*>(Qrow + (sb * 32 + ki) * KS + 16 * t + 8 * hh);
        S = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, qa),
                                                    __builtin_bit_cast(bf16x8_t, kf[t]), S, 0, 0, 0);
        if constexpr (kDK) {
          const short8_t ga = *reinterpret_cast<const short8_t*>(Grow + (sb * 32 + ki) * KS + 16 * t + 8 * hh);
          dP = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, ga),
                                                       __builtin_bit_cast(bf16x8_t, vf[t]), dP, 0, 0, 0);
        }
      }
      float pr[16], ds[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qr = sb * 32 + acc_row(r, hh);   // query of register r (row of S)
        pr[r] = fast_exp2(fmaf(S[r], c, -lb[qr]));
        if constexpr (kDK) ds[r] = pr[r] * (dP[r] - lb[T + qr]);
      }
      if constexpr (kDV) pv_block<VS, NDT>(MmaBf16{}, dV, Gtr, sb * 32, pr, lane);
      if constexpr (kDK) pv_block<VS, NDT>(MmaBf16{}, dK, Qtr, sb * 32, ds, lane);
    }
    if (qt + 1 < ntiles) stage_rows(qt + 1, smem + ((qt + 1) & 1) * IMG);
    __syncthreads();
  }
  if (!krow) return;
  const int64_t C = (int64_t)a.H * D;
  auto emit = [&](void* base, int64_t bs, int64_t ld, int which, const f32x16_t (&acc)[NDT], float mul) {
    if (a.kv_split > 1) {                       // partial of this split -> workspace (f32)
      float* dst = a.ws + (((int64_t)which * a.kv_split + split) * a.N + n) * a.K * C + (int64_t)key * C + h * D;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int dd = dt * 32 + 8 * g + 4 * hh;
          if (dd < D)
            store4(dst + dd, acc[dt][4 * g] * mul, acc[dt][4 * g + 1] * mul, acc[dt][4 * g + 2] * mul,
                   acc[dt][4 * g + 3] * mul);
        }
      return;
    }
    OUT* dst = static_cast<OUT*>(base) + (int64_t)n * bs + (int64_t)key * ld + h * D;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int dd = dt * 32 + 8 * g + 4 * hh;
        if (dd < D)
          store4(dst + dd, acc[dt][4 * g] * mul, acc[dt][4 * g + 1] * mul, acc[dt][4 * g + 2] * mul,
                 acc[dt][4 * g + 3] * mul);
      }
  };
  if constexpr (kDV) emit(a.dv, a.bsdv, a.lddv, 1, dV, 1.f);
  if constexpr (kDK) emit(a.dk, a.bsdk, a.lddk, 0, dK, a.scale);
}

// dk / dv [N, K, C] = sum over the splits (in split order) of the workspace partials
template <typename OUT>
__global__ __launch_bounds__(256) void bwd_kv_reduce_kernel(BwdArgs a, int64_t n4) {
  const int64_t plane = n4 * 4;                 // N * K * C
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
#pragma unroll
    for (int which = 0; which < 2; ++which) {
      const float* src = a.ws + (int64_t)which * a.kv_split * plane + 4 * i;
      f32x4_t s = *reinterpret_cast<const f32x4_t*>(src);
      for (int sp = 1; sp < a.kv_split; ++sp) s += *reinterpret_cast<const f32x4_t*>(src + sp * plane);
      OUT* dst = static_cast<OUT*>(which ? a.dv : a.dk) + 4 * i;
      store4(dst, s[0], s[1], s[2], s[3]);
    }
  }
}

// ---------------------------------------------------------------------------- launchers
template <typename IO, typename OUT, int D, int T, int W, int WANT>
static void launch_dkv(const BwdArgs& a, hipStream_t st) {
  BwdArgs b = a;
  b.n_tiles = (a.K + 32 * W - 1) / (32 * W);
  dim3 grid(b.n_tiles * a.N * a.H * a.kv_split), block(64 * W);
  launch_kernel((bwd_dkv_kernel<IO, OUT, D, T, W, WANT>), grid, block, 0, st, b);
}

constexpr int kBwdWaves = 4;
template <int D>
struct BwdTile {
  static constexpr int T = D >= 128 ? 32 : 64;
};

// query split of the key/value pass: double while the key workgroups leave the chip idle
static int kv_split_for(int N, int H, int P, int K, int T) {
  const int key_wgs = (K + 32 * kBwdWaves - 1) / (32 * kBwdWaves) * N * H;
  int split = 1;
  while (key_wgs * split < 512 && split * 2 * T <= P) split *= 2;
  return split;
}

int bwd_kv_split(int N, int H, int P, int K, int d) {
  return kv_split_for(N, H, P, K, d >= 128 ? 32 : 64);
}

// d >= 128: dV and dK in two passes (each keeps 5 O^T tiles of accumulators, not 10)
template <typename IO, typename OUT, int D, int T, int W>
static void launch_kv_out(const BwdArgs& a, hipStream_t st) {
  if constexpr (D >= 128) {
    launch_dkv<IO, OUT, D, T, W, 1>(a, st);
    launch_dkv<IO, OUT, D, T, W, 2>(a, st);
  } else {
    launch_dkv<IO, OUT, D, T, W, 3>(a, st);
  }
  if (a.kv_split > 1) {
    const int64_t n4 = (int64_t)a.N * a.K * a.H * D / 4;
    int64_t blocks = (n4 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    launch_kernel((bwd_kv_reduce_kernel<OUT>), dim3((unsigned)blocks), dim3(256), 0, st, a, n4);
  }
}

template <typename IO, int D>
static int launch_bwd_d(BwdArgs a, hipStream_t st) {
  constexpr int T = BwdTile<D>::T;
  constexpr int W = kBwdWaves;
  const int64_t nd = (int64_t)a.N * a.H * a.P;
  launch_kernel((bwd_delta_kernel<IO, D>), dim3((unsigned)((nd + 255) / 256)), dim3(256), 0, st, a);
  {
    BwdArgs b = a;
    b.n_tiles = (a.P + 32 * W - 1) / (32 * W);
    launch_kernel((bwd_dq_kernel<IO, D, T, W>), dim3(b.n_tiles * a.N * a.H), dim3(64 * W), 0, st, b);
  }
  // key/value pass: split the queries when the key tiles alone leave the chip idle
  a.kv_split = kv_split_for(a.N, a.H, a.P, a.K, T);
  if (a.kv_split > 1 && !a.ws) return P2P_E_ARG;   // the caller sized the workspace with bwd_kv_split
  if (a.kv_f32) launch_kv_out<IO, float, D, T, W>(a, st);
  else launch_kv_out<IO, IO, D, T, W>(a, st);
  return (int)hipGetLastError();
}

template <typename IO>
static int dispatch_bwd(const BwdArgs& a, int d, hipStream_t st) {
  switch (d) {
    case 40: return launch_bwd_d<IO, 40>(a, st);
    case 64: return launch_bwd_d<IO, 64>(a, st);
    case 80: return launch_bwd_d<IO, 80>(a, st);
    case 160: return launch_bwd_d<IO, 160>(a, st);
    default: return P2P_E_HEAD_DIM;
  }
}

int run_attn_bwd(const BwdArgs& a, int io_dtype, int d, hipStream_t st) {
  if (io_dtype == P2P_DTYPE_F32) return dispatch_bwd<float>(a, d, st);
  return dispatch_bwd<uint16_t>(a, d, st);
}

}  // namespace p2p
