// Key-split self-attention for the small SD geometries (16x16 and 8x8 layers: P = K <= 256 at
// d = 160, ptp_utils.py:195-206), bf16 inputs, O only (no kept maps, no autograd).
//
// At these sizes a (entry, head) is 256 x 256 x 160: the per-tile kernel walks 8 key tiles one
// global round trip after another, on 128 workgroups.  Here one workgroup = one 32-query block
// of one (entry, head), and its W waves split the KEYS: wave w owns keys [w KW, (w+1) KW).
// Every wave issues all of its loads at once -- its V rows go global -> LDS by DMA
// (global_load_lds, no VGPRs), its K rows straight into A-operand registers (key on the lane),
// Q into B-operand registers -- so the whole workgroup waits ONE round trip.  Then
//   S^T = K_w Q^T (MFMA), m_w = row max over the wave's keys, p = exp2(c s - m_w),
//   l_w = sum p (f32), O_w^T = V_w^T P^T (bf16 MFMA, V^T fragments by ds_read_b64_tr_b16),
// each wave writes (O_w, m_w, l_w) into its own (now dead) V region, one barrier, and the
// workgroup combines:  O = sum_w O_w 2^(m_w - M) / sum_w l_w 2^(m_w - M),  M = max_w m_w.
// qk_src implements the source-map injection (Q, K of entry qk_src[n], V of n).
#include "p2p_device.h"
#include "p2p_kernels.h"

namespace p2p {
namespace {

// D: head dim (multiple of 32, no padding columns); W waves x KBW 32-key blocks per wave
template <int D, int W, int KBW>
__global__ __launch_bounds__(64 * W, 2) void self_split_kernel(SelfArgs a) {
  static_assert(D % 32 == 0, "d tiles without padding");
  constexpr int NKT = D / 16;      // 16-deep k steps of Q K^T
  constexpr int NDT = D / 32;      // 32-row tiles of O^T
  constexpr int KW = 32 * KBW;     // keys per wave
  constexpr int VROW = D * 2;      // bytes per V row in LDS (dense: one DMA instruction = 1 KiB)
  static_assert(VStrideBf16<D>::value == D, "dense V rows are conflict-free for the transposed reads");
  constexpr int VREG = KW * VROW;  // bytes of one wave's V region
  constexpr int OS = D + 4;          // O partial row stride (floats): rows on distinct banks
  constexpr int OREG = 32 * OS * 4;  // its O partial: [32 rows][OS] f32
  constexpr int REG = VREG > OREG ? VREG : OREG;
  __shared__ __attribute__((aligned(16))) char smem[W * REG];
  __shared__ float ml[W][2][32];      // m_w, l_w of every row

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
  const int K = a.K;
  const float c = a.scale_log2;
  const int p = qt * 32 + qi;
  const bool prow = p < a.P;
  const int key0 = wave * KW;

  const uint16_t* const qp = static_cast<const uint16_t*>(a.q) + (int64_t)src * a.bsq + h * D;
  const uint16_t* const kp = static_cast<const uint16_t*>(a.k) + (int64_t)src * a.bsk + h * D;
  const uint16_t* const vp = static_cast<const uint16_t*>(a.v) + (int64_t)n * a.bsv + h * D;
  char* const reg = smem + wave * REG;
  uint16_t* const Vw = reinterpret_cast<uint16_t*>(reg);

  // ---- every load of this wave at once.  V: row r of the wave (key key0 + r) lands at
  // Vw + r * D; one DMA instruction moves 64 x 16 bytes = 1024 / VROW rows.  Rows past K read
  // row K-1 (their p is 0; any finite value will do).
  {
    constexpr int CPR = D / 8;                 // 16-byte chunks per row
    constexpr int NI = KW * CPR / 64;          // DMA instructions per wave
    static_assert((KW * CPR) % 64 == 0, "whole instructions");
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int cidx = i * 64 + lane;
      const int r = cidx / CPR;
      const int ch = cidx - r * CPR;
      const int key = min(key0 + r, K - 1);
      const uint16_t* g = vp + (int64_t)key * a.ldv + ch * 8;
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(g),
                                       reinterpret_cast<__attribute__((address_space(3))) void*>(
                                           reinterpret_cast<uintptr_t>(Vw + i * 512)),
                                       16, 0, 0);
    }
  }
  short8_t qf[NKT];
#pragma unroll
  for (int t = 0; t < NKT; ++t)
    qf[t] = prow ? *reinterpret_cast<const short8_t*>(qp + (int64_t)p * a.ldq + 16 * t + 8 * hh) : short8_t{};
  short8_t kf[KBW][NKT];
#pragma unroll
  for (int kb = 0; kb < KBW; ++kb) {
    const int key = min(key0 + kb * 32 + qi, K - 1);
#pragma unroll
    for (int t = 0; t < NKT; ++t) kf[kb][t] = *reinterpret_cast<const short8_t*>(kp + (int64_t)key * a.ldk + 16 * t + 8 * hh);
  }

  // ---- S^T = K_w Q^T, the wave's row max and exponentials
  float sv[KBW][16];
#pragma unroll
  for (int kb = 0; kb < KBW; ++kb) {
    f32x16_t acc = {};
#pragma unroll
    for (int t = 0; t < NKT; ++t)
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, kf[kb][t]),
                                                    __builtin_bit_cast(bf16x8_t, qf[t]), acc, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 16; ++r)
      sv[kb][r] = (key0 + kb * 32 + acc_row(r, hh) < K) ? acc[r] : -INFINITY;
  }
  float mx = -INFINITY;
#pragma unroll
  for (int kb = 0; kb < KBW; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sv[kb][r]);
  mx = fmaxf(mx, other_half(mx)) * c;   // every wave owns >= 1 key below K: mx is finite
  float ls = 0.f;
#pragma unroll
  for (int kb = 0; kb < KBW; ++kb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float e = fast_exp2(fmaf(sv[kb][r], c, -mx));
      sv[kb][r] = e;
      ls += e;
    }
  ls += other_half(ls);

  // ---- O_w^T = V_w^T P^T once the wave's V rows have landed
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the DMA (and every other load) retired
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  f32x16_t O[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) O[dt] = f32x16_t{};
#pragma unroll
  for (int kb = 0; kb < KBW; ++kb) pv_block<D, NDT>(MmaBf16{}, O, Vw, kb * 32, sv[kb], lane);

  // ---- the partial into the wave's own region (its V is dead once every lane's reads are in):
  // O_w as [32 rows][OS] f32; m_w, l_w per row beside it
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  float* const Ow = reinterpret_cast<float*>(reg);
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *reinterpret_cast<f32x4_t*>(Ow + qi * OS + dt * 32 + 8 * g + 4 * hh) =
          f32x4_t{O[dt][4 * g], O[dt][4 * g + 1], O[dt][4 * g + 2], O[dt][4 * g + 3]};
  if (hh == 0) {
    ml[wave][0][qi] = mx;
    ml[wave][1][qi] = ls;
  }
  __syncthreads();

  // ---- combine: thread t -> (row, 4-column chunk) pairs, whole rows of O out as bf16
  constexpr int CH = 32 * D / 4;   // 4-column chunks of the 32 x D block
  for (int i = tid; i < CH; i += 64 * W) {
    const int row = i / (D / 4);
    const int col = (i - row * (D / 4)) * 4;
    float m[W], M = -INFINITY;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      m[w] = ml[w][0][row];
      M = fmaxf(M, m[w]);
    }
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
    float L = 0.f;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      const float* ow = reinterpret_cast<const float*>(smem + w * REG);
      const float f = fast_exp2(m[w] - M);
      L += ml[w][1][row] * f;
      acc += *reinterpret_cast<const f32x4_t*>(ow + row * OS + col) * f;
    }
    const int pr = qt * 32 + row;
    if (pr < a.P) {
      const float inv = 1.f / L;
      uint16_t* const op = static_cast<uint16_t*>(a.o) + (int64_t)n * a.bso + h * D + (int64_t)pr * a.ldo + col;
      store4(op, acc[0] * inv, acc[1] * inv, acc[2] * inv, acc[3] * inv);
    }
  }
}

// d = 160 with more keys (the 16x16 layers: P = K = 256): one workgroup = 128 queries (4 waves x
// 32) of one (entry, head), 32-key tiles through a 4-stage LDS ring filled by global_load_lds DMA
// (no VGPRs), three tiles in flight: the per-tile kernel's one-tile-ahead register prefetch left
// every 32-key tile waiting on its own round trip.  Each wave issues exactly 6 DMA instructions per
// tile (3 K, 3 V; slots past the tile fetch a harmless chunk), so "tile kt has landed" is the
// counted wait vmcnt(12) (tiles kt+1, kt+2 still in flight), then one barrier per tile.  K rows
// sit at 21 16-byte slots (336 B: the b128 fragment reads of 16 rows hit 16 bank slots; slot 20 is
// padding), V rows at 20 (320 B, conflict-free for the transposed reads).  Online softmax with the
// defer-max rule, f32 row sums; the output leaves through LDS as whole 16-byte row chunks.
constexpr int kRingStages = 4;

constexpr int kRingStageBytes = 2 * 12 * 1024;   // K: 12 DMA instructions x 1 KiB, V: the same

template <int D, int W>
__global__ __launch_bounds__(64 * W, 1) void self_ring_kernel(SelfArgs a) {
  static_assert(D == 160, "the slot layout below is for d = 160");
  static_assert(W == 1 || W == 2 || W == 4, "24 DMA instructions per tile split evenly");
  constexpr int kPer = 12 / W;          // K (and V) DMA instructions per wave per tile
  constexpr int kWait = 2 * 2 * kPer;   // this wave's DMAs of two tiles still in flight
  constexpr int NKT = D / 16, NDT = D / 32, KCH = D / 8, KSL = KCH + 1;
  constexpr float kThr = 8.0f;
  __shared__ __attribute__((aligned(16))) char ring[kRingStages * kRingStageBytes];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hh = lane >> 5, qi = lane & 31;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int qt = logical % a.n_qtiles;
  const int nh = logical / a.n_qtiles;
  const int h = nh % a.H, n = nh / a.H;
  const int src = a.qk_src[n];
  const int K = a.K;
  const float c = a.scale_log2;
  const int p = qt * 32 * W + wave * 32 + qi;
  const uint16_t* const qp = static_cast<const uint16_t*>(a.q) + (int64_t)src * a.bsq + h * D;
  const uint16_t* const kp = static_cast<const uint16_t*>(a.k) + (int64_t)src * a.bsk + h * D;
  const uint16_t* const vp = static_cast<const uint16_t*>(a.v) + (int64_t)n * a.bsv + h * D;

  short8_t qf[NKT];
  {
    const int pr = min(p, a.P - 1);   // rows past P: any valid row, never stored
#pragma unroll
    for (int t = 0; t < NKT; ++t) qf[t] = *reinterpret_cast<const short8_t*>(qp + (int64_t)pr * a.ldq + 16 * t + 8 * hh);
  }
  // Q retired before any DMA is in flight: hipcc then knows it complete, and its waits inside the
  // loop cannot end up counting (and draining) the ring
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
  const int ntiles = (K + 31) / 32;
  // this wave's 3 K and 3 V DMA instructions of tile kt into stage kt % kRingStages
  const uint32_t ring_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)ring;
  auto issue = [&](int kt) __attribute__((always_inline)) {
    const uint32_t st = __builtin_amdgcn_readfirstlane(ring_lds + (kt % kRingStages) * kRingStageBytes);
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int i = wave * kPer + j;              // instruction 0..11 of the tile
      const int slot = i * 64 + lane;
      int row = slot / KSL, ch = slot - row * KSL;
      if (ch >= KCH || row >= 32) { row = 0; ch = 0; }   // padding slot: fetch any valid chunk
      const int key = min(kt * 32 + row, K - 1);
      glds16(kp + (int64_t)key * a.ldk + ch * 8, __builtin_amdgcn_readfirstlane(st + i * 1024));
      int vrow = slot / KCH, vch = slot - vrow * KCH;
      if (vrow >= 32) { vrow = 0; vch = 0; }
      const int vkey = min(kt * 32 + vrow, K - 1);
      glds16(vp + (int64_t)vkey * a.ldv + vch * 8, __builtin_amdgcn_readfirstlane(st + 12 * 1024 + i * 1024));
    }
  };
  // three tiles in flight (tiles past the last re-fetch the last one: the counted waits stay uniform)
#pragma unroll
  for (int j = 0; j < 3; ++j) issue(min(j, ntiles - 1));

  f32x16_t O[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) O[dt] = f32x16_t{};
  float m_run = -INFINITY, l_run = 0.f;
  for (int kt = 0; kt < ntiles; ++kt) {
    // vmcnt(kWait): this wave's DMAs of tile kt landed (tiles kt+1, kt+2 still in flight)
    __builtin_amdgcn_s_waitcnt((0x0F70 | (kWait & 15)) | ((kWait >> 4) << 14));
    __syncthreads();                           // ... and every other wave's
    const char* const st = ring + (kt % kRingStages) * kRingStageBytes;
    const uint16_t* const Kt = reinterpret_cast<const uint16_t*>(st);
    const uint16_t* const Vt = reinterpret_cast<const uint16_t*>(st + 12 * 1024);
    // Q K^T as two independent accumulator chains (even / odd k steps): one wave per SIMD has no
    // partner to hide a 10-deep dependent MFMA chain behind
    f32x16_t acc2[2] = {f32x16_t{}, f32x16_t{}};
#pragma unroll
    for (int t = 0; t < NKT; ++t) {
      const short8_t kf = *reinterpret_cast<const short8_t*>(Kt + (qi * KSL + 2 * t + hh) * 8);
      acc2[t & 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, kf),
                                                            __builtin_bit_cast(bf16x8_t, qf[t]), acc2[t & 1], 0, 0, 0);
    }
    const f32x16_t acc = acc2[0] + acc2[1];
    // the stage read two tiles ago is free for tile kt + 3 once every wave passed this barrier
    issue(min(kt + 3, ntiles - 1));
    float sv[16];
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      sv[r] = (kt * 32 + acc_row(r, hh) < K) ? acc[r] : -INFINITY;
      mx = fmaxf(mx, sv[r]);
    }
    mx = fmaxf(mx, other_half(mx)) * c;
    if (!__all(mx <= m_run + kThr)) {
      const float mnew = fmaxf(m_run, mx);
      const float alpha = fast_exp2(m_run - mnew);
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) O[dt][r] *= alpha;
      l_run *= alpha;
      m_run = mnew;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      sv[r] = fast_exp2(fmaf(sv[r], c, -m_run));
      l_run += sv[r];
    }
    pv_block<D, NDT>(MmaBf16{}, O, Vt, 0, sv, lane);
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the trailing re-fetches retired
  __syncthreads();                      // every wave is done with the ring
  const float inv = 1.f / (l_run + other_half(l_run));
  // epilogue through LDS: wave w's 32 rows at ring + w * 32 * (D + 8) * 2, then 16-byte row chunks
  constexpr int OS = D + 8;
  uint16_t* const orow = reinterpret_cast<uint16_t*>(ring) + wave * 32 * OS;
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      store4(orow + qi * OS + dt * 32 + 8 * g + 4 * hh, O[dt][4 * g] * inv, O[dt][4 * g + 1] * inv,
             O[dt][4 * g + 2] * inv, O[dt][4 * g + 3] * inv);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  uint16_t* const obase = static_cast<uint16_t*>(a.o) + (int64_t)n * a.bso + h * D;
#pragma unroll
  for (int c0 = 0; c0 < 32 * KCH; c0 += 64) {
    const int cidx = c0 + lane;
    const int row = cidx / KCH, ch = cidx - row * KCH;
    const int pr = qt * 32 * W + wave * 32 + row;
    if (pr < a.P)
      *reinterpret_cast<short8_t*>(obase + (int64_t)pr * a.ldo + ch * 8) =
          *reinterpret_cast<const short8_t*>(orow + row * OS + ch * 8);
  }
}

// d = 160, 128 < K <= 256 (the 16x16 layers), all 256 CUs: one workgroup = 64 queries (two
// 32-row blocks qb) of one (entry, head) x the two key HALVES kh: wave (qb, kh) streams the th =
// ceil(ntiles / 2) 32-key tiles of its half through its half's 3-stage DMA ring, so each wave runs
// half the serial tile chain of the 128-query ring kernel above on twice the workgroups; the
// halves meet once at the end (O_1, m_1, l_1 through LDS into the kh = 0 wave).  Q arrives by DMA
// too, in the same counted stream as the first tiles (the 128-query kernel drains its Q loads
// with vmcnt(0) before the first DMA: one more round trip).  Per wave and tile exactly 11 DMA
// instructions (the half's 11 K + 11 V split between its two waves), so the wait for tile s with
// tile s + 1 in flight is vmcnt(11), and vmcnt(0) on the half's last tile.
constexpr int kHalfStages = 3;
constexpr int kHalfStageBytes = 22 * 1024;                   // K: 11 x 1 KiB (21-slot rows), V: 11
constexpr int kHalfQBytes = 12 * 1024;                       // Q of one block: 12 x 1 KiB (21-slot rows)
constexpr int kHalfLds = 2 * kHalfQBytes + 2 * kHalfStages * kHalfStageBytes;   // 156 KiB

__global__ __launch_bounds__(256, 1) void self_halves_kernel(SelfArgs a) {
  constexpr int D = 160, NKT = D / 16, NDT = D / 32, KCH = D / 8, KSL = KCH + 1;
  constexpr float kThr = 8.0f;
  __shared__ __attribute__((aligned(16))) char lds[kHalfLds];

  const int tid = threadIdx.x, lane = tid & 63, hh = lane >> 5, qi = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int qb = wave & 1, kh = wave >> 1;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int qt = logical % a.n_qtiles;
  const int nh = logical / a.n_qtiles;
  const int h = nh % a.H, n = nh / a.H;
  const int src = a.qk_src[n];
  const int K = a.K, P = a.P;
  const float c = a.scale_log2;
  const int ntiles = (K + 31) / 32;
  const int th = (ntiles + 1) >> 1;          // tiles per half; half 1 starts at tile th < ntiles
  const int t0 = kh * th;
  const int q0 = qt * 64 + qb * 32;           // this wave's first query row
  const uint16_t* const qp = static_cast<const uint16_t*>(a.q) + (int64_t)src * a.bsq + h * D;
  const uint16_t* const kp = static_cast<const uint16_t*>(a.k) + (int64_t)src * a.bsk + h * D;
  const uint16_t* const vp = static_cast<const uint16_t*>(a.v) + (int64_t)n * a.bsv + h * D;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)lds;
  const uint32_t ring0 = lds0 + 2 * kHalfQBytes + kh * (kHalfStages * kHalfStageBytes);

  // Q of block qb: 12 instructions of 21-slot rows (slot 20 and slots past row 31: padding), the
  // block's two waves 6 each; rows past P read row P - 1 (never stored)
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const int i = kh * 6 + j;
    const int slot = i * 64 + lane;
    int row = slot / KSL, ch = slot - row * KSL;
    if (ch >= KCH || row >= 32) { row = 0; ch = 0; }
    glds16(qp + (int64_t)min(q0 + row, P - 1) * a.ldq + ch * 8, __builtin_amdgcn_readfirstlane(lds0 + qb * kHalfQBytes + i * 1024));
  }
  // this wave's share of tile t0 + s of its half into stage s % 3: K instructions qb*6 .. (6 / 5),
  // V instructions qb*5 .. (5 / 6; V's instruction 10 is padding)
  auto issue = [&](int s) __attribute__((always_inline)) {
    const uint32_t st = __builtin_amdgcn_readfirstlane(ring0 + (s % kHalfStages) * kHalfStageBytes);
    const int kt = t0 + s;
#pragma unroll
    for (int j = 0; j < 11; ++j) {
      const bool isk = qb == 0 ? j < 6 : j < 5;
      const int i = qb == 0 ? (isk ? j : j - 6) : (isk ? 6 + j : j);   // instruction within K or V
      const int slot = i * 64 + lane;
      if (isk) {
        int row = slot / KSL, ch = slot - row * KSL;
        if (ch >= KCH || row >= 32) { row = 0; ch = 0; }
        glds16(kp + (int64_t)min(kt * 32 + row, K - 1) * a.ldk + ch * 8, __builtin_amdgcn_readfirstlane(st + i * 1024));
      } else {
        int row = slot / KCH, ch = slot - row * KCH;
        if (row >= 32) { row = 0; ch = 0; }
        glds16(vp + (int64_t)min(kt * 32 + row, K - 1) * a.ldv + ch * 8,
               __builtin_amdgcn_readfirstlane(st + 11 * 1024 + i * 1024));
      }
    }
  };
  issue(0);
  if (th > 1) issue(1);

  short8_t qf[NKT];
  f32x16_t O[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) O[dt] = f32x16_t{};
  float m_run = -INFINITY, l_run = 0.f;
  for (int s = 0; s < th; ++s) {
    // this wave's DMAs of tile s (and, at s = 0, of Q) landed; tile s + 1 may still be in flight
    if (s + 1 < th) __builtin_amdgcn_s_waitcnt(0x0F70 | 11);
    else __builtin_amdgcn_s_waitcnt(0x0F70);
    __syncthreads();                           // ... and the other waves' shares
    if (s == 0) {
      const uint16_t* const Qs = reinterpret_cast<const uint16_t*>(lds + qb * kHalfQBytes);
#pragma unroll
      for (int t = 0; t < NKT; ++t) qf[t] = *reinterpret_cast<const short8_t*>(Qs + (qi * KSL + 2 * t + hh) * 8);
    }
    const char* const st = lds + 2 * kHalfQBytes + kh * (kHalfStages * kHalfStageBytes) + (s % kHalfStages) * kHalfStageBytes;
    const uint16_t* const Kt = reinterpret_cast<const uint16_t*>(st);
    const uint16_t* const Vt = reinterpret_cast<const uint16_t*>(st + 11 * 1024);
    f32x16_t acc2[2] = {f32x16_t{}, f32x16_t{}};
#pragma unroll
    for (int t = 0; t < NKT; ++t) {
      const short8_t kf = *reinterpret_cast<const short8_t*>(Kt + (qi * KSL + 2 * t + hh) * 8);
      acc2[t & 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, kf),
                                                            __builtin_bit_cast(bf16x8_t, qf[t]), acc2[t & 1], 0, 0, 0);
    }
    const f32x16_t acc = acc2[0] + acc2[1];
    // the stage read at s - 1 is free for tile s + 2 once every wave passed this barrier
    if (s + 2 < th) issue(s + 2);
    const int kt = t0 + s;
    float sv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) sv[r] = acc[r];
    if (kt * 32 + 32 > K) {                   // wave-uniform: only a tile reaching past K
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (kt * 32 + acc_row(r, hh) >= K) sv[r] = -INFINITY;
    }
    float mx = sv[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, sv[r]);
    mx = fmaxf(mx, other_half(mx)) * c;        // -inf only for a tile wholly past K (never a half's first)
    if (!__all(mx <= m_run + kThr)) {
      const float mnew = fmaxf(m_run, mx);
      const float alpha = fast_exp2(m_run - mnew);
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) O[dt][r] *= alpha;
      l_run *= alpha;
      m_run = mnew;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      sv[r] = fast_exp2(fmaf(sv[r], c, -m_run));
      l_run += sv[r];
    }
    pv_block<D, NDT>(MmaBf16{}, O, Vt, 0, sv, lane);
  }
  __syncthreads();   // every wave is done with the rings (no DMA in flight: the last wait was vmcnt(0))

  // ---- the halves meet: wave (qb, 1) hands (O, m, l) to wave (qb, 0) as 21 lane-major 16-byte
  // chunks (conflict-free), then wave (qb, 0) writes the rows through LDS as 16-byte row chunks
  f32x4_t* const part = reinterpret_cast<f32x4_t*>(lds) + qb * 21 * 64;
  if (kh == 1) {
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        part[(dt * 4 + g) * 64 + lane] = f32x4_t{O[dt][4 * g], O[dt][4 * g + 1], O[dt][4 * g + 2], O[dt][4 * g + 3]};
    part[20 * 64 + lane] = f32x4_t{m_run, l_run, 0.f, 0.f};
  }
  __syncthreads();
  if (kh == 1) return;
  const f32x4_t ml1 = part[20 * 64 + lane];
  const float M = fmaxf(m_run, ml1[0]);
  const float f0 = fast_exp2(m_run - M), f1 = fast_exp2(ml1[0] - M);
  float l = l_run * f0 + ml1[1] * f1;
  const float inv = 1.f / (l + other_half(l));
  constexpr int OS = D + 8;
  uint16_t* const orow = reinterpret_cast<uint16_t*>(lds + 2 * 21 * 1024) + qb * 32 * OS;
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4_t o1 = part[(dt * 4 + g) * 64 + lane];
      store4(orow + qi * OS + dt * 32 + 8 * g + 4 * hh, (O[dt][4 * g] * f0 + o1[0] * f1) * inv,
             (O[dt][4 * g + 1] * f0 + o1[1] * f1) * inv, (O[dt][4 * g + 2] * f0 + o1[2] * f1) * inv,
             (O[dt][4 * g + 3] * f0 + o1[3] * f1) * inv);
    }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  uint16_t* const obase = static_cast<uint16_t*>(a.o) + (int64_t)n * a.bso + h * D;
#pragma unroll
  for (int c0 = 0; c0 < 32 * KCH; c0 += 64) {
    const int cidx = c0 + lane;
    const int row = cidx / KCH, ch = cidx - row * KCH;
    const int pr = q0 + row;
    if (pr < P)
      *reinterpret_cast<short8_t*>(obase + (int64_t)pr * a.ldo + ch * 8) = *reinterpret_cast<const short8_t*>(orow + row * OS + ch * 8);
  }
}

template <int D, int W, int KBW>
hipError_t launch_split(const SelfArgs& a, hipStream_t st) {
  SelfArgs b = a;
  b.n_qtiles = (a.P + 31) / 32;
  dim3 grid(b.n_qtiles * a.H * a.N), block(64 * W);
  launch_kernel((self_split_kernel<D, W, KBW>), grid, block, 0, st, b);
  return hipGetLastError();
}

template <int W>
hipError_t launch_ring(const SelfArgs& a, hipStream_t st) {
  SelfArgs b = a;
  b.n_qtiles = (a.P + 32 * W - 1) / (32 * W);
  dim3 grid(b.n_qtiles * a.H * a.N), block(64 * W);
  launch_kernel((self_ring_kernel<160, W>), grid, block, 0, st, b);
  return hipGetLastError();
}

}  // namespace

// d = 160, bf16 inputs, O only, K > 128: the 4-stage DMA ring
bool self_ring_eligible(const SelfArgs& a, int d) {
  return d == 160 && a.K > 128 && a.lse == nullptr && a.n_maps == 0;
}

int run_self_ring(const SelfArgs& a, int d, hipStream_t st) {
  (void)d;
  if (a.K <= 256) {
    SelfArgs b = a;
    b.n_qtiles = (a.P + 63) / 64;
    dim3 grid(b.n_qtiles * a.H * a.N), block(256);
    launch_kernel(self_halves_kernel, grid, block, 0, st, b);
    return (int)hipGetLastError();
  }
  return (int)launch_ring<4>(a, st);
}

// d = 160, bf16 inputs, O only, K <= 128 (the 8x8 layers): the waves split the keys (W =
// ceil(K / 64) waves of 64 keys, or 2 x 32 for K <= 64).  Measured against the per-tile kernel
// (tools/small_bench.py, profiles/r03/small): 8x8 (K = 64) 7.84 -> 6.21 us; 16x16 (K = 256)
// 14.73 -> 16.51 us -- every 32-query workgroup then pulls the head's whole K and V through its
// CU (4x the per-tile kernel's L2 -> CU traffic), so K > 128 keeps the per-tile kernel
bool self_split_eligible(const SelfArgs& a, int d) {
  return d == 160 && a.K >= 1 && a.K <= 128 && a.lse == nullptr && a.n_maps == 0;
}

int run_self_split(const SelfArgs& a, int d, hipStream_t st) {
  (void)d;
  if (a.K <= 32) return (int)launch_split<160, 1, 1>(a, st);
  if (a.K <= 64) return (int)launch_split<160, 2, 1>(a, st);
  if (a.K <= 128) return (int)launch_split<160, 2, 2>(a, st);
  if (a.K <= 192) return (int)launch_split<160, 3, 2>(a, st);
  return (int)launch_split<160, 4, 2>(a, st);
}

}  // namespace p2p
