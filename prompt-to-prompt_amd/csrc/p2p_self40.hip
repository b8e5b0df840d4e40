// d = 40 self-attention, O only: the G1/G7 layers of the SD-v1.4 U-Net (P = K = 4096, 8 heads)
// without kept maps or autograd -- the dominant kernel of the hot path (ptp_utils.py:195-206).
//
// Round-3 form: software-pipelined over 32x32 blocks.  A wave owns QB 32-row query blocks; the
// blocks of a tile are walked in the order x = (32-key sub-block, query block), and step x issues
//     Q K^T of block x+1 (3 MFMAs)  |  exp2 + bf16 pack of block x (16 v_exp, 8 v_cvt_pk)  |  P V of block x-1 (4 MFMAs)
// so every MFMA has exponentials of an independent block beside it and every exponential an
// MFMA: the wave's own instruction stream interleaves the matrix pipe and the VALU instead of
// relying on a co-resident wave to fill the gaps (MI355X_MICROARCH.md, "one wave per SIMD").
// K/V fragments for sub-block sb+1 are read from LDS while sub-block sb computes (double-
// buffered fragments), and the next tile's K/V are staged into the other LDS buffer by
// register staging spread over the second half of the tile.
//
// Arithmetic (the F16 form of round 2, kept): Q is prescaled by c = scale*log2(e) and rounded
// to f16; K is staged as f16 (exact for bf16 values in range); d pads to 48 and the padding
// column carries the reference point (K[:,40] = 1, Q[:,40] = -m), so S^T = c s - m leaves the
// MFMA and p = exp2(S^T) costs one v_exp.  V's column 40 is 1, so O^T row 40 is the row sum of
// the same bf16 p that P V uses.  The reference point m of a query row is the maximum over the
// first 32 keys (no per-tile maximum); a tile whose row sum passes 2^64 moves m up by 64 and
// rescales O by the exact factor.  Anything outside the fast form's range -- |c q| or |k| past
// the f16 range, |m| >= 65504, a non-finite row sum or O element -- flags the workgroup, which
// recomputes everything on the exact bf16 path (unscaled bf16 Q and K, running max per
// sub-block).
#include <type_traits>
#include <utility>

#include "p2p_device.h"
#include "p2p_kernels.h"

namespace p2p {
namespace {

typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_t;

// Head-dim geometry.  d = 40 (G1/G7): the F16 form (Q prescaled by c in f16, K staged as f16,
// -m in the padding column 40 of the 48-deep Q K^T); d = 80 (G2/G6): the bf16 form (raw bf16 Q
// and K, 5 k steps with no padding, p = exp2(fma(s, c, -m))).  O^T's row D is the row sum (V's
// column D is 1).
template <int D>
struct Geom;
template <>
struct Geom<40> {
  static constexpr bool F16 = true;
  static constexpr int NKT = 3;    // 16-deep k steps of Q K^T (d padded to 48, column 40 = -m)
  static constexpr int NDT = 2;    // 32-row tiles of O^T (rows 0-39 data, 40 row sums)
  static constexpr int KS = 56;    // K row in LDS: 112 B, a b128 read of 16 rows hits 16 slots
};
template <>
struct Geom<80> {
  static constexpr bool F16 = false;
  static constexpr int NKT = 5;
  static constexpr int NDT = 3;    // rows 0-79 data, 80 row sums
  static constexpr int KS = 88;    // 176 B: 16 rows of a b128 read on 16 distinct slots
};
constexpr int kVS = 96;    // bf16 elements per V row in LDS: 192 B, conflict-free transposed reads

template <int... I, typename F>
__device__ __forceinline__ void static_for_impl(std::integer_sequence<int, I...>, F&& f) {
  (f(std::integral_constant<int, I>{}), ...);
}
// f(integral_constant<int, i>) for i = 0 .. N-1, unrolled at compile time
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(std::make_integer_sequence<int, N>{}, f);
}

__device__ __forceinline__ short8_t lds_b128(const uint16_t* p) { return *reinterpret_cast<const short8_t*>(p); }

__device__ __forceinline__ void mma_f16(f32x16_t& acc, const short8_t& k, const short8_t& q) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, k), __builtin_bit_cast(f16x8_t, q), acc,
                                               0, 0, 0);
}
__device__ __forceinline__ void mma_bf16(f32x16_t& acc, const short8_t& a, const short8_t& b) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), acc,
                                                0, 0, 0);
}

#ifdef P2P_EXPERIMENTS
// Diagnostic build (FORM bit 16, experiments library only): per-wave shader-clock stamps of the
// first 256 workgroups, read back by p2p_diag_self40_stamps (tools/s40_stamps.py).
// slots 38 / 39: s_memrealtime (100 MHz, one clock for every XCD) at the start / end, for the
// launch's workgroup timeline; stamps of the first 1024 workgroups
constexpr int kStampSlots = 40;
constexpr int kStampWgs = 1024;
__device__ unsigned long long g_s40_stamps[kStampWgs * 8 * kStampSlots];
#endif

// One workgroup = WAVES waves x QB query blocks of 32 rows = 32*QB*WAVES queries of one (entry,
// head); BK-key tiles, double-buffered in LDS.
//
// FORM bits (measured-and-dropped variants live in git history, DESIGN.md §4 cites their logs):
//   1        LEAN fragment buffering (one K and one V fragment set per wave)
//   16       clock stamps (experiments build only)
//   128      split staging: waves 0..WAVES/2-1 stage K (the f16 conversion), the rest V
//   256/512/16384  the younger half holds priority 1 for 3 of every 4 steps
//   8388608  K's f16 range check as a packed-u16 maximum
template <int kD, int WAVES, int QB, int BK, bool SCHED, int FORM>
__global__ __launch_bounds__(64 * WAVES, WAVES >= 8 ? 2 : 1) void self40_kernel(SelfArgs a) {
  using G = Geom<kD>;
  constexpr bool kF16 = G::F16;
  constexpr int kNKT = G::NKT;
  constexpr int kNDT = G::NDT;
  constexpr int kKS = G::KS;
  constexpr int kCPR = kD / 8;   // 16-byte chunks per K/V row
  constexpr int kDK = 16 * kNKT;
  constexpr int kDV = 32 * kNDT;
  static_assert(kDV > kD && (!kF16 || kDK > kD), "padding for the row-sum and -m columns");
  // O^T row kD (the row sums): d tile kLdt, register kLr of the low lane half
  constexpr int kLdt = kD / 32;
  constexpr int kLrr = kD % 32;
  constexpr int kLr = (kLrr & 3) + 4 * (kLrr >> 3);
  static_assert(((kLrr >> 2) & 1) == 0, "the row sum sits in the low lane half");
  constexpr int NSB = BK / 32;
  constexpr int NT = 64 * WAVES;
  constexpr int NCH = (BK * kCPR + NT - 1) / NT;
  constexpr int KBUF = BK * kKS;
  constexpr int VBUF = BK * kVS;
  constexpr int X = NSB * QB;   // pipeline steps (32x32 blocks) per tile
  constexpr float kThr = 8.0f;  // exact path: defer-max threshold (log2 units)
  // FORM bit 128 (split staging): waves 0..WAVES/2-1 stage K (the f16 conversion), the younger
  // half -- the VALU-arbitration loser -- stages V (copy only); else every wave stages both
  constexpr bool kSplit = (FORM & 128) != 0;
  constexpr int SCH = (BK * kCPR + NT / 2 - 1) / (NT / 2);   // chunks per thread, split staging
  constexpr int CMAX = kSplit ? SCH : NCH;
  // staging writes: chunk i of the next tile at step kWs + i (X - kWs) / n (several per step
  // when there are more chunks than steps), from the middle of the tile on -- the loads issued at
  // its start have landed by then
  constexpr int kWs = X / 2;
  constexpr int kWe = X;
  auto nchunks = [](auto role) { return decltype(role)::value == 0 ? NCH : SCH; };
  // K and V tile buffers; after the last tile the same LDS holds each wave's output rows (epilogue)
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * KBUF + 2 * VBUF];
  uint16_t* const Ks = smem;
  uint16_t* const Vs = smem + 2 * KBUF;
  constexpr int kOS = kD + 8;   // output row in LDS: 16-byte aligned, rows on distinct banks
  static_assert(WAVES * 32 * QB * kOS <= 2 * KBUF + 2 * VBUF, "epilogue rows fit the tile buffers");
  __shared__ int wg_flag;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int hh = lane >> 5;
  const int qi = lane & 31;

  // every kernel argument the prologue reads is pinned here, so all of them arrive in ONE scalar
  // round trip (each a.field is a scalar load; hipcc otherwise spreads them over the prologue in a
  // chain of dependent waits); the entry's qk_src is the one dependent load after it
  asm volatile("" ::"s"(a.n_qtiles), "s"(a.H), "s"(a.P), "s"(a.K), "s"(a.q), "s"(a.k), "s"(a.v), "s"(a.o),
               "s"(a.ldq), "s"(a.ldk), "s"(a.ldv), "s"(a.ldo), "s"(a.bsq), "s"(a.bsk), "s"(a.bsv), "s"(a.bso),
               "s"(a.scale_log2));
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  auto stamp = [&](int idx) __attribute__((always_inline)) {
#ifdef P2P_EXPERIMENTS
    if constexpr ((FORM & 16) != 0)
      if (logical < kStampWgs && lane == 0 && idx < kStampSlots) {
        g_s40_stamps[(logical * WAVES + wave) * kStampSlots + idx] = __builtin_amdgcn_s_memtime();
        if (idx == 0 || idx == 37)
          g_s40_stamps[(logical * WAVES + wave) * kStampSlots + 38 + (idx == 37)] = __builtin_amdgcn_s_memrealtime();
      }
#endif
  };
  stamp(0);
  // query tiles fastest: with xcd_remap's contiguous chunks one XCD runs all tiles of an (entry,
  // head), so that head's K / V come from its L2 (heads fastest measured no faster and raised the
  // reads, profiles/r03 variant 128)
  const int qt = logical % a.n_qtiles;
  const int h = (logical / a.n_qtiles) % a.H;
  const int n = logical / a.n_qtiles / a.H;
  const int src = a.qk_src[n];
  // first query of this wave, in a scalar register (the Q buffer resource stays scalar)
  const int pw = __builtin_amdgcn_readfirstlane((qt * WAVES + wave) * 32 * QB);
  const int K = a.K;
  const float c = a.scale_log2;

  const uint16_t* const qp = static_cast<const uint16_t*>(a.q) + (int64_t)src * a.bsq + h * kD;
  const uint16_t* const kp = static_cast<const uint16_t*>(a.k) + (int64_t)src * a.bsk + h * kD;
  const uint16_t* const vp = static_cast<const uint16_t*>(a.v) + (int64_t)n * a.bsv + h * kD;

  // padding columns (written once; staging writes columns 0..D-1 only): F16 K column D = f16 1.0
  // (the -m column), D+1..DK-1 = 0; V column D = bf16 1.0 (row sums), D+1..DV-1 = 0
  for (int r = tid; r < 2 * BK; r += NT) {
#pragma unroll
    for (int j = 0; j < (kDK - kD) / 8; ++j)
      *reinterpret_cast<short8_t*>(Ks + r * kKS + kD + 8 * j) =
          short8_t{(short)(j == 0 && kF16 ? 0x3C00 : 0), 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < (kDV - kD) / 8; ++j)
      *reinterpret_cast<short8_t*>(Vs + r * kVS + kD + 8 * j) =
          short8_t{(short)(j == 0 ? 0x3F80 : 0), 0, 0, 0, 0, 0, 0, 0};
  }
  if (tid == 0) wg_flag = 0;

  // ---- Q fragments: lane (qi, hh) of block b, k step t holds Q[p][16t + 8hh .. +7]
  bool ovf = false;
  // FORM bit 8388608: K's f16 range check as a running packed u16 maximum of the bf16 magnitudes
  // (v_and + v_pk_max_u16 per pair), compared once at the end: a bf16 magnitude >= 0x4780 (65536,
  // past the f16 range; inf / NaN included) sends the workgroup to the exact path -- instead of an
  // f32 |x| maximum per chunk (the fmaxf NaN canonicalisation made that ~3.5 VALU per pair)
  constexpr bool kU16Max = (FORM & 8388608) != 0;
  typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));
  typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
  u16x2_t kmag = {0, 0};
  short8_t qf[QB][kNKT];
  // Q rows by range-checked buffer loads from this wave's first row on (rows >= P read as zeros),
  // issued unconditionally: a branch around every fragment load made hipcc re-load the row stride
  // from the kernel arguments and wait for it before each load of the prologue
  const __amdgpu_buffer_rsrc_t rq = make_rsrc(qp + (int64_t)pw * a.ldq, ((int64_t)(a.P - 1 - pw) * a.ldq + kD) * 2);
  auto load_q = [&](bool prescale) __attribute__((always_inline)) {
#pragma unroll
    for (int b = 0; b < QB; ++b)
#pragma unroll
      for (int t = 0; t < kNKT; ++t) {
        const int col = 16 * t + 8 * hh;
        short8_t v = __builtin_bit_cast(
            short8_t, __builtin_amdgcn_raw_buffer_load_b128(rq, ((32 * b + qi) * (int)a.ldq + col) * 2, 0, 0));
        if (col >= kD) v = short8_t{0, 0, 0, 0, 0, 0, 0, 0};   // (d = 40: the padding columns 40..47)
        if (prescale) {
          float mx = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float x = bf2f((uint16_t)v[j]) * c;
            mx = fmaxf(mx, fabsf(x));
            v[j] = (short)__builtin_bit_cast(uint16_t, (_Float16)x);
          }
          ovf |= !(mx < 65520.f);
        }
        qf[b][t] = v;
      }
  };
  load_q(kF16);
  // F16: Q column D (k step D/16, lane half (D%16)/8, element D%8) holds -m
  auto set_mcol = [&](int b, float m) __attribute__((always_inline)) {
    if constexpr (kF16)
      if (hh == (kD % 16) / 8) qf[b][kD / 16][kD % 8] = (short)__builtin_bit_cast(uint16_t, (_Float16)(-m));
  };

  // ---- K/V staging: chunk i of this thread = row cidx / 5, 16-byte chunk cidx % 5 (role 0: both
  // K and V of the chunk; split staging: role 1 = K chunks of threads 0..NT/2-1, role 2 = V
  // chunks of the others, each thread holding SCH of them in kreg)
  const bool young = __builtin_amdgcn_readfirstlane(wave) >= WAVES / 2;
  const bool vrole = young;
  const int stid = kSplit ? tid - (young ? NT / 2 : 0) : tid;   // (position within the half)
  const int sstride = kSplit ? NT / 2 : NT;
  short8_t kreg[CMAX], vreg[NCH];
  uint32_t koff[CMAX], voff[NCH];
  int lrow[CMAX], lch[CMAX];
#pragma unroll
  for (int i = 0; i < CMAX; ++i) {
    const int cidx = stid + i * sstride;
    const int row = min(cidx / kCPR, BK - 1);
    const int ch = cidx - (cidx / kCPR) * kCPR;
    lrow[i] = row;
    lch[i] = ch;
    koff[i] = (uint32_t)((row * (int)(kSplit && vrole ? a.ldv : a.ldk) + ch * 8) * 2);
    if (i < NCH) voff[i] = (uint32_t)((row * (int)a.ldv + ch * 8) * 2);
  }
  const int64_t kbytes = ((int64_t)(K - 1) * a.ldk + kD) * 2;
  const int64_t vbytes = ((int64_t)(K - 1) * a.ldv + kD) * 2;
  const int64_t kstep = (int64_t)BK * a.ldk * 2;
  const int64_t vstep = (int64_t)BK * a.ldv * 2;
  auto chunk_live = [&](int i, auto role) __attribute__((always_inline)) {
    constexpr int sn = decltype(role)::value == 0 ? NT : NT / 2;
    return (BK * kCPR) % sn == 0 || stid + i * sn < BK * kCPR;
  };
  auto stage_load = [&](int kt, auto role) __attribute__((always_inline)) {
    constexpr int kRole = decltype(role)::value;
    const __amdgpu_buffer_rsrc_t rk = make_rsrc(reinterpret_cast<const char*>(kp) + kt * kstep, kbytes - kt * kstep);
    const __amdgpu_buffer_rsrc_t rv = make_rsrc(reinterpret_cast<const char*>(vp) + kt * vstep, vbytes - kt * vstep);
#pragma unroll
    for (int i = 0; i < nchunks(role); ++i)
      if (chunk_live(i, role)) {
        kreg[i] = __builtin_bit_cast(short8_t, __builtin_amdgcn_raw_buffer_load_b128(kRole == 2 ? rv : rk, (int)koff[i], 0, 0));
        if constexpr (kRole == 0)
          vreg[i] = __builtin_bit_cast(short8_t, __builtin_amdgcn_raw_buffer_load_b128(rv, (int)voff[i], 0, 0));
      }
  };
  // chunk i into LDS buffer buf: K as f16 (fast form; exact for magnitudes in [2^-14, 65504] --
  // smaller ones become f16 subnormals, absolute error < 2^-25 --, RTZ packing would clamp past
  // 65504 silently, so the range is checked) or raw bf16 (exact path)
  auto stage_write = [&](int i, int buf, bool as_f16, auto role) __attribute__((always_inline)) {
    constexpr int kRole = decltype(role)::value;
    if (!chunk_live(i, role)) return;
    if constexpr (kRole == 2) {
      *reinterpret_cast<short8_t*>(Vs + buf * VBUF + lrow[i] * kVS + lch[i] * 8) = kreg[i];
      return;
    }
    uint16_t* const kd = Ks + buf * KBUF + lrow[i] * kKS + lch[i] * 8;
    if (as_f16 && kU16Max) {
      const u32x4_t wv = __builtin_bit_cast(u32x4_t, kreg[i]);
      u32x4_t hv;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t w = wv[j];
        kmag = __builtin_elementwise_max(kmag, __builtin_bit_cast(u16x2_t, w & 0x7fff7fffu));
        hv[j] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(__uint_as_float(w << 16),
                                                                       __uint_as_float(w & 0xffff0000u)));
      }
      *reinterpret_cast<u32x4_t*>(kd) = hv;
    } else if (as_f16) {
      short8_t hv;
      float mx = 0.f;
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const float x0 = bf2f((uint16_t)kreg[i][j]), x1 = bf2f((uint16_t)kreg[i][j + 1]);
        mx = fmaxf(mx, fmaxf(fabsf(x0), fabsf(x1)));
        const auto pk = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(x0, x1));
        hv[j] = (short)(pk & 0xffff);
        hv[j + 1] = (short)(pk >> 16);
      }
      ovf |= !(mx < 65504.f);
      *reinterpret_cast<short8_t*>(kd) = hv;
    } else {
      *reinterpret_cast<short8_t*>(kd) = kreg[i];
    }
    if constexpr (kRole == 0) *reinterpret_cast<short8_t*>(Vs + buf * VBUF + lrow[i] * kVS + lch[i] * 8) = vreg[i];
  };
  // a whole tile into buf, for the role(s) of this wave (prologue and exact recompute)
  auto stage_all = [&](int kt, int buf, bool as_f16) __attribute__((always_inline)) {
    auto go = [&](auto role) __attribute__((always_inline)) {
      stage_load(kt, role);
#pragma unroll
      for (int i = 0; i < nchunks(role); ++i) stage_write(i, buf, as_f16, role);
    };
    if constexpr (!kSplit) go(std::integral_constant<int, 0>{});
    else if (vrole) go(std::integral_constant<int, 2>{});
    else go(std::integral_constant<int, 1>{});
  };

  const int ntiles = (K + BK - 1) / BK;
  const int nfull = K / BK;
  f32x16_t O[QB][kNDT];
  float m_ref[QB];
#pragma unroll
  for (int b = 0; b < QB; ++b)
#pragma unroll
    for (int dt = 0; dt < kNDT; ++dt) O[b][dt] = f32x16_t{};

  // LDS fragment reads: K^T operand of sub-block sb (3 k steps), V^T operand (2 k steps x 2 d tiles)
  auto read_k = [&](const uint16_t* Kb, int sb, short8_t (&kf)[kNKT]) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < kNKT; ++t) kf[t] = lds_b128(Kb + (sb * 32 + qi) * kKS + 16 * t + 8 * hh);
  };
  auto read_v = [&](const uint16_t* Vb, int sb, short8_t (&vf)[2][kNDT]) __attribute__((always_inline)) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int dt = 0; dt < kNDT; ++dt) vf[s2][dt] = vt_frag<kVS>(Vb, sb * 32, s2, dt * 32, lane).v;
  };

  stage_all(0, 0, kF16);
  __syncthreads();

  // ---- reference point: the row maximum of c s over the first 32 keys (F16: Q column D is still 0)
  {
    short8_t kf[kNKT];
    read_k(Ks, 0, kf);
#pragma unroll
    for (int b = 0; b < QB; ++b) {
      f32x16_t acc = f32x16_t{};
#pragma unroll
      for (int t = 0; t < kNKT; ++t) {
        if constexpr (kF16) mma_f16(acc, kf[t], qf[b][t]);
        else mma_bf16(acc, kf[t], qf[b][t]);
      }
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, acc[r]);
      mx = fmaxf(mx, other_half(mx));
      if constexpr (!kF16) mx *= c;
      const float m = kF16 ? (float)(_Float16)mx : mx;   // F16: representable in Q's f16 column
      ovf |= !(fabsf(m) < (kF16 ? 65504.f : INFINITY));
      m_ref[b] = m;
      set_mcol(b, m);
    }
  }

  stamp(1);
  bool bad = false;
  // ---- one tile of the fast form, software-pipelined over its X blocks.  more: the next tile
  // is staged during this one (compile-time, so the tile body is one basic block); masked: keys
  // past K in this tile
  auto tile = [&](int kt, auto more, auto masked, auto role) __attribute__((always_inline)) {
    constexpr bool kMore = decltype(more)::value;
    constexpr bool kMasked = decltype(masked)::value;
    constexpr int kNcw = nchunks(role);
    const int buf = kt & 1;
    if constexpr (kMore) stage_load(kt + 1, role);
    const uint16_t* const Kb = Ks + buf * KBUF;
    const uint16_t* const Vb = Vs + buf * VBUF;
    // LEAN: one K and one V fragment set, each re-read right after its last reader (K of
    // sub-block sb+1 after the last Q K^T on sb, V of sb after the last P V on sb-1)
    constexpr bool kLean = (FORM & 1) != 0;
    constexpr bool kLeanK = kLean;
    short8_t kf[2][kNKT];
    short8_t vf[2][2][kNDT];
    f32x16_t S[2];
    short8_t pf[2][2];
    read_k(Kb, 0, kf[0]);
    read_v(Vb, 0, vf[0]);
    auto kslot = [](int sb) { return kLeanK ? 0 : (sb & 1); };
    auto vslot = [](int sb) { return kLean ? 0 : (sb & 1); };
    auto qk = [&](int x) __attribute__((always_inline)) {
      const int sb = x / QB, b = x % QB;
      S[x & 1] = f32x16_t{};
#pragma unroll
      for (int t = 0; t < kNKT; ++t) {
        if constexpr (kF16) mma_f16(S[x & 1], kf[kslot(sb)][t], qf[b][t]);
        else mma_bf16(S[x & 1], kf[kslot(sb)][t], qf[b][t]);
      }
    };
    auto pv = [&](int x) __attribute__((always_inline)) {
      const int sb = x / QB, b = x % QB;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int dt = 0; dt < kNDT; ++dt) mma_bf16(O[b][dt], vf[vslot(sb)][s2][dt], pf[x & 1][s2]);
    };
    auto ex = [&](int x) __attribute__((always_inline)) {
      const int sb = x / QB, b = x % QB;
      float e[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float s = kF16 ? S[x & 1][r] : fmaf(S[x & 1][r], c, -m_ref[b]);
        if constexpr (kMasked)
          if (kt * BK + sb * 32 + acc_row(r, hh) >= K) s = -INFINITY;
        e[r] = fast_exp2(s);
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[x & 1][s2][j] = (short)f2bf(e[8 * s2 + j]);
    };
    qk(0);
    if constexpr (SCHED) __builtin_amdgcn_sched_barrier(0);
    static_for<X>([&](auto xc) __attribute__((always_inline)) {
      constexpr int x = decltype(xc)::value;
      // FORM bit 256: the younger half holds priority 1 for the first half of every kAlt steps
      // (bit 512: kAlt = 4, else 2), so the two waves of a SIMD share the VALU evenly
      // (bit 16384, with 512: priority 1 for 3 of every 4 steps)
      if constexpr ((FORM & 256) != 0) {
        constexpr int kAlt = (FORM & 512) ? 4 : 2;
        constexpr int kOn = (FORM & 16384) ? 3 : kAlt / 2;
        if constexpr (x % kAlt == 0) { if (young) __builtin_amdgcn_s_setprio(1); }
        if constexpr (x % kAlt == kOn) { if (young) __builtin_amdgcn_s_setprio(0); }
      }
      constexpr int sb = x / QB, b = x % QB;
      // K of sub-block sb+1: LEAN after this step's Q K^T when it was the last one on sb
      // (b == QB-2: Q K^T of block x+1 = (sb, QB-1)), else early into the other slot
      // (QB == 1: block x+1 is already on sb+1, so its K is read at the start of this step)
      constexpr bool kRdK = (kLeanK ? b == (QB >= 2 ? QB - 2 : 0) : b == 0) && sb + 1 < NSB;
      constexpr bool kRdKEarly = kLeanK && kRdK && QB == 1;
      // V: LEAN reads V(sb) after this step's P V on block x-1 = (sb-1, QB-1); else V(sb+1) early
      constexpr bool kRdV = kLean ? (b == 0 && sb >= 1) : (b == (QB > 1 ? 1 : 0) && sb + 1 < NSB);
      // the next tile's chunks go to the other buffer over the second half of the tile (every
      // wave has passed the barrier that ended the tile which last read that buffer)
      // chunks [c0, c1) of this thread are written in this step
      constexpr int kWn = kWe - kWs;
      constexpr bool kInW = x >= kWs && x < kWe;
      constexpr int c0 = kInW ? ((x - kWs) * kNcw + kWn - 1) / kWn : 0;
      constexpr int c1 = kInW ? ((x + 1 - kWs) * kNcw + kWn - 1) / kWn : 0;
      constexpr bool kStw = kMore && c1 > c0;
      constexpr bool kStwK = kStw && decltype(role)::value != 2;   // the write converts K
      if constexpr (!kLeanK && kRdK) read_k(Kb, sb + 1, kf[(sb + 1) & 1]);
      if constexpr (kRdKEarly) read_k(Kb, sb + 1, kf[0]);
      if constexpr (!kLean && kRdV) read_v(Vb, sb + 1, vf[(sb + 1) & 1]);
      if constexpr (x + 1 < X) qk(x + 1);
      ex(x);
      if constexpr (kLeanK && kRdK && !kRdKEarly) read_k(Kb, sb + 1, kf[0]);
      if constexpr (x >= 1) pv(x - 1);
      if constexpr (kLean && kRdV) read_v(Vb, sb, vf[0]);
      if constexpr (kStw)
#pragma unroll
        for (int i = c0; i < c1; ++i) stage_write(i, buf ^ 1, kF16, role);
      if constexpr (SCHED) {
        // one MFMA per slot (this step's Q K^T first, then P V), the step's exponentials and
        // VALU spread evenly over the slots; LDS reads early, or (LEAN) after their last reader
        // (masks: MFMA 0x8, VALU 0x2 -- which excludes the transcendental v_exp --, TRANS
        // 0x400, DS_READ 0x100, DS_WRITE 0x200)
        constexpr int nq = x + 1 < X ? kNKT : 0;
        constexpr int nm = nq + (x >= 1 ? 2 * kNDT : 0);
        constexpr int ne = 16;
        constexpr int nv = 8 + (kF16 ? 0 : 16) + (kStwK && kF16 ? 24 * (c1 - c0) : 0) + (kMasked ? 32 : 0);
        constexpr int nr = (!kLeanK && kRdK ? kNKT : 0) + (!kLean && kRdV ? 4 * kNDT : 0);
        if constexpr (kRdKEarly) __builtin_amdgcn_sched_group_barrier(0x100, kNKT, 0);
        static_for<nm>([&](auto ic) __attribute__((always_inline)) {
          constexpr int i = decltype(ic)::value;
          constexpr int te = (ne * (i + 1)) / nm - (ne * i) / nm;
          constexpr int tv = (nv * (i + 1)) / nm - (nv * i) / nm;
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x400, te, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, tv, 0);
          if constexpr (nr > 0) __builtin_amdgcn_sched_group_barrier(0x100, (nr * (i + 1)) / nm - (nr * i) / nm, 0);
          if constexpr (kLeanK && kRdK && !kRdKEarly && i >= nq && i < nq + kNKT)
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          if constexpr (kStw && i < 2) __builtin_amdgcn_sched_group_barrier(0x200, c1 - c0, 0);
        });
        if constexpr (kLean && kRdV) __builtin_amdgcn_sched_group_barrier(0x100, 4 * kNDT, 0);   // ds_read_b64_tr x2 per fragment
        __builtin_amdgcn_sched_barrier(0);
      }
    });
    pv(X - 1);
    stamp(2 + 2 * kt);
    // row sums (O^T row 40 = d tile 1, register 4 of the low lane half): a sum past 2^64 moves
    // the reference point up by 64 (rounded to f16) and rescales O by the exact factor
    // The last P V of block QB-1 was issued just above; its row sum is read after explicit padding
    // and before the first rescale branch.  Without it the wait states the compiler put on the
    // branch fall-through proved short on gfx950 (d = 80: the copy read for the lane-half swap
    // saw the pre-MFMA value on one half, so the halves disagreed about the rescale)
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    float lsums[QB];
#pragma unroll
    for (int b = 0; b < QB; ++b) {
      const float own = O[b][kLdt][kLr];
      lsums[b] = own + other_half(own);
    }
#pragma unroll
    for (int b = 0; b < QB; ++b) {
      const float lsum = lsums[b];
      bad |= !(lsum < INFINITY);
      constexpr float kResc = 0x1p64f;
      if (__builtin_expect(__any(lsum > kResc), 0)) {
        if (lsum > kResc) {
          const float mnew = kF16 ? (float)(_Float16)(m_ref[b] + 64.f) : m_ref[b] + 64.f;
          ovf |= !(fabsf(mnew) < (kF16 ? 65504.f : INFINITY));
          const float f = fast_exp2(m_ref[b] - mnew);
#pragma unroll
          for (int dt = 0; dt < kNDT; ++dt)
#pragma unroll
            for (int r = 0; r < 16; ++r) O[b][dt][r] *= f;
          m_ref[b] = mnew;
          set_mcol(b, mnew);
        }
      }
    }
    __syncthreads();
    stamp(3 + 2 * kt);
  };
  constexpr std::false_type kNo{};
  constexpr std::true_type kYes{};
  auto run_tiles = [&](auto role) __attribute__((always_inline)) {
    for (int kt = 0; kt + 1 < ntiles; ++kt) tile(kt, kYes, kNo, role);
    if (nfull == ntiles) tile(ntiles - 1, kNo, kNo, role);
    else tile(ntiles - 1, kNo, kYes, role);
  };
  if constexpr (!kSplit) run_tiles(std::integral_constant<int, 0>{});
  else if (vrole) run_tiles(std::integral_constant<int, 2>{});
  else run_tiles(std::integral_constant<int, 1>{});

  {
    // a row sum can stay finite while an O element overflowed (p near 2^128 times a large |v|):
    // any non-finite accumulator also sends the workgroup to the exact recompute
    float nf = 0.f;
#pragma unroll
    for (int b = 0; b < QB; ++b)
#pragma unroll
      for (int dt = 0; dt < kNDT; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) nf = __builtin_fmaf(O[b][dt][r], 0.f, nf);   // NaN iff some O is inf/NaN
    bad |= !(nf == 0.f);
    if constexpr (kU16Max) ovf |= kmag.x >= 0x4780 || kmag.y >= 0x4780;
    const bool any_bad = __any(bad || ovf);
    if (lane == 0 && any_bad) atomicOr(&wg_flag, 1);
  }
  __syncthreads();
  if (__builtin_expect(wg_flag != 0, 0)) {
    // ---- exact recompute: bf16 Q and K as they are, S = Q K^T in f32, running max per
    // 32-key sub-block with the defer-max rule (the sub-block's P V follows at once)
    load_q(false);
    float m_run[QB];
#pragma unroll
    for (int b = 0; b < QB; ++b) {
      m_run[b] = -INFINITY;
#pragma unroll
      for (int dt = 0; dt < kNDT; ++dt) O[b][dt] = f32x16_t{};
    }
    for (int kt = 0; kt < ntiles; ++kt) {
      stage_all(kt, 0, false);
      __syncthreads();
      for (int sb = 0; sb < NSB; ++sb) {
        short8_t kf[kNKT];
        short8_t vf[2][kNDT];
        read_k(Ks, sb, kf);
        read_v(Vs, sb, vf);
#pragma unroll
        for (int b = 0; b < QB; ++b) {
          f32x16_t acc = f32x16_t{};
#pragma unroll
          for (int t = 0; t < kNKT; ++t) mma_bf16(acc, kf[t], qf[b][t]);
          float sv[16];
          float mx = -INFINITY;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            sv[r] = (kt * BK + sb * 32 + acc_row(r, hh) < K) ? acc[r] * c : -INFINITY;
            mx = fmaxf(mx, sv[r]);
          }
          mx = fmaxf(mx, other_half(mx));
          if (!__all(mx <= m_run[b] + kThr)) {
            const float mnew = fmaxf(m_run[b], mx);
            const float alpha = mnew == -INFINITY ? 1.f : fast_exp2(m_run[b] - mnew);
#pragma unroll
            for (int dt = 0; dt < kNDT; ++dt)
#pragma unroll
              for (int r = 0; r < 16; ++r) O[b][dt][r] *= alpha;
            m_run[b] = mnew;
          }
          short8_t pb[2];
#pragma unroll
          for (int r = 0; r < 16; ++r) pb[r >> 3][r & 7] = (short)f2bf(fast_exp2(sv[r] - m_run[b]));
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int dt = 0; dt < kNDT; ++dt) mma_bf16(O[b][dt], vf[s2][dt], pb[s2]);
        }
      }
      __syncthreads();
    }
  }

  stamp(36);
  // ---- epilogue: O / l.  O^T has the query on the lane, so a direct store would touch 64 rows
  // (64 cache lines) per instruction; the wave writes its rows to LDS instead (the tile buffers
  // are dead: every wave has passed the last tile's barrier) and stores them back as contiguous
  // 16-byte chunks, consecutive lanes along a row
  uint16_t* const orow = smem + wave * (32 * QB * kOS);
#pragma unroll
  for (int b = 0; b < QB; ++b) {
    const float l = __shfl(O[b][kLdt][kLr], lane & 31);
    const float inv = 1.f / l;
#pragma unroll
    for (int dt = 0; dt < kNDT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int dd = dt * 32 + 8 * g + 4 * hh;
        if (dd < kD)
          store4(orow + (32 * b + qi) * kOS + dd, O[b][dt][4 * g] * inv, O[b][dt][4 * g + 1] * inv,
                 O[b][dt][4 * g + 2] * inv, O[b][dt][4 * g + 3] * inv);
      }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  {
    constexpr int kChunks = 32 * QB * kCPR;
    uint16_t* const obase = static_cast<uint16_t*>(a.o) + (int64_t)n * a.bso + h * kD;
#pragma unroll
    for (int c0 = 0; c0 < kChunks; c0 += 64) {
      const int cidx = c0 + lane;
      const int row = cidx / kCPR, ch = cidx - (cidx / kCPR) * kCPR;
      const int p = pw + row;
      if ((kChunks % 64 == 0 || cidx < kChunks) && p < a.P)
        *reinterpret_cast<short8_t*>(obase + (int64_t)p * a.ldo + ch * 8) =
            *reinterpret_cast<const short8_t*>(orow + row * kOS + ch * 8);
    }
  }
  stamp(37);
}

template <int D, int WAVES, int QB, int BK, bool SCHED = true, int FORM = 0>
hipError_t launch(const SelfArgs& a, hipStream_t st) {
  SelfArgs b = a;
  b.n_qtiles = (a.P + 32 * QB * WAVES - 1) / (32 * QB * WAVES);
  dim3 grid(b.n_qtiles * a.H * a.N), block(64 * WAVES);
  launch_kernel((self40_kernel<D, WAVES, QB, BK, SCHED, FORM>), grid, block, 0, st, b);
  return hipGetLastError();
}

}  // namespace

bool self40_eligible(const SelfArgs& a, int d) {
  if (d == 40) return a.P >= 2048 && a.K >= 256;
  if (d == 80) return a.P >= 512 && a.K >= 256;
  return false;
}

// variant: 0 = production shapes; the experiments build also honours the A/B shapes below
// (every other measured shape is in git history; DESIGN.md §4 and profiles/ hold the logs)
int run_self40(const SelfArgs& a, int d, hipStream_t st) {
#ifdef S40_ONLY
  return (int)launch<S40_ONLY>(a, st);
#else
  if (d == 80) {
    switch (a.variant) {
#ifdef P2P_EXPERIMENTS
      case 164: return (int)launch<80, 8, 1, 128, true, 1 | 128 | 256 | 512 | 16384 | 16>(a, st);  // default + stamps
#endif
      // d = 80: 8 waves x ONE 32-row query block (two waves per SIMD), 128-key tiles, split staging
      // and the younger half's priority duty of the d = 40 kernel.  In the pipeline (bench.py,
      // HIP events) 36.8-37.2 -> 30.9-31.2 us against round 4's 4 waves x 2 blocks (one wave per
      // SIMD), which is as fast only with hot inputs: the second wave hides the cold Q / K / V
      // loads the layer meets after its QKV GEMM (profiles/r05/d80_ab/; 4 x 1 x 64: 34.0, 8 x 1 x
      // 64: 35.9, without split staging or priority: 32.0-33.0)
      default: return (int)launch<80, 8, 1, 128, true, 1 | 128 | 256 | 512 | 16384>(a, st);
    }
  }
  switch (a.variant) {
#ifdef P2P_EXPERIMENTS
    case 163: return (int)launch<40, 8, 2, 256, true, 17281 | 8388608 | 16>(a, st);   // default with clock stamps
#endif
    case 17281: return (int)launch<40, 8, 2, 256, true, 1 | 128 | 256 | 512 | 16384>(a, st);   // round-3 default
    // LEAN fragments, split staging (waves 0-3 K, 4-7 V), the younger half holding priority 1 on
    // three of every four steps (round 3: 0.1867 ms vs 0.1880-0.1885 for priority on alternate step
    // pairs and 0.2056 for round 2, profiles/r03/g1_ab/r03y_ab.log), and K's f16 range check as a
    // packed-u16 maximum (round 4: 0.1864-0.1865 vs 0.1881-0.1889 ms, profiles/r04/ab/g1_r04h.log)
    default: return (int)launch<40, 8, 2, 256, true, 1 | 128 | 256 | 512 | 16384 | 8388608>(a, st);
  }
#endif
}

}  // namespace p2p

#ifdef P2P_EXPERIMENTS
extern "C" int p2p_diag_self40_stamps(void* dst, int64_t bytes) {
  const int64_t n = (int64_t)sizeof(p2p::g_s40_stamps);
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(p2p::g_s40_stamps), bytes < n ? bytes : n, 0, hipMemcpyDeviceToHost);
}
#endif
