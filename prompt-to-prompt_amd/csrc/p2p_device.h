// Device-side building blocks for the Prompt-to-Prompt attention kernels (gfx950 / CDNA4).
//
// Fragment convention used by every kernel in this library:
//   * scores are computed TRANSPOSED, S^T = K * Q^T, with v_mfma_f32_32x32x16_bf16 (or the
//     exact-f32 v_mfma_f32_32x32x2_f32 in check mode).  A 32x32 S^T block leaves the query q on
//     the lane (q = lane & 31) and 16 keys in the 16 accumulator registers:
//         key(r, h) = (r & 3) + 8 * (r >> 2) + 4 * h,   h = lane >> 5.
//     A softmax row (one query) therefore lives in ONE lane pair (q, q+32): row max / row sum
//     are 16 register ops plus one cross-half exchange.
//   * the PV product is computed transposed too, O^T = V^T * P^T, with the S^T accumulator
//     used directly as the B operand (no LDS round trip for P).  O^T leaves q on the lane, so
//     the online-softmax rescale and the final 1/l are per-lane scalars.
//   * an "8-element k fragment" is the same data in both precisions: lane (row = lane&31,
//     h = lane>>5) holds elements k = 8h + j, j = 0..7.  bf16 packs them into one MFMA; f32
//     issues 8 MFMAs (k pair {j, 8+j} each), which sums the same 16 products.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace p2p {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) short short4_t;
typedef __attribute__((ext_vector_type(8))) short short8_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;

constexpr float kLog2e = 1.4426950408889634f;

__device__ __forceinline__ uint16_t f2bf(float x) {
  return __builtin_bit_cast(uint16_t, (__bf16)x);
}
__device__ __forceinline__ float bf2f(uint16_t x) {
  return __builtin_bit_cast(float, ((uint32_t)x) << 16);
}

// S^T / O^T accumulator row for register r of lane-half h.
__device__ __forceinline__ constexpr int acc_row(int r, int h) {
  return (r & 3) + 8 * (r >> 2) + 4 * h;
}

// ------------------------------------------------------------------ precision traits
// bf16 operands, f32 accumulate: the production path.
struct MmaBf16 {
  using elem = uint16_t;  // LDS / operand element
  struct frag {
    short8_t v;
  };
  static constexpr int kElemBytes = 2;

  __device__ __forceinline__ static void mma(f32x16_t& acc, const frag& a, const frag& b) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a.v),
                                                  __builtin_bit_cast(bf16x8_t, b.v), acc, 0, 0, 0);
  }
  __device__ __forceinline__ static elem from_float(float x) { return f2bf(x); }
  // 8 consecutive elements from LDS (16-byte aligned).
  __device__ __forceinline__ static frag load8(const elem* p) {
    frag f;
    f.v = *reinterpret_cast<const short8_t*>(p);
    return f;
  }
  __device__ __forceinline__ static frag zero() {
    frag f;
    f.v = short8_t{0, 0, 0, 0, 0, 0, 0, 0};
    return f;
  }
  // Pack accumulator registers [8s, 8s+8) of an S^T block into a B fragment.
  __device__ __forceinline__ static frag pack_p(const float* p) {
    frag f;
#pragma unroll
    for (int j = 0; j < 8; ++j) f.v[j] = (short)f2bf(p[j]);
    return f;
  }
};

// Exact f32 operands (v_mfma_f32_32x32x2_f32): the 1e-5 check mode.
struct MmaF32 {
  using elem = float;
  struct frag {
    float v[8];
  };
  static constexpr int kElemBytes = 4;

  __device__ __forceinline__ static void mma(f32x16_t& acc, const frag& a, const frag& b) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.v[j], b.v[j], acc, 0, 0, 0);
  }
  __device__ __forceinline__ static elem from_float(float x) { return x; }
  __device__ __forceinline__ static frag load8(const elem* p) {
    frag f;
    const f32x4_t a = *reinterpret_cast<const f32x4_t*>(p);
    const f32x4_t b = *reinterpret_cast<const f32x4_t*>(p + 4);
    f.v[0] = a[0]; f.v[1] = a[1]; f.v[2] = a[2]; f.v[3] = a[3];
    f.v[4] = b[0]; f.v[5] = b[1]; f.v[6] = b[2]; f.v[7] = b[3];
    return f;
  }
  __device__ __forceinline__ static frag zero() {
    frag f;
#pragma unroll
    for (int j = 0; j < 8; ++j) f.v[j] = 0.f;
    return f;
  }
  __device__ __forceinline__ static frag pack_p(const float* p) {
    frag f;
#pragma unroll
    for (int j = 0; j < 8; ++j) f.v[j] = p[j];
    return f;
  }
};

// ------------------------------------------------------------------ global I/O helpers
// Raw register staging: the global bytes of one 8-element chunk, converted at LDS-write time.
template <typename IO>
struct Chunk8;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;

// Buffer resource over [base, base + bytes): raw (stride 0) loads past `bytes` return zeros.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, int64_t bytes) {
  const int n = bytes > 0x7fffffff ? 0x7fffffff : (bytes < 0 ? 0 : (int)bytes);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, n, 0x00020000);
}

template <>
struct Chunk8<float> {
  f32x4_t a, b;
  __device__ __forceinline__ void load(const float* src) {
    a = *reinterpret_cast<const f32x4_t*>(src);
    b = *reinterpret_cast<const f32x4_t*>(src + 4);
  }
  __device__ __forceinline__ void load_buf(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    a = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
    b = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off + 16, 0, 0));
  }
  __device__ __forceinline__ void clear() {
    a = f32x4_t{0.f, 0.f, 0.f, 0.f};
    b = a;
  }
  __device__ __forceinline__ float at(int j) const { return j < 4 ? a[j] : b[j - 4]; }
  __device__ __forceinline__ void store(uint16_t* dst) const {
    short8_t v;
    v[0] = (short)f2bf(a[0]); v[1] = (short)f2bf(a[1]); v[2] = (short)f2bf(a[2]); v[3] = (short)f2bf(a[3]);
    v[4] = (short)f2bf(b[0]); v[5] = (short)f2bf(b[1]); v[6] = (short)f2bf(b[2]); v[7] = (short)f2bf(b[3]);
    *reinterpret_cast<short8_t*>(dst) = v;
  }
  __device__ __forceinline__ void store(float* dst) const {
    *reinterpret_cast<f32x4_t*>(dst) = a;
    *reinterpret_cast<f32x4_t*>(dst + 4) = b;
  }
  // split-bf16: hi = bf16(x), lo = bf16(x - hi), written to two planes
  __device__ __forceinline__ void store_split(uint16_t* hi, uint16_t* lo) const {
    short8_t vh, vl;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x = at(j);
      const uint16_t h = f2bf(x);
      vh[j] = (short)h;
      vl[j] = (short)f2bf(x - bf2f(h));
    }
    *reinterpret_cast<short8_t*>(hi) = vh;
    *reinterpret_cast<short8_t*>(lo) = vl;
  }
};
template <>
struct Chunk8<uint16_t> {
  short8_t v;
  __device__ __forceinline__ void load(const uint16_t* src) { v = *reinterpret_cast<const short8_t*>(src); }
  __device__ __forceinline__ void load_buf(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    v = __builtin_bit_cast(short8_t, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
  }
  __device__ __forceinline__ void clear() { v = short8_t{0, 0, 0, 0, 0, 0, 0, 0}; }
  __device__ __forceinline__ void store(uint16_t* dst) const { *reinterpret_cast<short8_t*>(dst) = v; }
  __device__ __forceinline__ void store(float* dst) const {
#pragma unroll
    for (int j = 0; j < 8; ++j) dst[j] = bf2f((uint16_t)v[j]);
  }
};

// ------------------------------------------------------------------ QK^T precision traits
// How S^T = K Q^T is formed.  K tiles live in LDS in `planes` planes of [rows][KS] elements
// (plane stride passed at the call site); Q fragments stay in registers.
//   QkBf16   : bf16 inputs, one bf16 MFMA per 16-deep k step (exact products of bf16 data)
//   QkSplit  : f32 inputs on the bf16 pipe, split-bf16 x = hi + lo, S = Kh Qh + Kh Ql + Kl Qh
//              (3 MFMAs; products to ~2^-16 relative, i.e. f32-grade logits)
//   QkF32    : exact f32 MFMA (check mode)
template <typename IO>
struct QkBf16 {
  using elem = uint16_t;
  static constexpr int planes = 1;
  static constexpr int kElemBytes = 2;
  struct frag {
    short8_t h;
  };
  __device__ __forceinline__ static frag zero() { return frag{short8_t{0, 0, 0, 0, 0, 0, 0, 0}}; }
  __device__ __forceinline__ static frag load_k(const elem* p, int) {
    return frag{*reinterpret_cast<const short8_t*>(p)};
  }
  __device__ __forceinline__ static frag load_q(const IO* src) {
    Chunk8<IO> c;
    c.load(src);
    frag f;
    uint16_t tmp[8] __attribute__((aligned(16)));
    c.store(tmp);
    f.h = *reinterpret_cast<const short8_t*>(tmp);
    return f;
  }
  __device__ __forceinline__ static void stage(const Chunk8<IO>& c, elem* dst, int) { c.store(dst); }
  __device__ __forceinline__ static void mma(f32x16_t& acc, const frag& k, const frag& q) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, k.h),
                                                  __builtin_bit_cast(bf16x8_t, q.h), acc, 0, 0, 0);
  }
};

struct QkSplit {
  using elem = uint16_t;
  static constexpr int planes = 2;
  static constexpr int kElemBytes = 2;
  struct frag {
    short8_t h, l;
  };
  __device__ __forceinline__ static frag zero() {
    return frag{short8_t{0, 0, 0, 0, 0, 0, 0, 0}, short8_t{0, 0, 0, 0, 0, 0, 0, 0}};
  }
  __device__ __forceinline__ static frag load_k(const elem* p, int plane) {
    return frag{*reinterpret_cast<const short8_t*>(p), *reinterpret_cast<const short8_t*>(p + plane)};
  }
  __device__ __forceinline__ static frag load_q(const float* src) {
    Chunk8<float> c;
    c.load(src);
    frag f;
    uint16_t h[8] __attribute__((aligned(16))), l[8] __attribute__((aligned(16)));
    c.store_split(h, l);
    f.h = *reinterpret_cast<const short8_t*>(h);
    f.l = *reinterpret_cast<const short8_t*>(l);
    return f;
  }
  __device__ __forceinline__ static void stage(const Chunk8<float>& c, elem* dst, int plane) {
    c.store_split(dst, dst + plane);
  }
  __device__ __forceinline__ static void mma(f32x16_t& acc, const frag& k, const frag& q) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, k.l),
                                                  __builtin_bit_cast(bf16x8_t, q.h), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, k.h),
                                                  __builtin_bit_cast(bf16x8_t, q.l), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, k.h),
                                                  __builtin_bit_cast(bf16x8_t, q.h), acc, 0, 0, 0);
  }
};

struct QkF32 {
  using elem = float;
  static constexpr int planes = 1;
  static constexpr int kElemBytes = 4;
  struct frag {
    float v[8];
  };
  __device__ __forceinline__ static frag zero() {
    frag f;
#pragma unroll
    for (int j = 0; j < 8; ++j) f.v[j] = 0.f;
    return f;
  }
  __device__ __forceinline__ static frag load_k(const elem* p, int) {
    frag f;
    const f32x4_t a = *reinterpret_cast<const f32x4_t*>(p);
    const f32x4_t b = *reinterpret_cast<const f32x4_t*>(p + 4);
    f.v[0] = a[0]; f.v[1] = a[1]; f.v[2] = a[2]; f.v[3] = a[3];
    f.v[4] = b[0]; f.v[5] = b[1]; f.v[6] = b[2]; f.v[7] = b[3];
    return f;
  }
  __device__ __forceinline__ static frag load_q(const float* src) { return load_k(src, 0); }
  __device__ __forceinline__ static void stage(const Chunk8<float>& c, elem* dst, int) { c.store(dst); }
  __device__ __forceinline__ static void mma(f32x16_t& acc, const frag& k, const frag& q) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(k.v[j], q.v[j], acc, 0, 0, 0);
  }
};

// Store 4 consecutive f32 results as IO elements.
__device__ __forceinline__ void store4(float* dst, float a, float b, float c, float d) {
  *reinterpret_cast<f32x4_t*>(dst) = f32x4_t{a, b, c, d};
}
__device__ __forceinline__ void store4(uint16_t* dst, float a, float b, float c, float d) {
  short4_t v;
  v[0] = (short)f2bf(a); v[1] = (short)f2bf(b); v[2] = (short)f2bf(c); v[3] = (short)f2bf(d);
  *reinterpret_cast<short4_t*>(dst) = v;
}

// AttentionStore read-add-write of one wave's [rows][K] block of post-edit maps: g (16-byte
// aligned, cnt = rows * K floats, cnt % 4 == 0) (+)= slab (the wave's LDS copy of the rows).
// Every running-sum read is issued first -- range-checked buffer loads (zeros past cnt), no
// branch, so they all fly together -- and only then the (masked) stores: ONE memory round trip.
// (Reads issued after stores would also wait for the stores: CDNA4's vmcnt counts both in order.)
// The same read-add-write in two halves, for a caller that issues the reads early (their values
// ride in registers until the slab is ready): rmw_load, then rmw_add_store.
template <int MAXF4>
__device__ __forceinline__ void rmw_load(const float* g, int cnt, int lane, f32x4_t (&buf)[(MAXF4 + 63) / 64]) {
  constexpr int IT = (MAXF4 + 63) / 64;
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(g, (int64_t)cnt * 4);
#pragma unroll
  for (int j = 0; j < IT; ++j)
    buf[j] = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, (lane + 64 * j) * 16, 0, 0));
}
template <int MAXF4>
__device__ __forceinline__ void rmw_add_store(float* g, const float* slab, int cnt, int lane,
                                              f32x4_t (&buf)[(MAXF4 + 63) / 64]) {
  constexpr int IT = (MAXF4 + 63) / 64;
  const int n4 = cnt / 4;
#pragma unroll
  for (int j = 0; j < IT; ++j) {
    const int i = lane + 64 * j;
    buf[j] += reinterpret_cast<const f32x4_t*>(slab)[i < n4 ? i : n4 - 1];
  }
#pragma unroll
  for (int j = 0; j < IT; ++j) {
    const int i = lane + 64 * j;
    if (i < n4) reinterpret_cast<f32x4_t*>(g)[i] = buf[j];
  }
}

template <int MAXF4>
__device__ __forceinline__ void store_rows_rmw(float* g, const float* slab, int cnt, bool accumulate, int lane) {
  constexpr int IT = (MAXF4 + 63) / 64;   // float4s per lane
  const int n4 = cnt / 4;
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(g, (int64_t)cnt * 4);
  f32x4_t buf[IT];
  if (accumulate) {
#pragma unroll
    for (int j = 0; j < IT; ++j)
      buf[j] = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, (lane + 64 * j) * 16, 0, 0));
  } else {
#pragma unroll
    for (int j = 0; j < IT; ++j) buf[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int j = 0; j < IT; ++j) {
    const int i = lane + 64 * j;
    buf[j] += reinterpret_cast<const f32x4_t*>(slab)[i < n4 ? i : n4 - 1];
  }
#pragma unroll
  for (int j = 0; j < IT; ++j) {
    const int i = lane + 64 * j;
    if (i < n4) reinterpret_cast<f32x4_t*>(g)[i] = buf[j];
  }
}

// ------------------------------------------------------------------ V^T operand fragments
// A operand of the PV MFMA for k-step s (16 keys) of a 32-key sub-block starting at LDS row
// `row0`, output columns [col0, col0+32): lane (d = lane&31, h) needs
//   V[row0 + 16s + 8(j>>2) + 4h + (j&3)][col0 + d],  j = 0..7
// which two ds_read_b64_tr_b16 deliver from a row-major [keys][VS] bf16 image.
template <int VS>
__device__ __forceinline__ MmaBf16::frag vt_frag(const uint16_t* V, int row0, int s, int col0, int lane) {
  const int h = lane >> 5;
  const int r = row0 + 16 * s + 4 * h + ((lane & 15) >> 2);
  const int c = col0 + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  typedef __attribute__((address_space(3))) short4_t lds_s4;
  const short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(V + r * VS + c));
  const short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(V + (r + 8) * VS + c));
  MmaBf16::frag f;
  f.v = short8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return f;
}

// PV for one 32-key sub-block with the transposed-accumulator convention, bf16 path:
// O[dt] += V^T[dt*32.., sub-block keys] * P^T[sub-block keys, q].
template <int VS, int NDT>
__device__ __forceinline__ void pv_block(MmaBf16, f32x16_t (&O)[NDT], const uint16_t* V, int row0,
                                         const float (&p)[16], int lane) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const MmaBf16::frag b = MmaBf16::pack_p(p + 8 * s);
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      const MmaBf16::frag a = vt_frag<VS>(V, row0, s, dt * 32, lane);
      MmaBf16::mma(O[dt], a, b);
    }
  }
}

// Exact-f32 path: 16 MFMAs (32x32x2) per sub-block and d-tile; MFMA t takes keys
// acc_row(t, h) from lane half h, which is exactly accumulator register t of the S^T block.
template <int VS, int NDT>
__device__ __forceinline__ void pv_block(MmaF32, f32x16_t (&O)[NDT], const float* V, int row0,
                                         const float (&p)[16], int lane) {
  const int h = lane >> 5;
  const int d = lane & 31;
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    const float* vr = V + (row0 + acc_row(t, h)) * VS + d;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
      O[dt] = __builtin_amdgcn_mfma_f32_32x32x2f32(vr[dt * 32], p[t], O[dt], 0, 0, 0);
  }
}

// ------------------------------------------------------------------ XCD-aware block remap
// Consecutive logical ids land on the same XCD (blocks b and b+8 share one under the
// observed round-robin dispatch); bijective for any grid size.  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7;
  const int q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// One global_load_lds_dwordx4 (16 bytes per lane into LDS at lds_off + lane * 16), as inline asm
// so hipcc does not track it: its own bookkeeping would drain every in-flight DMA with vmcnt(0)
// before the next LDS read of the ring (it cannot tell the stages apart).  The ring's waits are
// the explicit counted vmcnt below; the compiler's own waits only grow stricter with these newer
// operations in the in-order counter.  (cdna_hip_programming.md, the m0 recipe.)
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_off) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_off)
               : "memory");
}
// The value held by lane l ^ 32 (the other half of the wave), via v_permlane32_swap: no LDS
// round trip (ds_bpermute) on the softmax critical path.
__device__ __forceinline__ float other_half(float x) {
  const unsigned u = __float_as_uint(x);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  // r[0]: lanes 0-31 keep x, lanes 32-63 get the low half's x; r[1]: the high half's x everywhere
  return (threadIdx.x & 32) ? __uint_as_float(r[0]) : __uint_as_float(r[1]);
}

// Row stride (in elements) of an LDS tile read with ds_read_b128 by 16 distinct rows at the
// same column: a byte stride of 16 * odd spreads any 16 consecutive rows over all 16 slots.
template <int D, int ES>
struct KStride {
  static constexpr int bytes0 = D * ES;
  static constexpr int bytes = ((bytes0 / 16) % 2 == 0) ? bytes0 + 16 : bytes0;
  static constexpr int value = bytes / ES;
};

// Row stride (elements) of the bf16 V image read with ds_read_b64_tr_b16: the 4 rows x 2
// column groups one 32-lane half reads must fall on 8 distinct 8-dword bank slots, i.e.
// stride (dwords) = 16 or 48 mod 64.
template <int DV>
struct VStrideBf16 {
  static constexpr int dw0 = DV / 2;
  static constexpr int value = ((dw0 % 64) == 16 || (dw0 % 64) == 48) ? DV : (dw0 < 48 ? 96 : (dw0 < 80 ? 160 : 224));
};

}  // namespace p2p
