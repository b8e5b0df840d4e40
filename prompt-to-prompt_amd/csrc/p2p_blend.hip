// LocalBlend and AttentionStore helpers (bandwidth-bound, no MFMA).
//
// LocalBlend (null_text.py:41-70; main.py:35-52 is the two-prompt case):
//   maps   = cat_l reshape(store_l, [B, H, 1, 16, 16, W])           -> [B, L*H, 1, 16, 16, W]
//   m      = (maps * alpha).sum(-1).mean(1)                           -> [B, 1, 16, 16]
//   m      = max_pool2d(m, 3, 1, 1)          (pooled mask only)
//   m      = interpolate(m, x_t.shape[2:])   (nearest)
//   mask   = (m / max_{y,x} m) > th;  mask = mask[:1] | mask
//   mask  &= ~(substruct mask)               (optional, unpooled, th[1])
//   x_t    = x_t[:1] + mask * (x_t - x_t[:1])
// Kernel 1 reduces the word axis for every (prompt, layer x head) map; kernel 2 does the rest,
// one workgroup per prompt (each rebuilds prompt 0's mask, which gates every other prompt).
#include <type_traits>

#include "p2p_device.h"
#include "p2p_kernels.h"

namespace p2p {

constexpr int kBlendMaxPrompts = 16;

// grid (n_prompts, n_maps * heads, pixel chunks of kWsPix), 256 threads.  A chunk's rows
// [kWsPix, W] are one contiguous span of the store: the workgroup copies it to LDS with
// coalesced 16-byte loads, then every thread sums one pixel's words in index order.
constexpr int kWsPix = 64;

__global__ __launch_bounds__(256) void blend_wordsum_kernel(p2p_blend_args a) {
  const int b = blockIdx.x;
  const int j = blockIdx.y;                 // l * heads + hd
  const int l = j / a.heads_per_map;
  const int hd = j - l * a.heads_per_map;
  const int R2 = a.map_res * a.map_res;
  const int W = a.n_words;
  const int p0 = blockIdx.z * kWsPix;
  const int npix = min(kWsPix, R2 - p0);
  __shared__ float sa[128], ss[128];
  __shared__ __attribute__((aligned(16))) float rows[kWsPix * 128];
  for (int w = threadIdx.x; w < W; w += blockDim.x) {
    sa[w] = a.alpha_layers[b * W + w];
    ss[w] = a.substruct_layers ? a.substruct_layers[b * W + w] : 0.f;
  }
  const float* m = a.maps[l] + ((int64_t)(b * a.heads_per_map + hd) * R2 + p0) * W;
  const int n = npix * W;
  if ((((uintptr_t)m) & 15) == 0) {
    for (int i = threadIdx.x; i < n / 4; i += blockDim.x)
      reinterpret_cast<f32x4_t*>(rows)[i] = reinterpret_cast<const f32x4_t*>(m)[i];
    for (int i = (n & ~3) + threadIdx.x; i < n; i += blockDim.x) rows[i] = m[i];
  } else {
    for (int i = threadIdx.x; i < n; i += blockDim.x) rows[i] = m[i];
  }
  __syncthreads();
  const int pix = threadIdx.x;
  if (pix >= npix) return;
  const float* r = rows + pix * W;          // W odd (77): the 64 rows hit distinct banks
  float acc_a = 0.f, acc_s = 0.f;
  for (int w = 0; w < W; ++w) {
    const float v = r[w];
    acc_a += v * sa[w];
    acc_s += v * ss[w];
  }
  const int LH = a.n_maps * a.heads_per_map;
  a.word_sums[((int64_t)(b * 2 + 0) * LH + j) * R2 + p0 + pix] = acc_a;
  a.word_sums[((int64_t)(b * 2 + 1) * LH + j) * R2 + p0 + pix] = acc_s;
}

// x0 + m * (xb - x0) rounded exactly as the reference's three tensor ops (no fma contraction)
__device__ __forceinline__ float blend1(float x0, float xb, float m) {
#pragma clang fp contract(off)
  const float diff = xb - x0;
  const float t = m * diff;
  return x0 + t;
}

// one workgroup per prompt b: it rebuilds the source prompt's pooled mask next to its own (the
// source mask gates every prompt, mask = mask[:1] | mask), so the prompts run in parallel and no
// workgroup reads another's output (x_t[0] is never written: x_t[0] + mask * 0 == x_t[0])
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// LDS of one mask build (256 threads): mean maps, pooled maps, per-wave maxima, the mask per map
// pixel.  [0] = the group's source prompt, [1] = prompt b
struct BlendLds {
  float mean_a[2][256];
  float mean_s[2][256];
  float pooled[2][256];
  float red[4][4];
  float msrc[256];
};

// nearest upsampling (F.interpolate default): latent pixel yx -> map pixel
__device__ __forceinline__ int blend_src_of(int yx, int R, int lat_h, int lat_w) {
  const float sy = (float)R / (float)lat_h, sx = (float)R / (float)lat_w;
  const int Y = yx / lat_w, X = yx - Y * lat_w;
  return min((int)floorf(Y * sy), R - 1) * R + min((int)floorf(X * sx), R - 1);
}

// Prompt b's LocalBlend mask per map pixel (L.msrc, 1.f / 0.f) from the word sums of its group's
// source prompt (ws0) and its own (wsb), each [2, LH, R*R] (index 0: alpha-weighted, 1:
// substruct-weighted): mean over the LH maps, 3x3 max-pool, per-image max of the upsampled map,
// thresholds, mask[:1] | mask, substruct gate (null_text.py:41-67).  Called by all 256 threads of
// the workgroup (it synchronises); blend_finalize_kernel and latent_blend_kernel share it, so
// both build the same mask bit for bit.
__device__ __forceinline__ void build_blend_mask(const float* ws0, const float* wsb, int LH, int R, int lat_h, int lat_w,
                                 float th_pool, float th_sub, bool sub, BlendLds& L) {
  const int R2 = R * R;
  const int tid = threadIdx.x;
  // mean over the L*H maps (sum in index order, then / L*H as Tensor.mean does).  The four
  // (prompt, sum) planes -- source / b x alpha / substruct -- go to the four waves; a lane sums
  // four adjacent map pixels, so every load is one 16-byte row piece and a wave's LH loads of a
  // plane are all in flight at once (one memory round trip for the whole mask)
  {
    // (source | b) x (alpha | substruct); the wave index in a scalar register, so the plane's buffer
    // resource is scalar too (from a VGPR each of the 48 loads became a readfirstlane waterfall loop)
    const int g = __builtin_amdgcn_readfirstlane(tid >> 6), k = g & 1, sidx = g >> 1;
    const int px0 = (tid & 63) * 4;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    if (px0 < R2 && (sidx == 0 || sub)) {
      const float* base = (k ? wsb : ws0) + (int64_t)sidx * LH * R2;
      if ((R2 & 3) == 0) {
        // buffer loads: maps past LH read as 0 (range-checked), so the 48 loads of a batch are
        // issued unconditionally, all before the first add; adding those +0.0 to a sum of
        // non-negative terms leaves it bit for bit (the in-order sum over j < LH)
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(base, (int64_t)LH * R2 * 4);
        for (int j0 = 0; j0 < LH; j0 += 48) {
          f32x4_t v[48];
#pragma unroll
          for (int u = 0; u < 48; ++u)
            v[u] = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, ((j0 + u) * R2 + px0) * 4, 0, 0));
#pragma unroll
          for (int u = 0; u < 48; ++u)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[q] += v[u][q];
        }
      } else {
        for (int j = 0; j < LH; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (px0 + q < R2) acc[q] += base[(int64_t)j * R2 + px0 + q];
      }
    }
    float* const dst = sidx == 0 ? L.mean_a[k] : L.mean_s[k];
    float pmax = -INFINITY;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (px0 + q < R2) {
        const float mv = acc[q] / (float)LH;
        dst[px0 + q] = mv;
        pmax = fmaxf(pmax, mv);
      }
    // the wave holds its whole plane: its maximum needs no cross-wave reduction
    pmax = wave_max(pmax);
    if ((tid & 63) == 0) L.red[0][g] = pmax;
  }
  __syncthreads();
  if (lat_h >= R && lat_w >= R) {
    // Upsampling samples every map pixel, and a 3x3 max-pool keeps the plane's maximum (every
    // pixel lies in its own window), so the per-image maxima of the pooled / unpooled upsampled
    // maps are the four plane maxima above -- the same floats the generic path below reduces to.
    // Pool on the fly and threshold: one more barrier in all (mask per map pixel, gathered by the
    // nearest upsampling: identical per output pixel, evaluated R*R times instead of H*W)
    const float v0 = L.red[0][0], vb = L.red[0][1], s0m = L.red[0][2], sbm = L.red[0][3];
    for (int pix = tid; pix < R2; pix += 256) {
      const int y = pix / R, x = pix - y * R;
      float p0 = -INFINITY, pb = -INFINITY;
      for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
          const int yy = y + dy, xx = x + dx;
          if (yy >= 0 && yy < R && xx >= 0 && xx < R) {
            p0 = fmaxf(p0, L.mean_a[0][yy * R + xx]);
            pb = fmaxf(pb, L.mean_a[1][yy * R + xx]);
          }
        }
      bool mask = p0 / v0 > th_pool || pb / vb > th_pool;
      if (sub) mask = mask && !(L.mean_s[0][pix] / s0m > th_sub || L.mean_s[1][pix] / sbm > th_sub);
      L.msrc[pix] = mask ? 1.f : 0.f;
    }
    __syncthreads();
    return;
  }
  // generic path (latent smaller than the maps: the nearest down-sampling skips map pixels)
  // 3x3 max-pool, stride 1, padding 1 (padding never wins: -inf)
  for (int i = tid; i < 2 * R2; i += 256) {
    const int k = i / R2, pix = i - k * R2;
    const int y = pix / R, x = pix - y * R;
    float m = -INFINITY;
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        const int yy = y + dy, xx = x + dx;
        if (yy >= 0 && yy < R && xx >= 0 && xx < R) m = fmaxf(m, L.mean_a[k][yy * R + xx]);
      }
    L.pooled[k][pix] = m;
  }
  __syncthreads();
  // per-image max of the nearest-upsampled maps.  Upsampling (latent >= map resolution) samples
  // every source pixel, so the max over the grid is the max over the R*R sources.
  const bool all_sources = lat_h >= R && lat_w >= R;
  float m[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  for (int i = tid; i < (all_sources ? R2 : lat_h * lat_w); i += 256) {
    const int src = all_sources ? i : blend_src_of(i, R, lat_h, lat_w);
    m[0] = fmaxf(m[0], L.pooled[0][src]);
    m[1] = fmaxf(m[1], L.mean_s[0][src]);
    m[2] = fmaxf(m[2], L.pooled[1][src]);
    m[3] = fmaxf(m[3], L.mean_s[1][src]);
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) m[c] = wave_max(m[c]);
  if ((tid & 63) == 0)
#pragma unroll
    for (int c = 0; c < 4; ++c) L.red[tid >> 6][c] = m[c];
  __syncthreads();
  float vmax[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    vmax[c] = L.red[0][c];
    for (int w = 1; w < 4; ++w) vmax[c] = fmaxf(vmax[c], L.red[w][c]);
  }
  // mask of prompt b per source pixel (the thresholds of null_text.py:62-67), then gathered by
  // the nearest upsampling: identical per output pixel, evaluated R*R times instead of H*W
  for (int pix = tid; pix < R2; pix += 256) {
    const bool m0 = L.pooled[0][pix] / vmax[0] > th_pool;
    const bool mb = L.pooled[1][pix] / vmax[2] > th_pool;
    bool mask = m0 || mb;
    if (sub) {
      const bool s0 = L.mean_s[0][pix] / vmax[1] > th_sub;
      const bool sb = L.mean_s[1][pix] / vmax[3] > th_sub;
      mask = mask && !(s0 || sb);
    }
    L.msrc[pix] = mask ? 1.f : 0.f;
  }
  __syncthreads();
}

__global__ __launch_bounds__(256, 1) void blend_finalize_kernel(p2p_blend_args a) {
  const int b = blockIdx.x;
  const int R = a.map_res;
  const int R2 = R * R;
  const int LH = a.n_maps * a.heads_per_map;
  const int HW = a.lat_h * a.lat_w;
  __shared__ BlendLds L;
  build_blend_mask(a.word_sums, a.word_sums + (int64_t)b * 2 * LH * R2, LH, R, a.lat_h, a.lat_w, a.th_pool,
                   a.th_sub, a.substruct_layers != nullptr, L);
  // x_t[b] = x_t[0] + mask * (x_t[b] - x_t[0])
  for (int yx = threadIdx.x; yx < HW; yx += blockDim.x) {
    const float mf = L.msrc[blend_src_of(yx, R, a.lat_h, a.lat_w)];
    if (a.mask_out) a.mask_out[(int64_t)b * HW + yx] = mf != 0.f ? 1 : 0;
    if (b == 0 || !a.x_t) continue;  // x_t[0] + mask * 0 == x_t[0]; mask-only mode
    for (int ch = 0; ch < a.channels; ++ch) {
      const float x0 = a.x_t[(int64_t)(0 * a.channels + ch) * HW + yx];
      float* xb = a.x_t + (int64_t)(b * a.channels + ch) * HW + yx;
      *xb = blend1(x0, *xb, mf);
    }
  }
}

// dst = src * (1 / divisor): what `tensor / scalar` computes on the reference's cuda:0 device
// (the f32 reciprocal, then one multiply per element).
__global__ void store_scale_kernel(const float* __restrict__ src, float* __restrict__ dst, float inv, int64_t n) {
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride)
    reinterpret_cast<f32x4_t*>(dst)[i] = reinterpret_cast<const f32x4_t*>(src)[i] * inv;
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    dst[i] = src[i] * inv;
}

// ---------------------------------------------------------------- shader-clock probe
// Measurement only (bench.py's roofline clock): one wave per workgroup.  Each wave reads the
// shader-cycle counter (s_memtime: one tick per shader clock) and the constant 100 MHz counter
// (s_memrealtime), spins on the 100 MHz counter until `ticks` of it have passed, and reads both
// again -- clock = d(cycles) / d(ticks) x 100 MHz.  Both pairs are read in the same order, so the
// two windows are offset by the same read latency.  Consecutive workgroups land on different XCDs
// (round-robin dispatch), so n workgroups >= 8 sample every XCD.  Lanes 0 / 1 store (vector
// stores): out[2 wg] = cycles, out[2 wg + 1] = ticks.
__global__ void clock_probe_kernel(unsigned long long* __restrict__ out, unsigned ticks) {
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long r1 = r0;
  while (r1 - r0 < ticks) {
    __builtin_amdgcn_s_sleep(2);
    r1 = __builtin_amdgcn_s_memrealtime();
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x < 2) out[2 * blockIdx.x + threadIdx.x] = threadIdx.x == 0 ? c1 - c0 : r1 - r0;
}

// ---------------------------------------------------------------- fused latent update
// One denoising step's latent update (ptp_utils.py:72-75): classifier-free guidance
// (:73), the DDIM step (diffusers DDIMScheduler.step with eta = 0, restated by the reference as
// NullInversion.prev_step, null_text.py:471-479; the same formula with the inversion's
// coefficients is next_step, :481-489) and the LocalBlend latent blend with a precomputed mask
// (null_text.py:68-70 / main.py:50-52).  Every intermediate is rounded where the reference's
// torch ops round it: to bf16 for the products torch keeps in the U-Net's bf16 output dtype,
// to f32 elsewhere, with no fma contraction -- so the update is bit-identical to the eager
// sequence on the same inputs.
__device__ __forceinline__ float rnd_bf16(float x) { return bf2f(f2bf(x)); }

// explicit round-to-nearest ops: no fma contraction whatever the compile flags
__device__ __forceinline__ float mul_rn(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float add_rn(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float sub_rn(float a, float b) { return __fsub_rn(a, b); }

// prev_sample from one element's inputs (CFG combine + DDIM step): eu / ec the unconditional and
// conditional eps (ec unused without CFG), x the latent
// the step's scalar coefficients, copied out of the kernel-argument struct by value (a kernel that
// also indexes the struct's blend_sums[] array at run time would otherwise read every field through
// a vector load of the kernarg segment, one dependent round trip each)
struct DdimC {
  int cfg;
  float guidance, sqrt_beta_t, sqrt_alpha_t, sqrt_alpha_prev, sqrt_one_minus_alpha_prev;
  __device__ explicit DdimC(const p2p_latent_step_args& a)
      : cfg(a.cfg), guidance(a.guidance), sqrt_beta_t(a.sqrt_beta_t), sqrt_alpha_t(a.sqrt_alpha_t),
        sqrt_alpha_prev(a.sqrt_alpha_prev), sqrt_one_minus_alpha_prev(a.sqrt_one_minus_alpha_prev) {}
};

template <bool BF16, typename A>
__device__ __forceinline__ float ddim_from(const A& a, float eu, float ec, float x) {
  auto rd = [](float v) { return BF16 ? rnd_bf16(v) : v; };
  float noise;
  if (a.cfg) {
    const float diff = rd(sub_rn(ec, eu));
    const float gd = rd(mul_rn(a.guidance, diff));
    noise = rd(add_rn(eu, gd));
  } else {
    noise = eu;
  }
  // a 0-dim f32 factor times a bf16 tensor: torch casts the factor to bf16 first
  const float t1 = rd(mul_rn(rd(a.sqrt_beta_t), noise));
  const float x0 = __fdiv_rn(sub_rn(x, t1), a.sqrt_alpha_t);
  const float dir = rd(mul_rn(rd(a.sqrt_one_minus_alpha_prev), noise));
  return add_rn(mul_rn(a.sqrt_alpha_prev, x0), dir);
}

template <bool BF16>
__device__ __forceinline__ float eps_at(const p2p_latent_step_args& a, int64_t idx) {
  if constexpr (BF16) return bf2f(static_cast<const uint16_t*>(a.eps)[idx]);
  else return static_cast<const float*>(a.eps)[idx];
}

// prev_sample of prompt b at element i of its [C, H, W] latent
template <bool BF16>
__device__ __forceinline__ float ddim_prev(const p2p_latent_step_args& a, int b, int64_t i, int64_t chw) {
  const float eu = eps_at<BF16>(a, (int64_t)b * chw + i);
  const float ec = a.cfg ? eps_at<BF16>(a, (int64_t)(a.n_prompts + b) * chw + i) : 0.f;
  return ddim_from<BF16>(a, eu, ec, a.x[(int64_t)b * chw + i]);
}

template <bool BF16>
__global__ __launch_bounds__(256) void latent_step_kernel(p2p_latent_step_args a, int64_t chw) {
  const int HW = a.height * a.width;
  const int B = a.n_prompts;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int gs = a.group_size > 0 ? a.group_size : B;   // prompts per prompt group
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < chw; i += stride) {
    const int yx = (int)(i % HW);
    float prev0 = 0.f;
    bool blend = false;
    for (int b = 0; b < B; ++b) {
      const int bg = b % gs;                              // position inside its group
      float prev = ddim_prev<BF16>(a, b, i, chw);
      if (bg == 0) {
        prev0 = prev;                                     // the group's source prompt
        blend = a.mask && (!a.group_blend || a.group_blend[b / gs]);
      } else if (blend) {
        const float m = a.mask[(int64_t)b * HW + yx] ? 1.f : 0.f;
        prev = add_rn(prev0, mul_rn(m, sub_rn(prev, prev0)));
      }
      a.out[(int64_t)b * chw + i] = prev;
    }
  }
}

// The latent step with LocalBlend's mask built in the same launch (a.blend_sums): grid
// (pixel chunks of 256, prompts).  A workgroup of an edit prompt b whose group blends builds b's
// mask per map pixel from the folded word sums (build_blend_mask: ~160 KB of L2-resident sums, one
// round trip) and updates its chunk of b's latent -- recomputing the group source's prev_sample,
// which it blends towards, from the same inputs (bit-identical to the source workgroup's).  No
// workgroup reads another's output.  The kernel is latency-bound (1 MB per step): every thread
// issues its eps / x loads (4 pixels x 1 channel, for b and the source) before the mask build's,
// so the launch waits about two memory round trips; 64 workgroups keep the per-thread DDIM
// arithmetic (two IEEE divisions per element) short.
template <bool BF16>
__global__ __launch_bounds__(256, 1) void latent_blend_kernel(p2p_latent_step_args a, int64_t chw, int px_per_wg) {
  // every field this kernel reads, copied to scalars first (see DdimC)
  const int HW = a.height * a.width;
  const int b = blockIdx.y;
  const int NP = a.n_prompts, C = a.channels, H = a.height, W = a.width;
  const int gs = a.group_size > 0 ? a.group_size : NP;
  const int g = b / gs, bg = b - g * gs, b0 = b - bg;
  const float* const ws = a.blend_sums[g];
  const float* const xg = a.x;
  const void* const eg = a.eps;
  float* const og = a.out;
  const int lh = a.blend_lh, res = a.blend_res, use_sub = a.blend_sub;
  const float th_pool = a.blend_th_pool, th_sub = a.blend_th_sub;
  const DdimC dc(a);
  const bool blend = bg != 0 && ws != nullptr;          // workgroup-uniform
  __shared__ BlendLds L;
  // a workgroup covers px_per_wg = 256 pixels x 4 channels per pass: thread t takes channel
  // c0 + t / 64 and 4 adjacent pixels (16-byte pieces; HW % 4 == 0, checked by the launcher)
  const int px = blockIdx.x * px_per_wg + (threadIdx.x & 63) * 4;
  const int pxc = min(px, HW - 4);
  // raw loads first, unconditionally (clamped to valid addresses; the unused ones are discarded),
  // so no load sits in a branch with its own wait: every load of the pass is in flight at once
  using Raw = typename std::conditional<BF16, uint2, f32x4_t>::type;
  auto ld_eps = [eg](int64_t idx) __attribute__((always_inline)) -> Raw {
    if constexpr (BF16) return *reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(eg) + idx);
    else return *reinterpret_cast<const f32x4_t*>(static_cast<const float*>(eg) + idx);
  };
  auto unpack = [](const Raw& r) __attribute__((always_inline)) -> f32x4_t {
    if constexpr (BF16)
      return f32x4_t{__uint_as_float(r.x << 16), __uint_as_float(r.x & 0xffff0000u), __uint_as_float(r.y << 16),
                     __uint_as_float(r.y & 0xffff0000u)};
    else return r;
  };
  for (int c0 = 0; c0 < C; c0 += 4) {
    const int c = c0 + (threadIdx.x >> 6);
    const int64_t i = (int64_t)min(c, C - 1) * HW + pxc;
    Raw reu[2], rec[2];
    f32x4_t xv[2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int bb = s2 ? b0 : b;
      reu[s2] = ld_eps((int64_t)bb * chw + i);
      rec[s2] = ld_eps((int64_t)((dc.cfg ? NP : 0) + bb) * chw + i);
      xv[s2] = *reinterpret_cast<const f32x4_t*>(xg + (int64_t)bb * chw + i);
    }
    if (blend && c0 == 0) {
      const int R2 = res * res;
      build_blend_mask(ws, ws + (int64_t)bg * 2 * lh * R2, lh, res, H, W, th_pool, th_sub, use_sub != 0, L);
    }
    if (c >= C || px >= HW) continue;
    const f32x4_t eu = unpack(reu[0]), ec = unpack(rec[0]);
    f32x4_t o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float prev = ddim_from<BF16>(dc, eu[j], ec[j], xv[0][j]);
      if (blend) {
        const f32x4_t eu0 = unpack(reu[1]), ec0 = unpack(rec[1]);
        const float prev0 = ddim_from<BF16>(dc, eu0[j], ec0[j], xv[1][j]);
        const float m = L.msrc[blend_src_of(px + j, res, H, W)];
        prev = add_rn(prev0, mul_rn(m, sub_rn(prev, prev0)));
      }
      o[j] = prev;
    }
    *reinterpret_cast<f32x4_t*>(og + (int64_t)b * chw + (int64_t)c * HW + px) = o;
  }
}

int run_latent_step(const p2p_latent_step_args& a, hipStream_t st) {
  if (!a.eps || !a.x || !a.out || a.n_prompts < 1 || a.channels < 1 || a.height < 1 || a.width < 1 ||
      a.group_size < 0 || (a.group_size > 0 && a.n_prompts % a.group_size))
    return P2P_E_ARG;
  if (a.eps_dtype != P2P_DTYPE_F32 && a.eps_dtype != P2P_DTYPE_BF16) return P2P_E_DTYPE;
  const int64_t chw = (int64_t)a.channels * a.height * a.width;
  const int gs = a.group_size > 0 ? a.group_size : a.n_prompts;
  const int n_groups = a.n_prompts / gs;
  bool fused = false;
  for (int g = 0; g < P2P_MAX_GROUPS; ++g) {
    if (!a.blend_sums[g]) continue;
    if (g >= n_groups) return P2P_E_ARG;
    fused = true;
  }
  if (fused) {
    // the mask comes from the word sums; a precomputed mask as well would be ambiguous.  out must
    // not alias x: a source workgroup's writes would race with the edit workgroups' reads of x[g0]
    if (a.mask || a.group_blend || a.out == a.x || a.blend_lh < 1 || a.blend_res < 1 || (a.height * a.width) % 4 ||
        ((uintptr_t)a.x | (uintptr_t)a.out | (uintptr_t)a.eps) % 16 ||
        a.blend_res * a.blend_res > 256 || a.blend_res > a.height || a.blend_res > a.width)
      return P2P_E_ARG;
    constexpr int kPx = 256;    // latent pixels per workgroup (x 4 channels: 256 threads x 4 elements)
    const int hw = a.height * a.width;
    dim3 grid((hw + kPx - 1) / kPx, a.n_prompts);
    if (a.eps_dtype == P2P_DTYPE_BF16)
      launch_kernel(latent_blend_kernel<true>, grid, dim3(256), 0, st, a, chw, kPx);
    else
      launch_kernel(latent_blend_kernel<false>, grid, dim3(256), 0, st, a, chw, kPx);
    return (int)hipGetLastError();
  }
  int64_t blocks = (chw + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (a.eps_dtype == P2P_DTYPE_BF16)
    launch_kernel(latent_step_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, st, a, chw);
  else
    launch_kernel(latent_step_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, st, a, chw);
  return (int)hipGetLastError();
}

int run_localblend(const p2p_blend_args& a, hipStream_t st) {
  if (a.n_prompts < 1 || a.n_prompts > kBlendMaxPrompts || a.map_res * a.map_res > 256 || a.n_words > 128 ||
      a.n_maps < 1 || a.n_maps > 8 || !a.alpha_layers || (!a.x_t && !a.mask_out) || !a.word_sums ||
      a.lat_h < 1 || a.lat_w < 1)
    return P2P_E_ARG;
  for (int l = 0; l < a.n_maps; ++l)
    if (!a.maps[l] && !a.word_sums_ready) return P2P_E_ARG;
  dim3 g1(a.n_prompts, a.n_maps * a.heads_per_map, (a.map_res * a.map_res + kWsPix - 1) / kWsPix);
  if (!a.word_sums_ready) launch_kernel(blend_wordsum_kernel, g1, dim3(256), 0, st, a);
  launch_kernel(blend_finalize_kernel, dim3(a.n_prompts), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

int run_clock_probe(unsigned long long* out, int n_wg, int ticks, hipStream_t st) {
  launch_kernel(clock_probe_kernel, dim3((unsigned)n_wg), dim3(64), 0, st, out, (unsigned)ticks);
  return (int)hipGetLastError();
}

int run_store_scale(const float* src, float* dst, float divisor, int64_t n, hipStream_t st) {
  if (n <= 0) return 0;
  if (((uintptr_t)src | (uintptr_t)dst) & 15) return P2P_E_ALIGN;
  int64_t blocks = (n / 4 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 4096) blocks = 4096;
  const float inv = 1.0f / divisor;
  launch_kernel(store_scale_kernel, dim3((unsigned)blocks), dim3(256), 0, st, src, dst, inv, n);
  return (int)hipGetLastError();
}

}  // namespace p2p
