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
// Kernel 1 reduces the word axis for every (prompt, layer x head) map; kernel 2 does the rest
// for the whole prompt group in one workgroup (the mask of prompt 0 gates every other prompt).
#include "p2p_device.h"
#include "p2p_kernels.h"

namespace p2p {

constexpr int kBlendMaxPrompts = 16;

// grid (n_prompts, n_maps * heads), block = res*res threads (one per pixel)
__global__ __launch_bounds__(256) void blend_wordsum_kernel(p2p_blend_args a) {
  const int b = blockIdx.x;
  const int j = blockIdx.y;                 // l * heads + hd
  const int l = j / a.heads_per_map;
  const int hd = j - l * a.heads_per_map;
  const int R2 = a.map_res * a.map_res;
  const int W = a.n_words;
  __shared__ float sa[128], ss[128];
  for (int w = threadIdx.x; w < W; w += blockDim.x) {
    sa[w] = a.alpha_layers[b * W + w];
    ss[w] = a.substruct_layers ? a.substruct_layers[b * W + w] : 0.f;
  }
  __syncthreads();
  const int pix = threadIdx.x;
  if (pix >= R2) return;
  const float* m = a.maps[l] + ((int64_t)(b * a.heads_per_map + hd) * R2 + pix) * W;
  float acc_a = 0.f, acc_s = 0.f;
  for (int w = 0; w < W; ++w) {
    const float v = m[w];
    acc_a += v * sa[w];
    acc_s += v * ss[w];
  }
  const int LH = a.n_maps * a.heads_per_map;
  a.word_sums[((int64_t)(b * 2 + 0) * LH + j) * R2 + pix] = acc_a;
  a.word_sums[((int64_t)(b * 2 + 1) * LH + j) * R2 + pix] = acc_s;
}

// x0 + m * (xb - x0) rounded exactly as the reference's three tensor ops (no fma contraction)
__device__ __forceinline__ float blend1(float x0, float xb, float m) {
#pragma clang fp contract(off)
  const float diff = xb - x0;
  const float t = m * diff;
  return x0 + t;
}

// one workgroup for the whole prompt group
__global__ __launch_bounds__(256) void blend_finalize_kernel(p2p_blend_args a) {
  const int B = a.n_prompts;
  const int R = a.map_res;
  const int R2 = R * R;
  const int LH = a.n_maps * a.heads_per_map;
  const int HW = a.lat_h * a.lat_w;
  __shared__ float mean_a[kBlendMaxPrompts][256];
  __shared__ float mean_s[kBlendMaxPrompts][256];
  __shared__ float pooled[kBlendMaxPrompts][256];
  __shared__ float vmax[kBlendMaxPrompts][2];
  const int tid = threadIdx.x;
  const bool sub = a.substruct_layers != nullptr;

  // mean over the L*H maps (sum in index order, then / L*H as Tensor.mean does)
  for (int i = tid; i < B * R2; i += blockDim.x) {
    const int b = i / R2, pix = i - b * R2;
    float sa = 0.f, ss = 0.f;
    for (int j = 0; j < LH; ++j) {
      sa += a.word_sums[((int64_t)(b * 2 + 0) * LH + j) * R2 + pix];
      ss += a.word_sums[((int64_t)(b * 2 + 1) * LH + j) * R2 + pix];
    }
    mean_a[b][pix] = sa / (float)LH;
    mean_s[b][pix] = ss / (float)LH;
  }
  __syncthreads();
  // 3x3 max-pool, stride 1, padding 1 (padding never wins: -inf)
  for (int i = tid; i < B * R2; i += blockDim.x) {
    const int b = i / R2, pix = i - b * R2;
    const int y = pix / R, x = pix - y * R;
    float m = -INFINITY;
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        const int yy = y + dy, xx = x + dx;
        if (yy >= 0 && yy < R && xx >= 0 && xx < R) m = fmaxf(m, mean_a[b][yy * R + xx]);
      }
    pooled[b][pix] = m;
  }
  __syncthreads();
  // per-image max of the nearest-upsampled maps: a block-wide max over the upsampled grid
  const float sy = (float)R / (float)a.lat_h, sx = (float)R / (float)a.lat_w;
  __shared__ float red[2][256];
  for (int b = 0; b < B; ++b) {
    float m0 = -INFINITY, m1 = -INFINITY;
    for (int yx = tid; yx < HW; yx += blockDim.x) {
      const int Y = yx / a.lat_w, X = yx - Y * a.lat_w;
      const int src = min((int)floorf(Y * sy), R - 1) * R + min((int)floorf(X * sx), R - 1);
      m0 = fmaxf(m0, pooled[b][src]);
      m1 = fmaxf(m1, mean_s[b][src]);
    }
    red[0][tid] = m0;
    red[1][tid] = m1;
    __syncthreads();
    for (int s2 = blockDim.x / 2; s2 > 0; s2 >>= 1) {
      if (tid < s2) {
        red[0][tid] = fmaxf(red[0][tid], red[0][tid + s2]);
        red[1][tid] = fmaxf(red[1][tid], red[1][tid + s2]);
      }
      __syncthreads();
    }
    if (tid == 0) {
      vmax[b][0] = red[0][0];
      vmax[b][1] = red[1][0];
    }
    __syncthreads();
  }
  // masks + latent blend: x_t[b] = x_t[0] + mask * (x_t[b] - x_t[0])
  for (int i = tid; i < B * HW; i += blockDim.x) {
    const int b = i / HW, yx = i - b * HW;
    const int Y = yx / a.lat_w, X = yx - Y * a.lat_w;
    const int src = min((int)floorf(Y * sy), R - 1) * R + min((int)floorf(X * sx), R - 1);
    bool m0 = pooled[0][src] / vmax[0][0] > a.th_pool;
    bool mb = pooled[b][src] / vmax[b][0] > a.th_pool;
    bool mask = m0 || mb;
    if (sub) {
      const bool s0 = mean_s[0][src] / vmax[0][1] > a.th_sub;
      const bool sb = mean_s[b][src] / vmax[b][1] > a.th_sub;
      mask = mask && !(s0 || sb);
    }
    const float mf = mask ? 1.f : 0.f;
    if (a.mask_out) a.mask_out[(int64_t)b * HW + yx] = mask ? 1 : 0;
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

template <bool BF16>
__global__ __launch_bounds__(256) void latent_step_kernel(p2p_latent_step_args a, int64_t chw) {
  const int HW = a.height * a.width;
  const int B = a.n_prompts;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  auto rd = [](float x) { return BF16 ? rnd_bf16(x) : x; };
  auto ld = [&](int64_t idx) {
    if constexpr (BF16) return bf2f(static_cast<const uint16_t*>(a.eps)[idx]);
    else return static_cast<const float*>(a.eps)[idx];
  };
  const int gs = a.group_size > 0 ? a.group_size : B;   // prompts per prompt group
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < chw; i += stride) {
    const int yx = (int)(i % HW);
    float prev0 = 0.f;
    bool blend = false;
    for (int b = 0; b < B; ++b) {
      const int bg = b % gs;                              // position inside its group
      float noise;
      if (a.cfg) {
        const float eu = ld((int64_t)b * chw + i);
        const float ec = ld((int64_t)(B + b) * chw + i);
        const float diff = rd(sub_rn(ec, eu));
        const float gd = rd(mul_rn(a.guidance, diff));
        noise = rd(add_rn(eu, gd));
      } else {
        noise = ld((int64_t)b * chw + i);
      }
      const float x = a.x[(int64_t)b * chw + i];
      // a 0-dim f32 factor times a bf16 tensor: torch casts the factor to bf16 first
      const float t1 = rd(mul_rn(rd(a.sqrt_beta_t), noise));
      const float x0 = __fdiv_rn(sub_rn(x, t1), a.sqrt_alpha_t);
      const float dir = rd(mul_rn(rd(a.sqrt_one_minus_alpha_prev), noise));
      float prev = add_rn(mul_rn(a.sqrt_alpha_prev, x0), dir);
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

int run_latent_step(const p2p_latent_step_args& a, hipStream_t st) {
  if (!a.eps || !a.x || !a.out || a.n_prompts < 1 || a.channels < 1 || a.height < 1 || a.width < 1 ||
      a.group_size < 0 || (a.group_size > 0 && a.n_prompts % a.group_size))
    return P2P_E_ARG;
  if (a.eps_dtype != P2P_DTYPE_F32 && a.eps_dtype != P2P_DTYPE_BF16) return P2P_E_DTYPE;
  const int64_t chw = (int64_t)a.channels * a.height * a.width;
  int64_t blocks = (chw + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (a.eps_dtype == P2P_DTYPE_BF16)
    hipLaunchKernelGGL(latent_step_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, st, a, chw);
  else
    hipLaunchKernelGGL(latent_step_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, st, a, chw);
  return (int)hipGetLastError();
}

int run_localblend(const p2p_blend_args& a, hipStream_t st) {
  if (a.n_prompts < 1 || a.n_prompts > kBlendMaxPrompts || a.map_res * a.map_res > 256 || a.n_words > 128 ||
      a.n_maps < 1 || a.n_maps > 8 || !a.alpha_layers || (!a.x_t && !a.mask_out) || !a.word_sums ||
      a.lat_h < 1 || a.lat_w < 1)
    return P2P_E_ARG;
  for (int l = 0; l < a.n_maps; ++l)
    if (!a.maps[l]) return P2P_E_ARG;
  dim3 g1(a.n_prompts, a.n_maps * a.heads_per_map);
  hipLaunchKernelGGL(blend_wordsum_kernel, g1, dim3(256), 0, st, a);
  hipLaunchKernelGGL(blend_finalize_kernel, dim3(1), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

int run_store_scale(const float* src, float* dst, float divisor, int64_t n, hipStream_t st) {
  if (n <= 0) return 0;
  if (((uintptr_t)src | (uintptr_t)dst) & 15) return P2P_E_ALIGN;
  int64_t blocks = (n / 4 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 4096) blocks = 4096;
  const float inv = 1.0f / divisor;
  hipLaunchKernelGGL(store_scale_kernel, dim3((unsigned)blocks), dim3(256), 0, st, src, dst, inv, n);
  return (int)hipGetLastError();
}

}  // namespace p2p
