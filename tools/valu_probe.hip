// VALU / transcendental / MFMA issue-rate probe for gfx950 (planning aid for the attention kernels).
// Every wave runs ITER x 8 independent instructions of one kind; cycles per instruction per SIMD
// = (elapsed shader cycles) / (ITER * 8 * waves per SIMD).  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

constexpr int ITER = 2048;

#define OP8(op)                                                                                         \
  asm volatile(op " %0, %0\n\t" op " %1, %1\n\t" op " %2, %2\n\t" op " %3, %3\n\t" op " %4, %4\n\t" op \
               " %5, %5\n\t" op " %6, %6\n\t" op " %7, %7"                                              \
               : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7));

template <int KIND>
__global__ __launch_bounds__(256) void probe(float* out, long long* cyc) {
  float x0 = threadIdx.x * 1e-3f, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6,
        x7 = x0 + 7;
  f32x16 acc = {};
  bf16x8 a = {};
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITER; ++i) {
    if constexpr (KIND == 0) OP8("v_exp_f32")
    if constexpr (KIND == 1) OP8("v_exp_f16")
    if constexpr (KIND == 2) {
      asm volatile(
          "v_fma_f32 %0, %0, %0, %0\n\tv_fma_f32 %1, %1, %1, %1\n\tv_fma_f32 %2, %2, %2, %2\n\tv_fma_f32 %3, %3, %3, %3\n\t"
          "v_fma_f32 %4, %4, %4, %4\n\tv_fma_f32 %5, %5, %5, %5\n\tv_fma_f32 %6, %6, %6, %6\n\tv_fma_f32 %7, %7, %7, %7"
          : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7));
    }
    if constexpr (KIND == 3) {
      asm volatile(
          "v_max3_f32 %0, %0, %1, %2\n\tv_max3_f32 %1, %1, %2, %3\n\tv_max3_f32 %2, %2, %3, %4\n\tv_max3_f32 %3, %3, %4, %5\n\t"
          "v_max3_f32 %4, %4, %5, %6\n\tv_max3_f32 %5, %5, %6, %7\n\tv_max3_f32 %6, %6, %7, %0\n\tv_max3_f32 %7, %7, %0, %1"
          : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7));
    }
    if constexpr (KIND == 4) {  // exp and fma alternating: do they co-issue?
      asm volatile(
          "v_exp_f32 %0, %0\n\tv_fma_f32 %1, %1, %1, %1\n\tv_exp_f32 %2, %2\n\tv_fma_f32 %3, %3, %3, %3\n\t"
          "v_exp_f32 %4, %4\n\tv_fma_f32 %5, %5, %5, %5\n\tv_exp_f32 %6, %6\n\tv_fma_f32 %7, %7, %7, %7"
          : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7));
    }
    if constexpr (KIND == 5) {
      asm volatile(
          "v_cvt_pk_bf16_f32 %0, %0, %1\n\tv_cvt_pk_bf16_f32 %1, %1, %2\n\tv_cvt_pk_bf16_f32 %2, %2, %3\n\t"
          "v_cvt_pk_bf16_f32 %3, %3, %4\n\tv_cvt_pk_bf16_f32 %4, %4, %5\n\tv_cvt_pk_bf16_f32 %5, %5, %6\n\t"
          "v_cvt_pk_bf16_f32 %6, %6, %7\n\tv_cvt_pk_bf16_f32 %7, %7, %0"
          : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7));
    }
    if constexpr (KIND == 6) {  // packed f32 fma: 2 values per instruction
      typedef __attribute__((ext_vector_type(2))) float f2;
      f2 y0 = {x0, x1}, y1 = {x2, x3}, y2 = {x4, x5}, y3 = {x6, x7};
      asm volatile(
          "v_pk_fma_f32 %0, %0, %0, %0\n\tv_pk_fma_f32 %1, %1, %1, %1\n\tv_pk_fma_f32 %2, %2, %2, %2\n\tv_pk_fma_f32 %3, %3, %3, %3\n\t"
          "v_pk_fma_f32 %0, %0, %0, %0\n\tv_pk_fma_f32 %1, %1, %1, %1\n\tv_pk_fma_f32 %2, %2, %2, %2\n\tv_pk_fma_f32 %3, %3, %3, %3"
          : "+v"(y0), "+v"(y1), "+v"(y2), "+v"(y3));
      x0 = y0[0]; x1 = y0[1]; x2 = y1[0]; x3 = y1[1]; x4 = y2[0]; x5 = y2[1]; x6 = y3[0]; x7 = y3[1];
    }
    if constexpr (KIND == 7) {  // MFMA only (independent chain, 8 per iteration)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, a, acc, 0, 0, 0);
    }
    if constexpr (KIND == 8) {  // 8 exp + 1 MFMA per iteration in the same wave
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, a, acc, 0, 0, 0);
      OP8("v_exp_f32")
    }
    if constexpr (KIND == 9) {  // 8 fma + 1 MFMA
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, a, acc, 0, 0, 0);
      asm volatile(
          "v_fma_f32 %0, %0, %0, %0\n\tv_fma_f32 %1, %1, %1, %1\n\tv_fma_f32 %2, %2, %2, %2\n\tv_fma_f32 %3, %3, %3, %3\n\t"
          "v_fma_f32 %4, %4, %4, %4\n\tv_fma_f32 %5, %5, %5, %5\n\tv_fma_f32 %6, %6, %6, %6\n\tv_fma_f32 %7, %7, %7, %7"
          : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7));
    }
    if constexpr (KIND == 10) OP8("v_mov_b32")
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
  for (int r = 0; r < 16; ++r) s += acc[r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND>
void run(const char* name, float* out, long long* cyc, long long* hcyc) {
  for (int wps : {1, 2, 4, 8}) {   // waves per SIMD: 256-thread blocks, 4 waves (one per SIMD) each
    const int blocks = 256 * wps;
    hipLaunchKernelGGL(probe<KIND>, dim3(blocks), dim3(256), 0, 0, out, cyc);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(probe<KIND>, dim3(blocks), dim3(256), 0, 0, out, cyc);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    hipMemcpy(hcyc, cyc, blocks * sizeof(long long), hipMemcpyDeviceToHost);
    long long mx = 0;
    for (int i = 0; i < blocks; ++i) mx = hcyc[i] > mx ? hcyc[i] : mx;
    // per-wave cycles / instructions; per-SIMD throughput = wave cycles / (instr * wps)
    const double instr = (double)ITER * 8;
    printf("%-22s wps=%d  wave_cyc/instr=%.2f  simd_cyc/instr=%.2f  wall=%.3f ms\n", name, wps, mx / instr,
           mx / instr / wps, ms);
  }
}

int main() {
  float* out;
  long long *cyc, *hcyc;
  hipMalloc(&out, 256 * 8 * 256 * sizeof(float));
  hipMalloc(&cyc, 256 * 8 * sizeof(long long));
  hcyc = (long long*)malloc(256 * 8 * sizeof(long long));
  run<0>("v_exp_f32", out, cyc, hcyc);
  run<1>("v_exp_f16", out, cyc, hcyc);
  run<2>("v_fma_f32", out, cyc, hcyc);
  run<3>("v_max3_f32", out, cyc, hcyc);
  run<4>("exp+fma alternating", out, cyc, hcyc);
  run<5>("v_cvt_pk_bf16_f32", out, cyc, hcyc);
  run<6>("v_pk_fma_f32", out, cyc, hcyc);
  run<7>("mfma32x32x16 (per mfma)", out, cyc, hcyc);
  run<8>("1 mfma + 8 exp (per op)", out, cyc, hcyc);
  run<9>("1 mfma + 8 fma (per op)", out, cyc, hcyc);
  run<10>("v_mov_b32", out, cyc, hcyc);
  return 0;
}
