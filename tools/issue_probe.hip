// Issue-cost probe for the softmax forms of the d = 40 self-attention kernel (gfx950).
// Every wave runs ITER "blocks"; a block is the per-32x32-score-block instruction mix of the
// kernel's inner loop, written as inline asm so the order is fixed:
//   A (bf16 P, today):  7 MFMA 32x32x16 + 16 v_exp_f32 + 8 v_cvt_pk_bf16_f32
//   B (f16 P):          7 MFMA 32x32x16 + 8 v_cvt_pk_f16_f32 + 16 v_exp_f16 (SDWA, in place per half)
//   plus the pieces alone (VALU only) to price each instruction.
// Cycles per block per SIMD = wave cycles / (ITER * waves per SIMD).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/issue_probe tools/issue_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

constexpr int ITER = 1024;

#define R8 "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)

// 16 v_exp_f32 on 8 registers (twice each)
#define EXP32_16                                                                                      \
  "v_exp_f32 %0, %0\n\tv_exp_f32 %1, %1\n\tv_exp_f32 %2, %2\n\tv_exp_f32 %3, %3\n\t"                  \
  "v_exp_f32 %4, %4\n\tv_exp_f32 %5, %5\n\tv_exp_f32 %6, %6\n\tv_exp_f32 %7, %7\n\t"                  \
  "v_exp_f32 %0, %0\n\tv_exp_f32 %1, %1\n\tv_exp_f32 %2, %2\n\tv_exp_f32 %3, %3\n\t"                  \
  "v_exp_f32 %4, %4\n\tv_exp_f32 %5, %5\n\tv_exp_f32 %6, %6\n\tv_exp_f32 %7, %7\n\t"
#define EXPF16_LO(r) "v_exp_f16_sdwa " r ", " r " dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0\n\t"
#define EXPF16_HI(r) "v_exp_f16_sdwa " r ", " r " dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"

template <int KIND>
__global__ __launch_bounds__(256) void probe(float* out, long long* cyc) {
  float x0 = threadIdx.x * 1e-3f, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6,
        x7 = x0 + 7;
  float y0 = x0 * 0.5f, y1 = x1 * 0.5f;
  f32x16 acc0 = {}, acc1 = {};
  bf16x8 a = {};
  for (int j = 0; j < 8; ++j) a[j] = (__bf16)(threadIdx.x * 0.01f + j);
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITER; ++i) {
    if constexpr (KIND == 0) asm volatile(EXP32_16 : R8);
    if constexpr (KIND == 1)
      asm volatile(EXPF16_LO("%0") EXPF16_LO("%1") EXPF16_LO("%2") EXPF16_LO("%3") EXPF16_LO("%4") EXPF16_LO("%5")
                       EXPF16_LO("%6") EXPF16_LO("%7") EXPF16_HI("%0") EXPF16_HI("%1") EXPF16_HI("%2")
                           EXPF16_HI("%3") EXPF16_HI("%4") EXPF16_HI("%5") EXPF16_HI("%6") EXPF16_HI("%7")
                   : R8);
    if constexpr (KIND == 2)   // plain VOP1 v_exp_f16 (16 per block)
      asm volatile(
          "v_exp_f16 %0, %0\n\tv_exp_f16 %1, %1\n\tv_exp_f16 %2, %2\n\tv_exp_f16 %3, %3\n\t"
          "v_exp_f16 %4, %4\n\tv_exp_f16 %5, %5\n\tv_exp_f16 %6, %6\n\tv_exp_f16 %7, %7\n\t"
          "v_exp_f16 %0, %0\n\tv_exp_f16 %1, %1\n\tv_exp_f16 %2, %2\n\tv_exp_f16 %3, %3\n\t"
          "v_exp_f16 %4, %4\n\tv_exp_f16 %5, %5\n\tv_exp_f16 %6, %6\n\tv_exp_f16 %7, %7"
          : R8);
    if constexpr (KIND == 3)   // 8 v_cvt_pk_bf16_f32
      asm volatile(
          "v_cvt_pk_bf16_f32 %0, %0, %1\n\tv_cvt_pk_bf16_f32 %1, %1, %2\n\tv_cvt_pk_bf16_f32 %2, %2, %3\n\t"
          "v_cvt_pk_bf16_f32 %3, %3, %4\n\tv_cvt_pk_bf16_f32 %4, %4, %5\n\tv_cvt_pk_bf16_f32 %5, %5, %6\n\t"
          "v_cvt_pk_bf16_f32 %6, %6, %7\n\tv_cvt_pk_bf16_f32 %7, %7, %0"
          : R8);
    if constexpr (KIND == 4)   // 8 v_cvt_pk_f16_f32
      asm volatile(
          "v_cvt_pk_f16_f32 %0, %0, %1\n\tv_cvt_pk_f16_f32 %1, %1, %2\n\tv_cvt_pk_f16_f32 %2, %2, %3\n\t"
          "v_cvt_pk_f16_f32 %3, %3, %4\n\tv_cvt_pk_f16_f32 %4, %4, %5\n\tv_cvt_pk_f16_f32 %5, %5, %6\n\t"
          "v_cvt_pk_f16_f32 %6, %6, %7\n\tv_cvt_pk_f16_f32 %7, %7, %0"
          : R8);
    if constexpr (KIND == 5)   // 8 v_cvt_pkrtz_f16_f32
      asm volatile(
          "v_cvt_pkrtz_f16_f32 %0, %0, %1\n\tv_cvt_pkrtz_f16_f32 %1, %1, %2\n\tv_cvt_pkrtz_f16_f32 %2, %2, %3\n\t"
          "v_cvt_pkrtz_f16_f32 %3, %3, %4\n\tv_cvt_pkrtz_f16_f32 %4, %4, %5\n\tv_cvt_pkrtz_f16_f32 %5, %5, %6\n\t"
          "v_cvt_pkrtz_f16_f32 %6, %6, %7\n\tv_cvt_pkrtz_f16_f32 %7, %7, %0"
          : R8);
    if constexpr (KIND == 6) {   // A: 7 MFMA + 16 exp_f32 + 8 cvt_pk_bf16, interleaved
      asm volatile(
          "v_mfma_f32_32x32x16_bf16 %8, %10, %10, %8\n\t"
          "v_exp_f32 %0, %0\n\tv_exp_f32 %1, %1\n\tv_cvt_pk_bf16_f32 %2, %2, %3\n\t"
          "v_mfma_f32_32x32x16_bf16 %9, %10, %10, %9\n\t"
          "v_exp_f32 %4, %4\n\tv_exp_f32 %5, %5\n\tv_cvt_pk_bf16_f32 %6, %6, %7\n\t"
          "v_mfma_f32_32x32x16_bf16 %8, %10, %10, %8\n\t"
          "v_exp_f32 %2, %2\n\tv_exp_f32 %3, %3\n\tv_cvt_pk_bf16_f32 %0, %0, %1\n\t"
          "v_mfma_f32_32x32x16_bf16 %9, %10, %10, %9\n\t"
          "v_exp_f32 %6, %6\n\tv_exp_f32 %7, %7\n\tv_cvt_pk_bf16_f32 %4, %4, %5\n\tv_exp_f32 %0, %0\n\t"
          "v_mfma_f32_32x32x16_bf16 %8, %10, %10, %8\n\t"
          "v_exp_f32 %1, %1\n\tv_exp_f32 %2, %2\n\tv_cvt_pk_bf16_f32 %3, %3, %4\n\tv_exp_f32 %4, %4\n\t"
          "v_mfma_f32_32x32x16_bf16 %9, %10, %10, %9\n\t"
          "v_exp_f32 %5, %5\n\tv_exp_f32 %6, %6\n\tv_cvt_pk_bf16_f32 %7, %7, %0\n\tv_exp_f32 %7, %7\n\t"
          "v_mfma_f32_32x32x16_bf16 %8, %10, %10, %8\n\t"
          "v_exp_f32 %3, %3\n\tv_cvt_pk_bf16_f32 %1, %1, %2\n\tv_cvt_pk_bf16_f32 %5, %5, %6\n\t"
          : R8, "+v"(acc0), "+v"(acc1)
          : "v"(a));
    }
    if constexpr (KIND == 7) {   // B: 7 MFMA + 8 cvt_pk_f16 + 16 exp_f16 (SDWA halves), interleaved
      asm volatile(
          "v_mfma_f32_32x32x16_bf16 %8, %10, %10, %8\n\t"
          "v_cvt_pk_f16_f32 %0, %0, %1\n\t" EXPF16_LO("%2") EXPF16_HI("%2") EXPF16_LO("%3")
          "v_mfma_f32_32x32x16_bf16 %9, %10, %10, %9\n\t"
          "v_cvt_pk_f16_f32 %1, %1, %4\n\t" EXPF16_HI("%3") EXPF16_LO("%0") EXPF16_HI("%0")
          "v_mfma_f32_32x32x16_bf16 %8, %10, %10, %8\n\t"
          "v_cvt_pk_f16_f32 %4, %4, %5\n\t" EXPF16_LO("%1") EXPF16_HI("%1") EXPF16_LO("%6")
          "v_mfma_f32_32x32x16_bf16 %9, %10, %10, %9\n\t"
          "v_cvt_pk_f16_f32 %5, %5, %7\n\t" EXPF16_HI("%6") EXPF16_LO("%4") EXPF16_HI("%4")
          "v_mfma_f32_32x32x16_bf16 %8, %10, %10, %8\n\t"
          "v_cvt_pk_f16_f32 %2, %2, %6\n\t" EXPF16_LO("%5") EXPF16_HI("%5") EXPF16_LO("%7")
          "v_mfma_f32_32x32x16_bf16 %9, %10, %10, %9\n\t"
          "v_cvt_pk_f16_f32 %3, %3, %6\n\t" EXPF16_HI("%7") EXPF16_LO("%2") EXPF16_HI("%2")
          "v_mfma_f32_32x32x16_bf16 %8, %10, %10, %8\n\t"
          "v_cvt_pk_f16_f32 %6, %6, %0\n\tv_cvt_pk_f16_f32 %7, %7, %1\n\t"
          : R8, "+v"(acc0), "+v"(acc1)
          : "v"(a));
    }
    if constexpr (KIND == 8) {   // 7 MFMA alone
      asm volatile(
          "v_mfma_f32_32x32x16_bf16 %0, %2, %2, %0\n\tv_mfma_f32_32x32x16_bf16 %1, %2, %2, %1\n\t"
          "v_mfma_f32_32x32x16_bf16 %0, %2, %2, %0\n\tv_mfma_f32_32x32x16_bf16 %1, %2, %2, %1\n\t"
          "v_mfma_f32_32x32x16_bf16 %0, %2, %2, %0\n\tv_mfma_f32_32x32x16_bf16 %1, %2, %2, %1\n\t"
          "v_mfma_f32_32x32x16_bf16 %0, %2, %2, %0\n\t"
          : "+v"(acc0), "+v"(acc1)
          : "v"(a));
    }
    if constexpr (KIND == 9)   // 16 v_exp_f32, VOP3 encoding with the packed-math-free form (e64)
      asm volatile(
          "v_exp_f32_e64 %0, %0\n\tv_exp_f32_e64 %1, %1\n\tv_exp_f32_e64 %2, %2\n\tv_exp_f32_e64 %3, %3\n\t"
          "v_exp_f32_e64 %4, %4\n\tv_exp_f32_e64 %5, %5\n\tv_exp_f32_e64 %6, %6\n\tv_exp_f32_e64 %7, %7\n\t"
          "v_exp_f32_e64 %0, %0\n\tv_exp_f32_e64 %1, %1\n\tv_exp_f32_e64 %2, %2\n\tv_exp_f32_e64 %3, %3\n\t"
          "v_exp_f32_e64 %4, %4\n\tv_exp_f32_e64 %5, %5\n\tv_exp_f32_e64 %6, %6\n\tv_exp_f32_e64 %7, %7"
          : R8);
    if constexpr (KIND == 10)   // 16 v_exp_f32 interleaved 1:1 with v_add_f32 (co-issue of trans + VALU?)
      asm volatile(
          "v_exp_f32 %0, %0\n\tv_add_f32 %8, %8, %9\n\tv_exp_f32 %1, %1\n\tv_add_f32 %9, %9, %8\n\t"
          "v_exp_f32 %2, %2\n\tv_add_f32 %8, %8, %9\n\tv_exp_f32 %3, %3\n\tv_add_f32 %9, %9, %8\n\t"
          "v_exp_f32 %4, %4\n\tv_add_f32 %8, %8, %9\n\tv_exp_f32 %5, %5\n\tv_add_f32 %9, %9, %8\n\t"
          "v_exp_f32 %6, %6\n\tv_add_f32 %8, %8, %9\n\tv_exp_f32 %7, %7\n\tv_add_f32 %9, %9, %8\n\t"
          "v_exp_f32 %0, %0\n\tv_add_f32 %8, %8, %9\n\tv_exp_f32 %1, %1\n\tv_add_f32 %9, %9, %8\n\t"
          "v_exp_f32 %2, %2\n\tv_add_f32 %8, %8, %9\n\tv_exp_f32 %3, %3\n\tv_add_f32 %9, %9, %8\n\t"
          "v_exp_f32 %4, %4\n\tv_add_f32 %8, %8, %9\n\tv_exp_f32 %5, %5\n\tv_add_f32 %9, %9, %8\n\t"
          "v_exp_f32 %6, %6\n\tv_add_f32 %8, %8, %9\n\tv_exp_f32 %7, %7\n\tv_add_f32 %9, %9, %8\n\t"
          : R8, "+v"(y0), "+v"(y1));
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7 + y0 + y1;
  for (int r = 0; r < 16; ++r) s += acc0[r] + acc1[r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND>
void run(const char* name, float* out, long long* cyc, long long* hcyc) {
  for (int wps : {1, 2}) {   // waves per SIMD: 256-thread blocks (one wave per SIMD each), wps per CU
    const int blocks = 256 * wps;
    hipLaunchKernelGGL(probe<KIND>, dim3(blocks), dim3(256), 0, 0, out, cyc);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(probe<KIND>, dim3(blocks), dim3(256), 0, 0, out, cyc);
    hipDeviceSynchronize();
    hipMemcpy(hcyc, cyc, blocks * sizeof(long long), hipMemcpyDeviceToHost);
    long long mx = 0;
    double sum = 0;
    for (int i = 0; i < blocks; ++i) {
      mx = hcyc[i] > mx ? hcyc[i] : mx;
      sum += hcyc[i];
    }
    printf("%-44s wps=%d  wave_cyc/block=%7.1f (max %7.1f)  simd_cyc/block=%7.1f\n", name, wps,
           sum / blocks / ITER, (double)mx / ITER, sum / blocks / ITER / wps);
  }
}

int main() {
  float* out;
  long long *cyc, *hcyc;
  hipMalloc(&out, 256 * 8 * 256 * sizeof(float));
  hipMalloc(&cyc, 256 * 8 * sizeof(long long));
  hcyc = (long long*)malloc(256 * 8 * sizeof(long long));
  run<0>("16 v_exp_f32", out, cyc, hcyc);
  run<9>("16 v_exp_f32_e64", out, cyc, hcyc);
  run<1>("16 v_exp_f16 sdwa (in-place halves)", out, cyc, hcyc);
  run<2>("16 v_exp_f16 e32", out, cyc, hcyc);
  run<3>("8 v_cvt_pk_bf16_f32", out, cyc, hcyc);
  run<4>("8 v_cvt_pk_f16_f32", out, cyc, hcyc);
  run<5>("8 v_cvt_pkrtz_f16_f32", out, cyc, hcyc);
  run<10>("16 v_exp_f32 + 16 v_add_f32 interleaved", out, cyc, hcyc);
  run<8>("7 mfma 32x32x16", out, cyc, hcyc);
  run<6>("A: 7 mfma + 16 exp_f32 + 8 cvt_pk_bf16", out, cyc, hcyc);
  run<7>("B: 7 mfma + 8 cvt_pk_f16 + 16 exp_f16 sdwa", out, cyc, hcyc);
  return 0;
}
