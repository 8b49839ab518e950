// Issue cost of VALU instruction forms on gfx950 (diagnostic, not shipped): N independent chains of one instruction,
// cycles per instruction per wave from s_memtime, at 1 and 2 waves per SIMD. Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#define REP 64
#define ITER 256
typedef float f2 __attribute__((ext_vector_type(2)));
template <int OP>
__global__ void k(float* out, unsigned long long* cyc, float s) {
  float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7};
  unsigned u0 = threadIdx.x, u1 = u0 + 1, u2 = u0 + 2, u3 = u0 + 3;
  const float b = s, c = s * 0.5f;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int r = 0; r < REP / 8; ++r) {
      if (OP == 0) {  // v_fma_f32 x8
        asm volatile("v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_fma_f32 %2, %2, %8, %9\n v_fma_f32 %3, %3, %8, %9\n"
                     "v_fma_f32 %4, %4, %8, %9\n v_fma_f32 %5, %5, %8, %9\n v_fma_f32 %6, %6, %8, %9\n v_fma_f32 %7, %7, %8, %9"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));
      } else if (OP == 1) {  // v_pk_fma_f32 x8 (4 regs pairs, 2 rounds)
        asm volatile("v_pk_fma_f32 %0, %0, %4, %5\n v_pk_fma_f32 %1, %1, %4, %5\n v_pk_fma_f32 %2, %2, %4, %5\n v_pk_fma_f32 %3, %3, %4, %5\n"
                     "v_pk_fma_f32 %0, %0, %4, %5\n v_pk_fma_f32 %1, %1, %4, %5\n v_pk_fma_f32 %2, %2, %4, %5\n v_pk_fma_f32 %3, %3, %4, %5"
                     : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(f2{b, b}), "v"(f2{c, c}));
      } else if (OP == 2) {  // v_fma_mixlo_f16 x8 (f32 inputs, f16 result to the low half)
        asm volatile("v_fma_mixlo_f16 %0, %4, %5, %0 op_sel_hi:[0,0,1]\n v_fma_mixlo_f16 %1, %4, %5, %1 op_sel_hi:[0,0,1]\n"
                     "v_fma_mixlo_f16 %2, %4, %5, %2 op_sel_hi:[0,0,1]\n v_fma_mixlo_f16 %3, %4, %5, %3 op_sel_hi:[0,0,1]\n"
                     "v_fma_mixlo_f16 %0, %4, %5, %0 op_sel_hi:[0,0,1]\n v_fma_mixlo_f16 %1, %4, %5, %1 op_sel_hi:[0,0,1]\n"
                     "v_fma_mixlo_f16 %2, %4, %5, %2 op_sel_hi:[0,0,1]\n v_fma_mixlo_f16 %3, %4, %5, %3 op_sel_hi:[0,0,1]"
                     : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(b), "v"(c));
      } else if (OP == 3) {  // v_cvt_pk_f16_f32 x8
        asm volatile("v_cvt_pk_f16_f32 %0, %4, %5\n v_cvt_pk_f16_f32 %1, %4, %5\n v_cvt_pk_f16_f32 %2, %4, %5\n v_cvt_pk_f16_f32 %3, %4, %5\n"
                     "v_cvt_pk_f16_f32 %0, %4, %5\n v_cvt_pk_f16_f32 %1, %4, %5\n v_cvt_pk_f16_f32 %2, %4, %5\n v_cvt_pk_f16_f32 %3, %4, %5"
                     : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : "v"(a0), "v"(a1));
      } else if (OP == 4) {  // v_cvt_f32_f16 x8
        asm volatile("v_cvt_f32_f16 %0, %4\n v_cvt_f32_f16 %1, %4\n v_cvt_f32_f16 %2, %4\n v_cvt_f32_f16 %3, %4\n"
                     "v_cvt_f32_f16 %0, %5\n v_cvt_f32_f16 %1, %5\n v_cvt_f32_f16 %2, %5\n v_cvt_f32_f16 %3, %5"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(u0), "v"(u1));
      } else if (OP == 5) {  // v_pk_mul_f32 x8
        asm volatile("v_pk_mul_f32 %0, %0, %4\n v_pk_mul_f32 %1, %1, %4\n v_pk_mul_f32 %2, %2, %4\n v_pk_mul_f32 %3, %3, %4\n"
                     "v_pk_mul_f32 %0, %0, %4\n v_pk_mul_f32 %1, %1, %4\n v_pk_mul_f32 %2, %2, %4\n v_pk_mul_f32 %3, %3, %4"
                     : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(f2{b, b}));
      } else if (OP == 6) {  // v_exp_f32 x8
        asm volatile("v_exp_f32 %0, %0\n v_exp_f32 %1, %1\n v_exp_f32 %2, %2\n v_exp_f32 %3, %3\n"
                     "v_exp_f32 %4, %4\n v_exp_f32 %5, %5\n v_exp_f32 %6, %6\n v_exp_f32 %7, %7"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
      } else if (OP == 7) {  // v_mov_b32 x8
        asm volatile("v_mov_b32 %0, %8\n v_mov_b32 %1, %8\n v_mov_b32 %2, %8\n v_mov_b32 %3, %8\n"
                     "v_mov_b32 %4, %9\n v_mov_b32 %5, %9\n v_mov_b32 %6, %9\n v_mov_b32 %7, %9"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));
      } else if (OP == 8) {  // v_maximum3_f32 x8
        asm volatile("v_maximum3_f32 %0, %0, %8, %9\n v_maximum3_f32 %1, %1, %8, %9\n v_maximum3_f32 %2, %2, %8, %9\n v_maximum3_f32 %3, %3, %8, %9\n"
                     "v_maximum3_f32 %4, %4, %8, %9\n v_maximum3_f32 %5, %5, %8, %9\n v_maximum3_f32 %6, %6, %8, %9\n v_maximum3_f32 %7, %7, %8, %9"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));
      } else if (OP == 9) {  // v_permlane16_swap_b32 x8
        asm volatile("v_permlane16_swap_b32 %0, %1\n v_permlane16_swap_b32 %2, %3\n v_permlane16_swap_b32 %4, %5\n v_permlane16_swap_b32 %6, %7\n"
                     "v_permlane16_swap_b32 %0, %1\n v_permlane16_swap_b32 %2, %3\n v_permlane16_swap_b32 %4, %5\n v_permlane16_swap_b32 %6, %7"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
      } else if (OP == 10) {  // v_add_f32 x8
        asm volatile("v_add_f32 %0, %0, %8\n v_add_f32 %1, %1, %8\n v_add_f32 %2, %2, %8\n v_add_f32 %3, %3, %8\n"
                     "v_add_f32 %4, %4, %9\n v_add_f32 %5, %5, %9\n v_add_f32 %6, %6, %9\n v_add_f32 %7, %7, %9"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));
      } else if (OP == 11) {  // v_rcp_f32 x8
        asm volatile("v_rcp_f32 %0, %0\n v_rcp_f32 %1, %1\n v_rcp_f32 %2, %2\n v_rcp_f32 %3, %3\n"
                     "v_rcp_f32 %4, %4\n v_rcp_f32 %5, %5\n v_rcp_f32 %6, %6\n v_rcp_f32 %7, %7"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
      } else if (OP == 12) {  // v_pk_add_f32 x8
        asm volatile("v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4\n"
                     "v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4"
                     : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(f2{b, b}));
      } else if (OP == 13) {  // v_bfi_b32 x8
        asm volatile("v_bfi_b32 %0, %8, %0, %9\n v_bfi_b32 %1, %8, %1, %9\n v_bfi_b32 %2, %8, %2, %9\n v_bfi_b32 %3, %8, %3, %9\n"
                     "v_bfi_b32 %4, %8, %4, %9\n v_bfi_b32 %5, %8, %5, %9\n v_bfi_b32 %6, %8, %6, %9\n v_bfi_b32 %7, %8, %7, %9"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));
      }
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + p0.x + p1.y + p2.x + p3.y +
                                               (float)(u0 + u1 + u2 + u3);
  if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}
static const char* NAMES[] = {"v_fma_f32", "v_pk_fma_f32", "v_fma_mixlo_f16", "v_cvt_pk_f16_f32", "v_cvt_f32_f16",
                              "v_pk_mul_f32", "v_exp_f32", "v_mov_b32", "v_maximum3_f32", "v_permlane16_swap",
                              "v_add_f32", "v_rcp_f32", "v_pk_add_f32", "v_bfi_b32"};
template <int OP>
void run(int threads, float* out, unsigned long long* cyc, unsigned long long* h) {
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k<OP>, dim3(256), dim3(threads), 0, 0, out, cyc, 1.0001f);
  hipDeviceSynchronize();
  const int nw = 256 * threads / 64;
  hipMemcpy(h, cyc, nw * 8, hipMemcpyDeviceToHost);
  double s = 0; for (int i = 0; i < nw; ++i) s += h[i];
  printf("%-20s waves/SIMD %d: %.2f cycles per instruction per wave\n", NAMES[OP], threads / 256, s / nw / (ITER * REP));
}
template <int OP>
void both(float* out, unsigned long long* cyc, unsigned long long* h) { run<OP>(256, out, cyc, h); run<OP>(512, out, cyc, h); run<OP>(1024, out, cyc, h); }
int main() {
  float* out; unsigned long long* cyc; hipMalloc(&out, 256 * 1024 * 4); hipMalloc(&cyc, 256 * 16 * 8);
  static unsigned long long h[256 * 16];
  both<0>(out, cyc, h); both<10>(out, cyc, h); both<1>(out, cyc, h); both<5>(out, cyc, h); both<12>(out, cyc, h);
  both<2>(out, cyc, h); both<3>(out, cyc, h); both<4>(out, cyc, h); both<6>(out, cyc, h); both<11>(out, cyc, h);
  both<7>(out, cyc, h); both<8>(out, cyc, h); both<9>(out, cyc, h); both<13>(out, cyc, h);
  return 0;
}
