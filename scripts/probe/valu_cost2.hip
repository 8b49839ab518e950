// Issue cost of candidate split instructions and of MFMA on gfx950 (diagnostic, not shipped); see valu_cost.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#define REP 64
#define ITER 256
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
template <int OP>
__global__ void k(float* out, unsigned long long* cyc, float s) {
  float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  unsigned u0 = threadIdx.x * 0x3c003c01u, u1 = u0 + 1;
  h8 x = {(_Float16)s, (_Float16)1, 0, 0, 0, 0, 0, 0};
  f4 c0 = {a0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int r = 0; r < REP / 8; ++r) {
      if (OP == 0) {  // v_dot2_f32_f16 x8
        asm volatile("v_dot2_f32_f16 %0, %8, %9, %0\n v_dot2_f32_f16 %1, %8, %9, %1\n v_dot2_f32_f16 %2, %8, %9, %2\n v_dot2_f32_f16 %3, %8, %9, %3\n"
                     "v_dot2_f32_f16 %4, %8, %9, %4\n v_dot2_f32_f16 %5, %8, %9, %5\n v_dot2_f32_f16 %6, %8, %9, %6\n v_dot2_f32_f16 %7, %8, %9, %7"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(u0), "v"(u1));
      } else if (OP == 1) {  // v_dot2c_f32_f16 x8 (VOP2)
        asm volatile("v_dot2c_f32_f16 %0, %8, %9\n v_dot2c_f32_f16 %1, %8, %9\n v_dot2c_f32_f16 %2, %8, %9\n v_dot2c_f32_f16 %3, %8, %9\n"
                     "v_dot2c_f32_f16 %4, %8, %9\n v_dot2c_f32_f16 %5, %8, %9\n v_dot2c_f32_f16 %6, %8, %9\n v_dot2c_f32_f16 %7, %8, %9"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(u0), "v"(u1));
      } else if (OP == 2) {  // v_mfma_f32_16x16x32_f16 x8, 4 independent accumulators
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, x, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, x, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, x, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, x, c3, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, x, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, x, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, x, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, x, c3, 0, 0, 0);
      } else if (OP == 3) {  // 8 MFMA + 16 v_pk_fma_f32 interleaved (2 per MFMA)
        typedef float f2 __attribute__((ext_vector_type(2)));
        f2 p = {a0, a1}, q = {a2, a3};
#define MP(c) c = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, x, c, 0, 0, 0); \
        asm volatile("v_pk_fma_f32 %0, %0, %2, %2\n v_pk_fma_f32 %1, %1, %2, %2" : "+v"(p), "+v"(q) : "v"(f2{s, s}));
        MP(c0) MP(c1) MP(c2) MP(c3) MP(c0) MP(c1) MP(c2) MP(c3)
        a0 = p.x; a1 = p.y; a2 = q.x; a3 = q.y;
      } else if (OP == 4) {  // 8 MFMA + 8 v_exp_f32 interleaved (1 per MFMA)
#define ME(c, a) c = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, x, c, 0, 0, 0); asm volatile("v_exp_f32 %0, %0" : "+v"(a));
        ME(c0, a0) ME(c1, a1) ME(c2, a2) ME(c3, a3) ME(c0, a4) ME(c1, a5) ME(c2, a6) ME(c3, a7)
      } else if (OP == 5) {  // 8 MFMA + 32 v_pk_fma_f32 interleaved (4 per MFMA)
        typedef float f2 __attribute__((ext_vector_type(2)));
        f2 p = {a0, a1}, q = {a2, a3}, p2 = {a4, a5}, q2 = {a6, a7};
#define MQ(c) c = __builtin_amdgcn_mfma_f32_16x16x32_f16(x, x, c, 0, 0, 0); \
        asm volatile("v_pk_fma_f32 %0, %0, %4, %4\n v_pk_fma_f32 %1, %1, %4, %4\n v_pk_fma_f32 %2, %2, %4, %4\n v_pk_fma_f32 %3, %3, %4, %4" : "+v"(p), "+v"(q), "+v"(p2), "+v"(q2) : "v"(f2{s, s}));
        MQ(c0) MQ(c1) MQ(c2) MQ(c3) MQ(c0) MQ(c1) MQ(c2) MQ(c3)
        a0 = p.x; a1 = p.y; a2 = q.x; a3 = q.y; a4 = p2.x; a5 = p2.y; a6 = q2.x; a7 = q2.y;
      }
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + c0[0] + c1[1] + c2[2] + c3[3];
  if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}
static const char* NAMES[] = {"v_dot2_f32_f16", "v_dot2c_f32_f16", "mfma16x16x32_f16", "mfma+2pk_fma", "mfma+1exp",
                              "mfma+4pk_fma"};
template <int OP>
void run(int threads, float* out, unsigned long long* cyc, unsigned long long* h) {
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k<OP>, dim3(256), dim3(threads), 0, 0, out, cyc, 1.0001f);
  hipDeviceSynchronize();
  const int nw = 256 * threads / 64;
  hipMemcpy(h, cyc, nw * 8, hipMemcpyDeviceToHost);
  double s = 0; for (int i = 0; i < nw; ++i) s += h[i];
  printf("%-20s waves/SIMD %d: %.2f cycles per (MFMA or VALU) step per wave\n", NAMES[OP], threads / 256, s / nw / (ITER * REP));
}
template <int OP>
void both(float* out, unsigned long long* cyc, unsigned long long* h) { run<OP>(256, out, cyc, h); run<OP>(512, out, cyc, h); run<OP>(1024, out, cyc, h); }
int main() {
  float* out; unsigned long long* cyc; hipMalloc(&out, 256 * 1024 * 4); hipMalloc(&cyc, 256 * 16 * 8);
  static unsigned long long h[256 * 16];
  both<0>(out, cyc, h); both<1>(out, cyc, h); both<2>(out, cyc, h); both<3>(out, cyc, h); both<4>(out, cyc, h);
  both<5>(out, cyc, h);
  return 0;
}
