// MambaBlock as the reference runs it without mamba_ssm: the GLU gated-conv fallback
// (ultralytics/nn/modules/blocks_mamba.py:84-113 Conv1x1BN / GLUBlock, :198-236 MambaBlock.forward).
//
//   Y1 = SiLU(BN_i(W_i . x))                 [B, ch, H, W]     GEMM, BN + SiLU in the epilogue
//   P  = avg_pool_r(Y1)                       [B, ch, Hh, Wh]   Hh = H / r (floor), skipped for r = 1
//   Z  = W_pw1 . P                            [B, 4ch, Hh, Wh]  GEMM; rows [0, 2ch) = a, [2ch, 4ch) = g
//   D  = SiLU(BN(dw3x3(sigmoid(g) * a)))      [B, 2ch, Hh, Wh]  one kernel: GLU on the 18x18 halo tile in LDS
//   E  = W_pw2 . D                            [B, ch, Hh, Wh]   GEMM
//   F  = SiLU(BN_o(W_o . E))                  [B, C, Hh, Wh]    GEMM (out_proj before the upsample: nearest
//                                                               upsampling commutes with the pointwise 1x1 conv,
//                                                               BN and SiLU, so it runs on 1/r^2 of the pixels)
//   y  = x + up_nearest(F)                    [B, C, H, W]      (r = 1: the residual is fused into F's epilogue)
// The 1x1 convs are the library's exact-fp32 MFMA GEMM on NCHW operands (gemm_f32.h). BatchNorms are eval-form
// affines folded per channel on the device (the reference's fuse() leaves them unfused; the fold only changes
// rounding). Same op class as the MAFN operators: the three GEMMs dominate (57 GFLOP at P3 640^2 bs=32).
#include "common.h"
#include "gemm_f32.h"

namespace ys {

__global__ void mamba_fold_bn_kernel(const float* __restrict__ w, const float* __restrict__ b,
                                     const float* __restrict__ m, const float* __restrict__ v, float eps, int n,
                                     float* __restrict__ scale, float* __restrict__ shift) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float s = w[i] / sqrtf(v[i] + eps);
  scale[i] = s;
  shift[i] = b[i] - m[i] * s;
}

// F.avg_pool2d(kernel = stride = r, no padding): out[p][i][j] = sum_{di,dj} in[p][i*r+di][j*r+dj] / (r*r)
__global__ __launch_bounds__(256) void mamba_pool_kernel(const float* __restrict__ in, float* __restrict__ out, int H,
                                                         int W, int Hh, int Wh, int r) {
  const long plane = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= Hh * Wh) return;
  const int i = e / Wh, j = e - i * Wh;
  const float* src = in + plane * H * W + (long)(i * r) * W + j * r;
  float s = 0.f;
  for (int di = 0; di < r; ++di)
    for (int dj = 0; dj < r; ++dj) s += src[(long)di * W + dj];
  out[plane * Hh * Wh + e] = s / (float)(r * r);
}

// D[b][m] = SiLU(scale[m] * dw3x3(sigmoid(Z[b][hd+m]) * Z[b][m]) + shift[m]) on 16x16 output tiles; the GLU
// product is formed once per halo element in LDS (zero padding of the dw conv applies to the product).
// grid = (tiles_x, tiles_y, B * hd).
__global__ __launch_bounds__(256) void mamba_glu_dw_kernel(const float* __restrict__ Z, float* __restrict__ D, int hd,
                                                           int Hh, int Wh, const float* __restrict__ dw,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ shift) {
  __shared__ float t[18][19];
  const int plane = blockIdx.z;
  const int b = plane / hd, m = plane - b * hd;
  const long HWh = (long)Hh * Wh;
  const float* za = Z + ((long)b * 2 * hd + m) * HWh;
  const float* zg = za + (long)hd * HWh;
  const int oy = blockIdx.y * 16 - 1, ox = blockIdx.x * 16 - 1;
  for (int i = threadIdx.x; i < 18 * 18; i += 256) {
    const int ty = i / 18, tx = i - ty * 18;
    const int yy = oy + ty, xx = ox + tx;
    float v = 0.f;
    if (yy >= 0 && yy < Hh && xx >= 0 && xx < Wh) {
      const long o = (long)yy * Wh + xx;
      v = sigmoidf_(zg[o]) * za[o];
    }
    t[ty][tx] = v;
  }
  __syncthreads();
  const int ly = threadIdx.x >> 4, lx = threadIdx.x & 15;
  const int py = blockIdx.y * 16 + ly, px = blockIdx.x * 16 + lx;
  if (py >= Hh || px >= Wh) return;
  const float* k = dw + m * 9;
  const float v = k[0] * t[ly][lx] + k[1] * t[ly][lx + 1] + k[2] * t[ly][lx + 2] + k[3] * t[ly + 1][lx] +
                  k[4] * t[ly + 1][lx + 1] + k[5] * t[ly + 1][lx + 2] + k[6] * t[ly + 2][lx] +
                  k[7] * t[ly + 2][lx + 1] + k[8] * t[ly + 2][lx + 2];
  D[(long)plane * HWh + (long)py * Wh + px] = siluf_(v * scale[m] + shift[m]);
}

// y = x + F[nearest source pixel]; PyTorch's nearest rule for an explicit output size:
// src = min(floor(dst * (in / out)), in - 1) with a float scale. grid = (ceil(HW / 256), B * C).
__global__ __launch_bounds__(256) void mamba_up_res_kernel(const float* __restrict__ x, const float* __restrict__ F,
                                                           float* __restrict__ y, int H, int W, int Hh, int Wh) {
  const long plane = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= H * W) return;
  const int h = e / W, w = e - h * W;
  const float sh = (float)Hh / (float)H, sw = (float)Wh / (float)W;
  int ih = (int)floorf((float)h * sh), iw = (int)floorf((float)w * sw);
  ih = ih < Hh - 1 ? ih : Hh - 1;
  iw = iw < Wh - 1 ? iw : Wh - 1;
  const long o = plane * H * W + e;
  y[o] = x[o] + F[plane * Hh * Wh + (long)ih * Wh + iw];
}

struct MambaBufs {
  float *fold, *Y1, *P, *Z, *D, *E, *F;
};

template <class Alloc>
static void mamba_carve(Alloc& a, int B, int C, int H, int W, int ch, int r, MambaBufs* out) {
  const int Hh = H / r, Wh = W / r;
  const size_t HW = (size_t)H * W, HWh = (size_t)Hh * Wh;
  const int hd = 2 * ch;
  MambaBufs m{};
  m.fold = a.template take<float>(2 * ((size_t)ch + hd + C));
  m.Y1 = a.template take<float>((size_t)B * ch * HW);
  m.P = r > 1 ? a.template take<float>((size_t)B * ch * HWh) : m.Y1;
  m.Z = a.template take<float>((size_t)B * 2 * hd * HWh);
  m.D = a.template take<float>((size_t)B * hd * HWh);
  m.E = a.template take<float>((size_t)B * ch * HWh);
  m.F = r > 1 ? a.template take<float>((size_t)B * C * HWh) : nullptr;
  if (out) *out = m;
}

struct SizerAdapter {
  Sizer s;
  template <class T>
  T* take(size_t n) {
    s.take<T>(n);
    return reinterpret_cast<T*>(16);  // non-null marker; never dereferenced
  }
};

}  // namespace ys

using namespace ys;

YS_EXPORT size_t yolosod_mamba_glu_workspace(int B, int C, int H, int W, int ch, int reduction) {
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || ch <= 0 || reduction < 1) return 0;
  SizerAdapter a;
  mamba_carve(a, B, C, H, W, ch, reduction, nullptr);
  return a.s.off;
}

YS_EXPORT int yolosod_mamba_glu_forward(const float* x, float* y, int B, int C, int H, int W, int ch, int reduction,
                                        const float* in_w, const float* in_bn_w, const float* in_bn_b,
                                        const float* in_bn_mean, const float* in_bn_var, float in_bn_eps,
                                        const float* pw1_w, const float* dw_w, const float* bn_w, const float* bn_b,
                                        const float* bn_mean, const float* bn_var, float bn_eps, const float* pw2_w,
                                        const float* out_w, const float* out_bn_w, const float* out_bn_b,
                                        const float* out_bn_mean, const float* out_bn_var, float out_bn_eps,
                                        void* workspace, size_t workspace_bytes, void* stream) {
  YS_CHECK_ARG(x && y && in_w && in_bn_w && in_bn_b && in_bn_mean && in_bn_var && pw1_w && dw_w && bn_w && bn_b &&
                   bn_mean && bn_var && pw2_w && out_w && out_bn_w && out_bn_b && out_bn_mean && out_bn_var,
               "mamba: null pointer");
  YS_CHECK_ARG(B >= 0 && C > 0 && H > 0 && W > 0 && ch > 0 && reduction >= 1, "mamba: bad shape");
  YS_CHECK_ARG(H / reduction >= 1 && W / reduction >= 1, "mamba: seq_reduction %d too large for %dx%d", reduction, H,
               W);
  YS_CHECK_ARG(C % 32 == 0 && ch % 32 == 0, "mamba: C=%d and c_hidden=%d must be multiples of 32", C, ch);
  if (B == 0) return 0;
  const int r = reduction, hd = 2 * ch;
  const int Hh = H / r, Wh = W / r;
  const long HW = (long)H * W, HWh = (long)Hh * Wh;
  YS_CHECK_ARG((long)B * C < 65536 && (long)B * hd < 65536 && (long)B * ch < 65536, "mamba: too many planes");
  Carver cv(workspace, workspace_bytes);
  MambaBufs m{};
  mamba_carve(cv, B, C, H, W, ch, r, &m);
  YS_CHECK_ARG(m.fold && m.Y1 && m.P && m.Z && m.D && m.E && (r == 1 || m.F), "mamba: workspace too small (%zu)",
               workspace_bytes);
  hipStream_t st = (hipStream_t)stream;
  float* in_sc = m.fold;
  float* in_sh = in_sc + ch;
  float* mid_sc = in_sh + ch;
  float* mid_sh = mid_sc + hd;
  float* out_sc = mid_sh + hd;
  float* out_sh = out_sc + C;
  hipLaunchKernelGGL(mamba_fold_bn_kernel, dim3((ch + 255) / 256), dim3(256), 0, st, in_bn_w, in_bn_b, in_bn_mean,
                     in_bn_var, in_bn_eps, ch, in_sc, in_sh);
  hipLaunchKernelGGL(mamba_fold_bn_kernel, dim3((hd + 255) / 256), dim3(256), 0, st, bn_w, bn_b, bn_mean, bn_var,
                     bn_eps, hd, mid_sc, mid_sh);
  hipLaunchKernelGGL(mamba_fold_bn_kernel, dim3((C + 255) / 256), dim3(256), 0, st, out_bn_w, out_bn_b,
                     out_bn_mean, out_bn_var, out_bn_eps, C, out_sc, out_sh);
  YS_CHECK_LAUNCH("mamba_fold");
  int rc;
  // in_proj: Y1 = SiLU(BN_i(W_i . x)), M = ch, N = H*W, K = C, NCHW B operand, batched over images
  GemmArgs ga{};
  ga.A = in_w; ga.lda = C; ga.B = x; ga.b_bs = (long)C * HW; ga.ldb = (int)HW; ga.M = ch; ga.N = (int)HW; ga.K = C;
  ga.epi = epi_plain(m.Y1, (long)ch * HW, (int)HW);
  ga.epi.scale = in_sc; ga.epi.shift = in_sh; ga.epi.bn_mode = 1; ga.epi.act = 1;
  if ((rc = launch_gemm(ga, B, false, st))) return rc;
  if (r > 1) {
    hipLaunchKernelGGL(mamba_pool_kernel, dim3((unsigned)((HWh + 255) / 256), (unsigned)(B * ch)), dim3(256), 0, st,
                       m.Y1, m.P, H, W, Hh, Wh, r);
    YS_CHECK_LAUNCH("mamba_pool");
  }
  // GLUBlock.pw1: Z = W_pw1 . P, M = 2*hd
  ga = GemmArgs{};
  ga.A = pw1_w; ga.lda = ch; ga.B = m.P; ga.b_bs = (long)ch * HWh; ga.ldb = (int)HWh; ga.M = 2 * hd;
  ga.N = (int)HWh; ga.K = ch;
  ga.epi = epi_plain(m.Z, (long)2 * hd * HWh, (int)HWh);
  if ((rc = launch_gemm(ga, B, false, st))) return rc;
  hipLaunchKernelGGL(mamba_glu_dw_kernel, dim3((unsigned)((Wh + 15) / 16), (unsigned)((Hh + 15) / 16),
                     (unsigned)(B * hd)), dim3(256), 0, st, m.Z, m.D, hd, Hh, Wh, dw_w, mid_sc, mid_sh);
  YS_CHECK_LAUNCH("mamba_glu_dw");
  // GLUBlock.pw2: E = W_pw2 . D, M = ch, K = hd
  ga = GemmArgs{};
  ga.A = pw2_w; ga.lda = hd; ga.B = m.D; ga.b_bs = (long)hd * HWh; ga.ldb = (int)HWh; ga.M = ch; ga.N = (int)HWh;
  ga.K = hd;
  ga.epi = epi_plain(m.E, (long)ch * HWh, (int)HWh);
  if ((rc = launch_gemm(ga, B, false, st))) return rc;
  // out_proj on the reduced grid: F = SiLU(BN_o(W_o . E)); r = 1: + x straight into y
  ga = GemmArgs{};
  ga.A = out_w; ga.lda = ch; ga.B = m.E; ga.b_bs = (long)ch * HWh; ga.ldb = (int)HWh; ga.M = C; ga.N = (int)HWh;
  ga.K = ch;
  ga.epi = epi_plain(r > 1 ? m.F : y, (long)C * HWh, (int)HWh);
  ga.epi.scale = out_sc; ga.epi.shift = out_sh; ga.epi.bn_mode = 1; ga.epi.act = 1;
  if (r == 1) {
    ga.epi.res = x; ga.epi.res_bs = (long)C * HW; ga.epi.ldr = (int)HW;
  }
  if ((rc = launch_gemm(ga, B, false, st))) return rc;
  if (r > 1) {
    hipLaunchKernelGGL(mamba_up_res_kernel, dim3((unsigned)((HW + 255) / 256), (unsigned)(B * C)), dim3(256), 0, st,
                       x, m.F, y, H, W, Hh, Wh);
    YS_CHECK_LAUNCH("mamba_up_res");
  }
  return 0;
}
