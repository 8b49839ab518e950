// Transformer-shaped MAFN operators on gfx950: SwinBlock (window attention at P4/P2) and A2_Attn (area attention
// at P5), built from four device primitives:
//   * gemm_f32      - LDS-tiled GEMM on the exact-fp32 matrix cores (v_mfma_f32_32x32x2_f32), 128xBN x16 tiles,
//                     4 waves, fused epilogues (bias / folded-BN / SiLU / GELU / residual / Swin window-reverse).
//   * attn_f32      - per-(sequence, head, 64-query block) attention on v_mfma_f32_16x16x4_f32: Q in registers,
//                     K and V staged through LDS in 64-key chunks, scores for the whole (<=320-key) row kept in
//                     registers, softmax via 16-lane shuffles, P transposed through LDS for the P.V product.
//   * layernorm     - one wave per token row.
//   * swin_partition (depthwise 3x3 + zero pad + window partition, token-major out) / a2 pool + upsample.
// Numerics: fp32 in / fp32 accumulate everywhere (the MFMA f32 form is an exact f32 fma chain), matching the
// reference's fp32 PyTorch-CPU math to rounding.
//
// Reference semantics:
//   SwinBlock  ultralytics/nn/modules/blocks_transformer.py:8-171 (window_partition :8-47, window_reverse :49-79,
//              WindowAttention.forward :100-131, SwinBlock.forward :150-171)
//   A2_Attn    ultralytics/nn/modules/a2_attn.py:35-69
#include "common.h"
#include "gemm_f32.h"
#include <math.h>
#include <stdlib.h>

namespace ys {

// =================================================================================================
// LayerNorm over rows of C (token-major), one wave per row. y = (x-mean)*rstd*w + b, biased variance.
// =================================================================================================
template <int VPL>  // values per lane, C <= 64*VPL
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, float* __restrict__ y, long rows,
                                                        int C, const float* __restrict__ w,
                                                        const float* __restrict__ b, float eps) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* xr = x + row * C;
  float v[VPL];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + 64 * i;
    v[i] = (c < C) ? xr[c] : 0.f;
    s += v[i];
  }
  const float mean = wave_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + 64 * i;
    const float d = (c < C) ? v[i] - mean : 0.f;
    q += d * d;
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)C + eps);
  float* yr = y + row * C;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + 64 * i;
    if (c < C) yr[c] = (v[i] - mean) * rstd * w[c] + b[c];
  }
}

static int launch_layernorm(const float* x, float* y, long rows, int C, const float* w, const float* b, float eps,
                            hipStream_t st) {
  YS_CHECK_ARG(C > 0 && C <= 1024, "layernorm: C=%d unsupported", C);
  if (rows == 0) return 0;
  dim3 grid((unsigned)((rows + 3) / 4));
  if (C <= 64) hipLaunchKernelGGL((layernorm_kernel<1>), grid, dim3(256), 0, st, x, y, rows, C, w, b, eps);
  else if (C <= 128) hipLaunchKernelGGL((layernorm_kernel<2>), grid, dim3(256), 0, st, x, y, rows, C, w, b, eps);
  else if (C <= 256) hipLaunchKernelGGL((layernorm_kernel<4>), grid, dim3(256), 0, st, x, y, rows, C, w, b, eps);
  else if (C <= 512) hipLaunchKernelGGL((layernorm_kernel<8>), grid, dim3(256), 0, st, x, y, rows, C, w, b, eps);
  else hipLaunchKernelGGL((layernorm_kernel<16>), grid, dim3(256), 0, st, x, y, rows, C, w, b, eps);
  YS_CHECK_LAUNCH("layernorm");
  return 0;
}

// =================================================================================================
// Attention over packed QKV rows: qkv[(s*L + t)*ld + {0,C,2C} + h*hd + d]; out[(s*L + t)*ldo + h*hd + d].
// grid = (ceil(L/64), heads, n_seq). Each wave owns 16 query rows; the full score row (NKB*16 keys) lives in
// registers (NKB f32x4 accumulators), so softmax needs no rescaling.
// =================================================================================================
template <int HD, int NKB>
__global__ __launch_bounds__(256) void attn_f32_kernel(const float* __restrict__ qkv, int ld, int C,
                                                       float* __restrict__ out, int ldo, int L, float scale) {
  constexpr int HDP = HD < 16 ? 16 : HD;  // padded head dim for the P.V output blocks
  constexpr int KS = HDP + 1;             // LDS row stride of the K / V chunk
  constexpr int NK = NKB * 16;            // keys covered
  constexpr int PS = NK + 1;              // LDS row stride of P
  __shared__ float KV[64 * KS];
  __shared__ float Ps[4 * 16 * PS];

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int h = blockIdx.y;
  const long seq_row0 = (long)blockIdx.z * L;
  const int q0 = blockIdx.x * 64 + wv * 16;
  const int l15 = lane & 15, l4 = lane >> 4;

  // Q fragment: A[i = l&15][k = l>>4] over k-steps of 4 (scaled once, as q*scale in the MHA math path)
  // Loads without per-lane predicates where the shape allows (HD % 4 == 0): rows past L read row L - 1 (queries past
  // L are not stored; keys past L are masked before the softmax and meet P = 0 in P.V). A predicated load merged into
  // a phi whose copy waited for it: every Q / K / V load of the kernel was its own round trip.
  constexpr bool VEC = HD % 4 == 0 && HDP == HD;
  float qf[(HD + 3) / 4];
  {
    const int qrow = q0 + l15;
#pragma unroll
    for (int s = 0; s < (HD + 3) / 4; ++s) {
      const int d = 4 * s + l4;
      if (VEC)
        qf[s] = qkv[(seq_row0 + (qrow < L ? qrow : L - 1)) * ld + h * HD + d] * scale;
      else
        qf[s] = (qrow < L && d < HD) ? qkv[(seq_row0 + qrow) * ld + h * HD + d] * scale : 0.f;
    }
  }
  // a 64-key chunk of K (off = C) or V (off = 2C) into KV, all of a thread's loads issued before its LDS stores
  auto stage = [&](int ch, int off) {
    if constexpr (VEC) {
      constexpr int NE = 64 * HD / 256;
      float v[NE];
#pragma unroll
      for (int i = 0; i < NE; ++i) {
        const int e = tid + 256 * i, kr = e / HD, d = e % HD;
        const int key = ch * 64 + kr;
        v[i] = qkv[(seq_row0 + (key < L ? key : L - 1)) * ld + off + h * HD + d];
      }
#pragma unroll
      for (int i = 0; i < NE; ++i) {
        const int e = tid + 256 * i;
        KV[(e / HD) * KS + e % HD] = v[i];
      }
    } else {
      for (int e = tid; e < 64 * HDP; e += 256) {
        const int kr = e / HDP, d = e % HDP;
        const int key = ch * 64 + kr;
        KV[kr * KS + d] = (key < L && d < HD) ? qkv[(seq_row0 + key) * ld + off + h * HD + d] : 0.f;
      }
    }
  };

  f32x4 sacc[NKB];
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) sacc[kb] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- S = Q K^T, K staged in 64-key chunks ----
#pragma unroll
  for (int ch = 0; ch < (NKB + 3) / 4; ++ch) {
    __syncthreads();
    stage(ch, C);
    __syncthreads();
#pragma unroll
    for (int kb4 = 0; kb4 < 4; ++kb4) {
      const int kb = ch * 4 + kb4;
      if (kb < NKB) {
#pragma unroll
        for (int s = 0; s < (HD + 3) / 4; ++s) {
          const int d = 4 * s + l4;
          const float bk = (d < HD) ? KV[(kb4 * 16 + l15) * KS + d] : 0.f;
          sacc[kb] = __builtin_amdgcn_mfma_f32_16x16x4f32(qf[s], bk, sacc[kb], 0, 0, 0);
        }
      }
    }
  }

  // ---- softmax over keys; lane holds S[row = l4*4 + r][key = kb*16 + l15] ----
  float rmax[4], rsum[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) rmax[r] = -INFINITY;
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) {
    const bool valid = (kb * 16 + l15) < L;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (!valid) sacc[kb][r] = -INFINITY;
      rmax[r] = fmaxf(rmax[r], sacc[kb][r]);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) rmax[r] = fmaxf(rmax[r], __shfl_xor(rmax[r], o, 64));
    rsum[r] = 0.f;
  }
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float e = expf(sacc[kb][r] - rmax[r]);
      sacc[kb][r] = e;
      rsum[r] += e;
    }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) rsum[r] += __shfl_xor(rsum[r], o, 64);
    rsum[r] = 1.0f / rsum[r];
  }
  float* Pw = Ps + wv * 16 * PS;
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
    for (int r = 0; r < 4; ++r) Pw[(l4 * 4 + r) * PS + kb * 16 + l15] = sacc[kb][r] * rsum[r];

  // ---- O = P V, V staged in 64-key chunks ----
  f32x4 oacc[HDP / 16];
#pragma unroll
  for (int nb = 0; nb < HDP / 16; ++nb) oacc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ch = 0; ch < (NKB + 3) / 4; ++ch) {
    __syncthreads();
    stage(ch, 2 * C);
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int key = ch * 64 + 4 * s + l4;  // k index of this k-step for this lane
      if (ch * 64 + 4 * s < NK) {
        const float pa = Pw[l15 * PS + key];
#pragma unroll
        for (int nb = 0; nb < HDP / 16; ++nb) {
          const float vb = KV[(4 * s + l4) * KS + nb * 16 + l15];
          oacc[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(pa, vb, oacc[nb], 0, 0, 0);
        }
      }
    }
  }
#pragma unroll
  for (int nb = 0; nb < HDP / 16; ++nb) {
    const int d = nb * 16 + l15;
    if (d >= HD) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int qrow = q0 + l4 * 4 + r;
      if (qrow < L) out[(seq_row0 + qrow) * ldo + h * HD + d] = oacc[nb][r];
    }
  }
}

// Whole-sequence attention for head dim 64, L <= 256 (A2: L = 8 areas x W = 160 at 640^2): one workgroup per
// (sequence, head) with one wave per 16 queries, K and V of the head staged once in LDS (rows of 68 floats:
// conflict-free 16-B reads). S^T = K Q^T is accumulated per 16-key block so that the accumulator registers are
// directly the B operand of O^T = V^T P^T (keys permuted consistently): P never leaves registers. Q is scaled
// before the product (q * scaling, the MHA math path of a2_attn.py:53). grid = (heads, n_seq), 64 * ceil(L/16)
// threads.
template <int NKB>
__global__ __launch_bounds__(1024) void attn_seq64_kernel(const float* __restrict__ qkv, int ld, int C,
                                                          float* __restrict__ out, int ldo, int L, float scale) {
  constexpr int HD = 64, LK = HD + 4;
  extern __shared__ __attribute__((aligned(16))) float kv[];  // K [NKB*16][LK] | V [NKB*16][LK]
  float* Ks = kv;
  float* Vs = kv + NKB * 16 * LK;
  const int h = blockIdx.x;
  const long row0 = (long)blockIdx.y * L;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int l15 = lane & 15, g = lane >> 4;
  // stage K and V (float4 rows; keys >= L zero)
  for (int e = tid; e < NKB * 16 * (HD / 4); e += blockDim.x) {
    const int key = e / (HD / 4), q4 = e - key * (HD / 4);
    float4 k = make_float4(0.f, 0.f, 0.f, 0.f), v = k;
    if (key < L) {
      const float* src = qkv + (row0 + key) * ld + h * HD + 4 * q4;
      k = *reinterpret_cast<const float4*>(src + C);
      v = *reinterpret_cast<const float4*>(src + 2 * C);
    }
    *reinterpret_cast<float4*>(Ks + key * LK + 4 * q4) = k;
    *reinterpret_cast<float4*>(Vs + key * LK + 4 * q4) = v;
  }
  // this wave's 16 queries: lane (g, l15) holds Q[q0 + l15][16g .. 16g+16) * scale (MFMA k permuted by 16g)
  const int q = wv * 16 + l15;
  float4 qf[4];
  {
    const int qr = q < L ? q : L - 1;
    const float* src = qkv + (row0 + qr) * ld + h * HD + 16 * g;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float4 v = *reinterpret_cast<const float4*>(src + 4 * t);
      v.x *= scale; v.y *= scale; v.z *= scale; v.w *= scale;
      qf[t] = v;
    }
  }
  __syncthreads();
  f32x4 st[NKB];
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) {
    f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
    const float* kr = Ks + (kb * 16 + l15) * LK + 16 * g;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float4 k = *reinterpret_cast<const float4*>(kr + 4 * t);
      a = __builtin_amdgcn_mfma_f32_16x16x4f32(k.x, qf[t].x, a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_16x16x4f32(k.y, qf[t].y, a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_16x16x4f32(k.z, qf[t].z, a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_16x16x4f32(k.w, qf[t].w, a, 0, 0, 0);
    }
    st[kb] = a;
  }
  // lane holds S^T[key = kb*16 + 4g + r][query l15]: softmax over keys (in-lane, then the 4 lane groups)
  float mx = -INFINITY;
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (kb * 16 + 4 * g + r >= L) st[kb][r] = -INFINITY;
      mx = fmaxf(mx, st[kb][r]);
    }
  mx = xor32_max(xor16_max(mx));
  float sum = 0.f;
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float e = expf(st[kb][r] - mx);
      st[kb][r] = e;
      sum += e;
    }
  sum = xor32_sum(xor16_sum(sum));
  const float inv = 1.0f / sum;
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
    for (int r = 0; r < 4; ++r) st[kb][r] *= inv;
  // O^T[d][q] = sum_key V[key][d] P[q][key]
  f32x4 o[HD / 16];
#pragma unroll
  for (int db = 0; db < HD / 16; ++db) o[db] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float* vr = Vs + (kb * 16 + 4 * g + r) * LK + l15;
#pragma unroll
      for (int db = 0; db < HD / 16; ++db)
        o[db] = __builtin_amdgcn_mfma_f32_16x16x4f32(vr[db * 16], st[kb][r], o[db], 0, 0, 0);
    }
  if (q < L) {
    float* dst = out + (row0 + q) * ldo + h * HD + 4 * g;
#pragma unroll
    for (int db = 0; db < HD / 16; ++db) *reinterpret_cast<f32x4*>(dst + db * 16) = o[db];
  }
}

template <int HD>
static void launch_attn_hd(int nkb, dim3 grid, hipStream_t st, const float* qkv, int ld, int C, float* out, int ldo,
                           int L, float scale) {
#define YS_ATTN_CASE(NKBV)                                                                                   \
  if (nkb <= NKBV) {                                                                                         \
    hipLaunchKernelGGL((attn_f32_kernel<HD, NKBV>), grid, dim3(256), 0, st, qkv, ld, C, out, ldo, L, scale); \
    return;                                                                                                  \
  }
  YS_ATTN_CASE(4)
  YS_ATTN_CASE(8)
  YS_ATTN_CASE(10)
  YS_ATTN_CASE(12)
  YS_ATTN_CASE(16)
  YS_ATTN_CASE(20)
#undef YS_ATTN_CASE
}

static int launch_attention(const float* qkv, float* out, long n_seq, int L, int C, int heads, hipStream_t st) {
  YS_CHECK_ARG(heads > 0 && C % heads == 0, "attention: C=%d not divisible by heads=%d", C, heads);
  const int hd = C / heads;
  YS_CHECK_ARG(L > 0 && L <= 320, "attention: sequence length %d unsupported (1..320)", L);
  YS_CHECK_ARG(n_seq < 65536, "attention: too many sequences (%ld)", n_seq);
  const int nkb = (L + 15) / 16;
  const float scale = 1.0f / sqrtf((float)hd);
  if (hd == 64 && nkb <= 16 && (3 * C) % 4 == 0 && C % 4 == 0) {  // whole-sequence kernel (A2 at 640^2: L = 160)
    dim3 g2((unsigned)heads, (unsigned)n_seq);
#define YS_ATTN_SEQ(N)                                                                                       \
    if (nkb <= N) {                                                                                            \
      const size_t lds = (size_t)2 * N * 16 * 68 * sizeof(float); /* K | V for N key blocks */                \
      hipLaunchKernelGGL((attn_seq64_kernel<N>), g2, dim3(64 * nkb), lds, st, qkv, 3 * C, C, out, C, L, scale); \
      YS_CHECK_LAUNCH("attention_seq");                                                                       \
      return 0;                                                                                                \
    }
    YS_ATTN_SEQ(4) YS_ATTN_SEQ(8) YS_ATTN_SEQ(10) YS_ATTN_SEQ(12) YS_ATTN_SEQ(16)
#undef YS_ATTN_SEQ
  }
  dim3 grid((L + 63) / 64, heads, (unsigned)n_seq);
  switch (hd) {
    case 8: launch_attn_hd<8>(nkb, grid, st, qkv, 3 * C, C, out, C, L, scale); break;
    case 16: launch_attn_hd<16>(nkb, grid, st, qkv, 3 * C, C, out, C, L, scale); break;
    case 32: launch_attn_hd<32>(nkb, grid, st, qkv, 3 * C, C, out, C, L, scale); break;
    case 64: launch_attn_hd<64>(nkb, grid, st, qkv, 3 * C, C, out, C, L, scale); break;
    case 128: launch_attn_hd<128>(nkb, grid, st, qkv, 3 * C, C, out, C, L, scale); break;
    default: YS_CHECK_ARG(false, "attention: head dim %d unsupported (8,16,32,64,128)", hd);
  }
  YS_CHECK_LAUNCH("attention");
  return 0;
}

// =================================================================================================
// Swin: depthwise 3x3 (pad 1, no bias) + bottom/right zero pad + window partition -> token-major T[tok][C].
// Token order (img, wy, wx, iy, ix) as window_partition's permute(0,2,4,3,5,1) (blocks_transformer.py:43-46).
// grid = (8*ceil(nWin_total/8), ceil(C/64)), windows dealt to XCDs in contiguous ranges (neighbouring windows
// share cache lines of x); a 64-channel slab of the (wh+2)x(ww+2) halo patch is staged in LDS.
// =================================================================================================
__global__ __launch_bounds__(256) void swin_partition_kernel(const float* __restrict__ x, const float* __restrict__ dw,
                                                             float* __restrict__ T, int C, int H, int W, int wh,
                                                             int ww, int nWx, int nWin, long nwin_total) {
  extern __shared__ float patch[];  // [64][(wh+2)*(ww+2)]
  const int PH = wh + 2, PW = ww + 2, PP = PH * PW;
  const long per_xcd = (nwin_total + 7) >> 3;
  const long gw = (long)(blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  if (gw >= nwin_total) return;
  const int img = (int)(gw / nWin), win = (int)(gw % nWin);
  const int wy = win / nWx, wx = win % nWx;
  const int c0 = blockIdx.y * 64;
  const int nc = (C - c0 < 64) ? C - c0 : 64;
  const int h0 = wy * wh - 1, w0 = wx * ww - 1;
  const float* xb = x + ((long)img * C + c0) * H * W;
  for (int e = threadIdx.x; e < nc * PP; e += 256) {
    const int c = e / PP, r = e % PP;
    const int py = r / PW, px = r % PW;
    const int hh = h0 + py, ww_ = w0 + px;
    patch[e] = (hh >= 0 && hh < H && ww_ >= 0 && ww_ < W) ? xb[((long)c * H + hh) * W + ww_] : 0.f;
  }
  __syncthreads();
  const int L = wh * ww;
  float* Tw = T + (gw * L) * C + c0;
  for (int e = threadIdx.x; e < L * nc; e += 256) {
    const int tok = e / nc, c = e % nc;
    const int iy = tok / ww, ix = tok % ww;
    const int hh = wy * wh + iy, ww_ = wx * ww + ix;
    float v = 0.f;
    if (hh < H && ww_ < W) {
      const float* pc = patch + c * PP + iy * PW + ix;
      const float* k = dw + (long)(c0 + c) * 9;
      v = k[0] * pc[0] + k[1] * pc[1] + k[2] * pc[2] + k[3] * pc[PW] + k[4] * pc[PW + 1] + k[5] * pc[PW + 2] +
          k[6] * pc[2 * PW] + k[7] * pc[2 * PW + 1] + k[8] * pc[2 * PW + 2];
    }
    Tw[(long)tok * C + c] = v;
  }
}

// =================================================================================================
// A2: adaptive-avg-pool over rows to `A` areas (overlapping bins [floor(a*H/A), ceil((a+1)*H/A))), emitted
// token-major S[(img*A + a)*W + w][c]  (a2_attn.py:44-48).  grid = (B*A), 256 threads.
// =================================================================================================
__global__ __launch_bounds__(256) void a2_pool_tokens_kernel(const float* __restrict__ xp, float* __restrict__ S, int C,
                                                             int H, int W, int A) {
  // grid = (B*A, ceil(C/64)): the (64 channels x W) slab is averaged with lanes along w (row-contiguous reads),
  // transposed through LDS and stored token-major with lanes along c (coalesced)
  extern __shared__ float slab[];  // [64][W + 1]
  const int img = blockIdx.x / A, a = blockIdx.x % A;
  const int c0 = blockIdx.y * 64;
  const int nc = (C - c0 < 64) ? C - c0 : 64;
  const int r0 = (a * H) / A, r1 = ((a + 1) * H + A - 1) / A;
  const float inv = (float)(r1 - r0);
  const float* xb = xp + ((long)img * C + c0) * H * W;
  const int nr = r1 - r0;
  for (int e = threadIdx.x; e < nc * W; e += 256) {
    const int c = e / W, w = e - c * W;
    const float* src = xb + ((long)c * H + r0) * W + w;
    float s = 0.f;
    int r = 0;
    for (; r + 4 <= nr; r += 4) {  // the bin's rows as independent loads, summed in row order
      const float v0 = src[(long)r * W], v1 = src[(long)(r + 1) * W], v2 = src[(long)(r + 2) * W],
                  v3 = src[(long)(r + 3) * W];
      s += v0;
      s += v1;
      s += v2;
      s += v3;
    }
    for (; r < nr; ++r) s += src[(long)r * W];
    slab[c * (W + 1) + w] = s / inv;
  }
  __syncthreads();
  float* Sb = S + ((long)img * A + a) * W * C + c0;
  for (int e = threadIdx.x; e < nc * W; e += 256) {
    const int w = e / nc, c = e - w * nc;
    Sb[(long)w * C + c] = slab[c * (W + 1) + w];
  }
}

// A2 tail: y = x + SiLU(up_h(T) + b), T = out_proj_conv(Z) laid out [img][C][A][W]; bilinear along H with
// align_corners=False (a2_attn.py:60), identity along W (same size). Upsampling commutes with the 1x1 conv.
__global__ __launch_bounds__(256) void a2_upsample_out_kernel(const float* __restrict__ x, const float* __restrict__ T,
                                                              const float* __restrict__ bias, float* __restrict__ y,
                                                              int C, int H, int W, int A) {
  // grid = (img*C planes, ceil(H*W / 256)); the plane's A x W rows of T are tiny and L1/L2-resident
  const long pc = blockIdx.x;  // img*C + c
  const int c = (int)(pc % C);
  const int e = blockIdx.y * 256 + threadIdx.x;
  if (e >= H * W) return;
  const int h = e / W, w = e - h * W;
  const float sc = (float)A / (float)H;
  float src = sc * ((float)h + 0.5f) - 0.5f;
  if (src < 0.f) src = 0.f;
  const int y0 = (int)src;
  const int y1 = y0 + ((y0 < A - 1) ? 1 : 0);
  const float l1 = src - (float)y0, l0 = 1.0f - l1;
  const float* Tp = T + pc * A * W;
  const float u = l0 * Tp[y0 * W + w] + l1 * Tp[y1 * W + w];
  const long o = pc * H * W + e;
  y[o] = x[o] + siluf_(u + bias[c]);
}

// The same tail with 4 consecutive elements of a plane per thread (H*W % 4 == 0): 16-byte x loads and y stores.
// grid = ceil(planes * H*W / 1024).
__global__ __launch_bounds__(256) void a2_upsample_out4_kernel(const float* __restrict__ x, const float* __restrict__ T,
                                                               const float* __restrict__ bias, float* __restrict__ y,
                                                               int C, int H, int W, int A, long total4) {
  const long i4 = (long)blockIdx.x * 256 + threadIdx.x;
  if (i4 >= total4) return;
  const long HW = (long)H * W;
  const long o = i4 * 4;
  const long pc = o / HW;  // img*C + c (HW % 4 == 0: the 4 elements share the plane)
  const int c = (int)(pc % C);
  const int e0 = (int)(o - pc * HW);
  const float sc = (float)A / (float)H;
  const float* Tp = T + pc * A * W;
  const float b = bias[c];
  const f32x4 xv = *reinterpret_cast<const f32x4*>(x + o);
  f32x4 r;
  // one division for the quad: its pixels are consecutive (a row change is a step of h)
  int h = e0 / W, w = e0 - h * W;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (k > 0 && ++w == W) {
      w = 0;
      ++h;
    }
    float src = sc * ((float)h + 0.5f) - 0.5f;
    if (src < 0.f) src = 0.f;
    const int y0 = (int)src;
    const int y1 = y0 + ((y0 < A - 1) ? 1 : 0);
    const float l1 = src - (float)y0, l0 = 1.0f - l1;
    const float u = l0 * Tp[y0 * W + w] + l1 * Tp[y1 * W + w];
    r[k] = xv[k] + silu_fast_(u + b);  // hardware exp2 / rcp, as the conv epilogues (~2^-22 relative)
  }
  *reinterpret_cast<f32x4*>(y + o) = r;
}

// The same tail when W % 4 == 0: a thread's 4 pixels are 4 columns of one row, so the two T rows it interpolates are
// read as two 16-byte loads (the general form above loads 8 scalars, each its own L2 round trip) and the row's
// interpolation weights are computed once. grid = ceil(planes * H*W / 1024).
__global__ __launch_bounds__(256) void a2_upsample_out4w_kernel(const float* __restrict__ x, const float* __restrict__ T,
                                                                const float* __restrict__ bias, float* __restrict__ y,
                                                                int C, int H, int W, int A, long total4) {
  const long i4 = (long)blockIdx.x * 256 + threadIdx.x;
  if (i4 >= total4) return;
  const long HW = (long)H * W;
  const long o = i4 * 4;
  const long pc = o / HW;  // img*C + c
  const int c = (int)(pc % C);
  const int e0 = (int)(o - pc * HW);
  const int h = e0 / W, w = e0 - h * W;
  const f32x4 xv = *reinterpret_cast<const f32x4*>(x + o);
  float src = ((float)A / (float)H) * ((float)h + 0.5f) - 0.5f;
  if (src < 0.f) src = 0.f;
  const int y0 = (int)src;
  const int y1 = y0 + ((y0 < A - 1) ? 1 : 0);
  const float l1 = src - (float)y0, l0 = 1.0f - l1;
  const float* Tp = T + pc * A * W + w;
  const f32x4 t0 = *reinterpret_cast<const f32x4*>(Tp + y0 * W);
  const f32x4 t1 = *reinterpret_cast<const f32x4*>(Tp + y1 * W);
  const float b = bias[c];
  f32x4 r;
#pragma unroll
  for (int k = 0; k < 4; ++k) r[k] = xv[k] + silu_fast_(l0 * t0[k] + l1 * t1[k] + b);
  *reinterpret_cast<f32x4*>(y + o) = r;
}


struct SwinGeom {
  int wh, ww, Hp, Wp, nWy, nWx, nWin, L;
  long ntok;
};
static SwinGeom swin_geom(int B, int H, int W, int ws) {
  SwinGeom g;
  g.wh = H < ws ? H : ws;
  g.ww = W < ws ? W : ws;
  if (H <= ws && W <= ws) {  // single global window, no pad (blocks_transformer.py:25-28)
    g.wh = H;
    g.ww = W;
  }
  g.Hp = H + (g.wh - H % g.wh) % g.wh;
  g.Wp = W + (g.ww - W % g.ww) % g.ww;
  g.nWy = g.Hp / g.wh;
  g.nWx = g.Wp / g.ww;
  g.nWin = g.nWy * g.nWx;
  g.L = g.wh * g.ww;
  g.ntok = (long)B * g.nWin * g.L;
  return g;
}

}  // namespace ys

using namespace ys;

int yolosod_swin_fused_launch(const float* x, float* y, int B, int C, int H, int W, int num_heads, int wh, int ww,
                              int nWx, int nWin, const float* dw_w, const float* ln1_w, const float* ln1_b,
                              float ln1_eps, const float* in_proj_w, const float* in_proj_b, const float* out_proj_w,
                              const float* out_proj_b, const float* ln2_w, const float* ln2_b, float ln2_eps,
                              const float* mlp1_w, const float* mlp1_b, int mlp_hidden, const float* mlp2_w,
                              const float* mlp2_b, const float* pw_w, const float* bn_scale, const float* bn_shift,
                              hipStream_t st);
int yolosod_swin_wide_launch(const float* x, float* y, int B, int C, int H, int W, int num_heads, int wh, int ww,
                             int nWx, int nWin, const float* dw_w, const float* ln1_w, const float* ln1_b,
                             float ln1_eps, const float* in_proj_w, const float* in_proj_b, const float* out_proj_w,
                             const float* out_proj_b, const float* ln2_w, const float* ln2_b, float ln2_eps,
                             const float* mlp1_w, const float* mlp1_b, int mlp_hidden, const float* mlp2_w,
                             const float* mlp2_b, const float* pw_w, const float* bn_scale, const float* bn_shift,
                             hipStream_t st);

bool yolosod_swin_x3_ok(int C, int num_heads, int wh, int ww, int mlp_hidden);
size_t yolosod_swin_x3_workspace(int C, int mlp_hidden);
size_t yolosod_swin_x3_run_workspace(int B, int C, int H, int W);
int yolosod_swin_x3_launch(const float* x, float* y, int B, int C, int H, int W, int num_heads, int wh, int ww,
                           int nWx, int nWin,
                           const float* dw_w, const float* ln1_w, const float* ln1_b, float ln1_eps,
                           const float* in_proj_w, const float* in_proj_b, const float* out_proj_w,
                           const float* out_proj_b, const float* ln2_w, const float* ln2_b, float ln2_eps,
                           const float* mlp1_w, const float* mlp1_b, int mlp_hidden, const float* mlp2_w,
                           const float* mlp2_b, const float* pw_w, const float* bn_w, const float* bn_b,
                           const float* bn_mean, const float* bn_var, float bn_eps, void* workspace,
                           size_t workspace_bytes, hipStream_t st);

static int g_swin_fused = 1;  // the fused per-window kernels (test hook: 0 = the decomposed GEMM path)

static bool swin_fused_enabled() { return g_swin_fused != 0; }

// Test hook: route SwinBlock through the fused per-window kernel (1) or the decomposed GEMM path (0).
YS_EXPORT void yolosod_debug_set_swin_fused(int on) { g_swin_fused = on ? 1 : 0; }

static bool swin_wide_enabled() { return true; }

// shapes the fused per-window kernels handle: swin_fused.hip (C <= 128, windows of <= 49 tokens) and
// swin_wide.hip (C = 256 with 4 heads of 64, 7x7 windows)
static bool swin_fused_ok(int C, int heads, int wh, int ww, int mlp_hidden) {
  if (!swin_fused_enabled() || wh * ww > 49 || mlp_hidden != 2 * C) return false;
  if (C == 256 && heads == 4) return swin_wide_enabled() && wh == 7 && ww == 7;
  return (C == 64 && (heads == 2 || heads == 4)) || (C == 128 && (heads == 2 || heads == 4));
}

// =================================================================================================
// C ABI
// =================================================================================================
YS_EXPORT int yolosod_gemm_f32(const float* A, long a_bs, int lda, const float* B, long b_bs, int ldb, int b_kcontig,
                               float* C, long c_bs, int ldc, int M, int N, int K, int batch, const float* bias,
                               int bias_mode, int act, const float* res, void* stream) {
  GemmArgs g{};
  g.A = A; g.a_bs = a_bs; g.lda = lda;
  g.B = B; g.b_bs = b_bs; g.ldb = ldb;
  g.M = M; g.N = N; g.K = K;
  g.epi = epi_plain(C, c_bs, ldc);
  g.epi.bias = bias; g.epi.bias_mode = bias ? bias_mode : 0;
  g.epi.act = act;
  g.epi.res = res; g.epi.res_bs = c_bs; g.epi.ldr = ldc;
  return launch_gemm(g, batch, b_kcontig != 0, (hipStream_t)stream);
}

// 1x1 convolution (stride 1, no groups) on NCHW as a batched GEMM with the conv epilogue fused:
// out[b*out_bs + m*HW + p] = act(sum_k W[m][k] x[b*x_bs + k*HW + p] + bias[m]) (+ res[b*res_bs + m*HW + p]).
// out / res may be channel slices of larger concat buffers (batch strides > Cout*HW).
YS_EXPORT int yolosod_conv1x1(const float* x, long x_bs, const float* w, const float* bias, float* out, long out_bs,
                              const float* res, long res_bs, int B, int Cin, int Cout, long HW, int act,
                              void* stream) {
  YS_CHECK_ARG(x && w && out, "conv1x1: null pointer");
  GemmArgs g{};
  g.A = w; g.lda = Cin;
  g.B = x; g.b_bs = x_bs; g.ldb = (int)HW;
  g.M = Cout; g.N = (int)HW; g.K = Cin;
  g.epi = epi_plain(out, out_bs, (int)HW);
  g.epi.bias = bias; g.epi.bias_mode = bias ? 1 : 0;
  g.epi.act = act;
  g.epi.res = res; g.epi.res_bs = res_bs; g.epi.ldr = (int)HW;
  return launch_gemm(g, B, false, (hipStream_t)stream);
}

YS_EXPORT int yolosod_layernorm(const float* x, float* y, long rows, int C, const float* w, const float* b, float eps,
                                void* stream) {
  return launch_layernorm(x, y, rows, C, w, b, eps, (hipStream_t)stream);
}

YS_EXPORT int yolosod_attention(const float* qkv, float* out, long n_seq, int L, int C, int heads, void* stream) {
  return launch_attention(qkv, out, n_seq, L, C, heads, (hipStream_t)stream);
}

YS_EXPORT size_t yolosod_swin_workspace(int B, int C, int H, int W, int window, int mlp_hidden) {
  SwinGeom g = swin_geom(B, H, W, window);
  Sizer s;
  s.take<float>((size_t)g.ntok * C);  // T (residual stream)
  s.take<float>((size_t)g.ntok * C);  // U (LN out / attention out)
  const int wide = (3 * C > mlp_hidden) ? 3 * C : mlp_hidden;
  s.take<float>((size_t)g.ntok * wide);  // QKV / MLP hidden
  s.take<float>((size_t)C * 2);          // folded BN
  s.take<float>((size_t)g.ntok * 2);     // LayerNorm row statistics
  return s.off;
}

__global__ void fold_bn_kernel(const float* w, const float* b, const float* m, const float* v, float eps, int C,
                               float* scale, float* shift) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const float inv = 1.0f / sqrtf(v[c] + eps);
  const float sc = w[c] * inv;
  scale[c] = sc;
  shift[c] = b[c] - m[c] * sc;
}

YS_EXPORT size_t yolosod_swin_workspace_v2(int B, int C, int H, int W, int num_heads, int window,
                                           int mlp_hidden) {
  SwinGeom g = swin_geom(B, H, W, window);
  if (swin_fused_ok(C, num_heads, g.wh, g.ww, mlp_hidden)) {
    Sizer s;
    s.take<float>((size_t)C * 2);
    if (yolosod_swin_x3_ok(C, num_heads, g.wh, g.ww, mlp_hidden)) {
      const size_t x3 = yolosod_swin_x3_workspace(C, mlp_hidden) + yolosod_swin_x3_run_workspace(B, C, H, W);
      return x3 > s.off ? x3 : s.off;
    }
    return s.off;
  }
  return yolosod_swin_workspace(B, C, H, W, window, mlp_hidden);
}

int yolosod_swin_x3_run(const float* x, float* y, int B, int C, int H, int W, int num_heads, int wh, int ww, int nWx,
                        int nWin, const float* dw_w, float ln1_eps, const float* out_proj_b, float ln2_eps,
                        int mlp_hidden, const float* mlp2_b, const void* prep, size_t prep_bytes, void* ws,
                        size_t ws_bytes, hipStream_t st);

// Scratch of yolosod_swin_forward_prepared for this shape (0 for shapes whose prepared kernels need none).
YS_EXPORT size_t yolosod_swin_prepared_workspace(int B, int C, int H, int W, int num_heads, int window,
                                                 int mlp_hidden) {
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || window <= 0) return 0;
  SwinGeom g = swin_geom(B, H, W, window);
  if (!yolosod_swin_x3_ok(C, num_heads, g.wh, g.ww, mlp_hidden)) return 0;
  return yolosod_swin_x3_run_workspace(B, C, H, W);
}

// SwinBlock.forward on a prepared-parameter block (yolosod_swin_prepare): the shapes the fp16-split kernels take
// (7x7 windows, yolosod_swin_prep_bytes > 0, one image's C*H*W < 2^30); anything else is an error (use
// yolosod_swin_forward). The batch is walked in chunks of images whose window count stays below 2^31.
YS_EXPORT int yolosod_swin_forward_prepared(const float* x, float* y, int B, int C, int H, int W, int num_heads,
                                            int window, const float* dw_w, float ln1_eps, const float* out_proj_b,
                                            float ln2_eps, int mlp_hidden, const float* mlp2_b, const void* prep,
                                            size_t prep_bytes, void* workspace, size_t workspace_bytes,
                                            void* stream) {
  YS_CHECK_ARG(x && y && dw_w && out_proj_b && mlp2_b && prep, "swin_prepared: null pointer");
  YS_CHECK_ARG(B >= 0 && C > 0 && H > 0 && W > 0 && window > 0, "swin_prepared: bad shape");
  if (B == 0) return 0;
  YS_CHECK_ARG((long)C * H * W < (1L << 30), "swin_prepared: one image of %dx%dx%d is too large for the prepared kernels",
               C, H, W);
  SwinGeom g = swin_geom(B, H, W, window);
  const long per = ((1L << 31) - 1) / (g.nWin > 0 ? g.nWin : 1);
  const int bc = per < B ? (int)per : B;
  const long img_el = (long)C * H * W;
  for (int b0 = 0; b0 < B; b0 += bc) {
    const int nb = B - b0 < bc ? B - b0 : bc;
    const int r = yolosod_swin_x3_run(x + b0 * img_el, y + b0 * img_el, nb, C, H, W, num_heads, g.wh, g.ww, g.nWx,
                                      g.nWin, dw_w, ln1_eps, out_proj_b, ln2_eps, mlp_hidden, mlp2_b, prep, prep_bytes,
                                      workspace, workspace_bytes, (hipStream_t)stream);
    if (r < 0) return -1;
    YS_CHECK_ARG(r == 1, "swin_prepared: shape C=%d heads=%d window %dx%d has no prepared-parameter kernel", C,
                 num_heads, g.wh, g.ww);
  }
  return 0;
}

YS_EXPORT int yolosod_swin_forward(const float* x, float* y, int B, int C, int H, int W, int num_heads, int window,
                                   const float* dw_w, const float* ln1_w, const float* ln1_b, float ln1_eps,
                                   const float* in_proj_w, const float* in_proj_b, const float* out_proj_w,
                                   const float* out_proj_b, const float* ln2_w, const float* ln2_b, float ln2_eps,
                                   const float* mlp1_w, const float* mlp1_b, int mlp_hidden, const float* mlp2_w,
                                   const float* mlp2_b, const float* pw_w, const float* bn_w, const float* bn_b,
                                   const float* bn_mean, const float* bn_var, float bn_eps, void* workspace,
                                   size_t workspace_bytes, void* stream) {
  YS_CHECK_ARG(x && y && dw_w && ln1_w && ln1_b && in_proj_w && in_proj_b && out_proj_w && out_proj_b && ln2_w &&
                   ln2_b && mlp1_w && mlp1_b && mlp2_w && mlp2_b && pw_w && bn_w && bn_b && bn_mean && bn_var,
               "swin: null pointer");
  YS_CHECK_ARG(B >= 0 && C > 0 && H > 0 && W > 0 && window > 0, "swin: bad shape");
  YS_CHECK_ARG(C % 32 == 0 && mlp_hidden % 32 == 0, "swin: C and mlp_hidden must be multiples of 32");
  if (B == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  SwinGeom g = swin_geom(B, H, W, window);
  YS_CHECK_ARG(g.L <= 320, "swin: window of %d tokens unsupported", g.L);
  if (swin_fused_ok(C, num_heads, g.wh, g.ww, mlp_hidden)) {
    // C = 64: projection / MLP / pw GEMMs on bf16 matrix cores at fp32 accuracy (swin_x3.hip)
    const int rx = yolosod_swin_x3_launch(x, y, B, C, H, W, num_heads, g.wh, g.ww, g.nWx, g.nWin, dw_w, ln1_w, ln1_b, ln1_eps,
                                          in_proj_w, in_proj_b, out_proj_w, out_proj_b, ln2_w, ln2_b, ln2_eps,
                                          mlp1_w, mlp1_b, mlp_hidden, mlp2_w, mlp2_b, pw_w, bn_w, bn_b, bn_mean,
                                          bn_var, bn_eps, workspace, workspace_bytes, st);
    if (rx < 0) return -1;
    if (rx == 1) return 0;
    Carver cf(workspace, workspace_bytes);
    float* fold = cf.take<float>((size_t)C * 2);
    YS_CHECK_ARG(fold, "swin: workspace too small (%zu)", workspace_bytes);
    hipLaunchKernelGGL(fold_bn_kernel, dim3((C + 255) / 256), dim3(256), 0, st, bn_w, bn_b, bn_mean, bn_var, bn_eps,
                       C, fold, fold + C);
    auto launch = C == 256 ? yolosod_swin_wide_launch : yolosod_swin_fused_launch;
    const int r = launch(x, y, B, C, H, W, num_heads, g.wh, g.ww, g.nWx, g.nWin, dw_w, ln1_w, ln1_b, ln1_eps,
                         in_proj_w, in_proj_b, out_proj_w, out_proj_b, ln2_w, ln2_b, ln2_eps, mlp1_w, mlp1_b,
                         mlp_hidden, mlp2_w, mlp2_b, pw_w, fold, fold + C, st);
    if (r < 0) return -1;
    if (r == 1) return 0;
  }
  Carver cv(workspace, workspace_bytes);
  float* T = cv.take<float>((size_t)g.ntok * C);
  float* U = cv.take<float>((size_t)g.ntok * C);
  const int wide = (3 * C > mlp_hidden) ? 3 * C : mlp_hidden;
  float* Q = cv.take<float>((size_t)g.ntok * wide);
  float* bn_fold = cv.take<float>((size_t)C * 2);
  float* lns = cv.take<float>((size_t)g.ntok * 2);
  YS_CHECK_ARG(lns, "swin: workspace too small (%zu)", workspace_bytes);
  int rc;

  const size_t lds = (size_t)64 * (g.wh + 2) * (g.ww + 2) * sizeof(float);
  YS_CHECK_ARG(lds <= 64 * 1024, "swin: window %dx%d too large for the partition kernel", g.wh, g.ww);
  hipLaunchKernelGGL(swin_partition_kernel, dim3((unsigned)(8 * (((long)B * g.nWin + 7) / 8)), (C + 63) / 64),
                     dim3(256), lds, st, x, dw_w, T, C, H, W, g.wh, g.ww, g.nWx, g.nWin, (long)B * g.nWin);
  YS_CHECK_LAUNCH("swin_partition");
  GemmArgs ga{};
  // QKV = LN1(T) Win^T + b_in   (LN1(T) -> U once: U is free until the attention writes it)
  if ((rc = launch_ln_rows(T, C, g.ntok, C, ln1_eps, ln1_w, ln1_b, U, C, st))) return rc;
  ga.A = U; ga.lda = C; ga.B = in_proj_w; ga.ldb = C; ga.M = (int)g.ntok; ga.N = 3 * C; ga.K = C;
  ga.epi = epi_plain(Q, 0, 3 * C);
  ga.epi.bias = in_proj_b; ga.epi.bias_mode = 2;
  if ((rc = launch_gemm(ga, 1, true, st))) return rc;
  if ((rc = launch_attention(Q, U, (long)B * g.nWin, g.L, C, num_heads, st))) return rc;
  // T = T + (O Wo^T + bo)
  ga = GemmArgs{};
  ga.A = U; ga.lda = C; ga.B = out_proj_w; ga.ldb = C; ga.M = (int)g.ntok; ga.N = C; ga.K = C;
  ga.epi = epi_plain(T, 0, C);
  ga.epi.bias = out_proj_b; ga.epi.bias_mode = 2; ga.epi.res = T; ga.epi.ldr = C;
  if ((rc = launch_gemm(ga, 1, true, st))) return rc;
  // Hd = GELU(LN2(T) W1^T + b1)
  ga = GemmArgs{};
  if ((rc = launch_ln_rows(T, C, g.ntok, C, ln2_eps, ln2_w, ln2_b, U, C, st))) return rc;  // the out-proj has read U
  ga.A = U; ga.lda = C; ga.B = mlp1_w; ga.ldb = C; ga.M = (int)g.ntok; ga.N = mlp_hidden; ga.K = C;
  ga.epi = epi_plain(Q, 0, mlp_hidden);
  ga.epi.bias = mlp1_b; ga.epi.bias_mode = 2; ga.epi.act = 2;
  if ((rc = launch_gemm(ga, 1, true, st))) return rc;
  // T = T + (Hd W2^T + b2)
  ga = GemmArgs{};
  ga.A = Q; ga.lda = mlp_hidden; ga.B = mlp2_w; ga.ldb = mlp_hidden; ga.M = (int)g.ntok; ga.N = C; ga.K = mlp_hidden;
  ga.epi = epi_plain(T, 0, C);
  ga.epi.bias = mlp2_b; ga.epi.bias_mode = 2; ga.epi.res = T; ga.epi.ldr = C;
  if ((rc = launch_gemm(ga, 1, true, st))) return rc;
  // y = x + SiLU(BN(pw . T)) with window reverse + crop: M = out channel, N = token
  float* bn_scale = bn_fold;
  float* bn_shift = bn_fold + C;
  hipLaunchKernelGGL(fold_bn_kernel, dim3((C + 255) / 256), dim3(256), 0, st, bn_w, bn_b, bn_mean, bn_var, bn_eps, C,
                     bn_scale, bn_shift);
  ga = GemmArgs{};
  ga.A = pw_w; ga.lda = C; ga.B = T; ga.ldb = C; ga.M = C; ga.N = (int)g.ntok; ga.K = C;
  ga.epi = epi_plain(y, 0, C);
  ga.epi.scale = bn_scale; ga.epi.shift = bn_shift; ga.epi.bn_mode = 1; ga.epi.act = 1;
  ga.epi.res = x;
  ga.epi.swin = 1; ga.epi.sw_H = H; ga.epi.sw_W = W; ga.epi.sw_wh = g.wh; ga.epi.sw_ww = g.ww;
  ga.epi.sw_nWx = g.nWx; ga.epi.sw_nWin = g.nWin;
  if ((rc = launch_gemm(ga, 1, true, st))) return rc;
  return 0;
}

// A2's GEMMs (proj, QKV, output): fp16 two-term split products (default) or exact fp32 MFMA (YOLOSOD_A2_X2=0)
static int g_a2_x2 = -1;
static bool a2_x2() {
  if (g_a2_x2 < 0) {
    const char* e = getenv("YOLOSOD_A2_X2");
    g_a2_x2 = (e && e[0] == '0') ? 0 : 1;
  }
  return g_a2_x2 != 0;
}
// Test hooks: A2 GEMMs as fp16 splits (1) or exact fp32 MFMA (0); every gemm_f32 call as fp16 splits (1) or as its
// caller asks (0)
YS_EXPORT int yolosod_debug_set_a2_x2(int on) {
  const int prev = a2_x2() ? 1 : 0;
  g_a2_x2 = on ? 1 : 0;
  return prev;
}
YS_EXPORT void yolosod_debug_set_gemm_x2(int on) { gemm_x2_forced() = on ? 1 : -1; }

bool yolosod_a2_fused_ok(int C, int num_heads, int L);
size_t yolosod_a2_fused_prep_bytes(int C);
int yolosod_a2_fused_prepare(int C, const float* proj_w, const float* ln_w, const float* ln_b, const float* in_w,
                             const float* in_b, void* prep, size_t prep_bytes, hipStream_t st);
int yolosod_a2_fused_run(const float* S, const float* stats, float* O, int B, int L, int C, int num_heads,
                         const void* prep, size_t prep_bytes, hipStream_t st);
bool yolosod_a2_proj_pool_ok(int C, int H, int W, int A);
int yolosod_a2_proj_pool_run(const float* x, const float* proj_b, float* S, int B, int C, int H, int W, int A,
                             const void* prep, size_t prep_bytes, hipStream_t st);

YS_EXPORT size_t yolosod_a2_workspace(int B, int C, int H, int W, int num_areas) {
  const long ntok = (long)B * num_areas * W;
  Sizer s;
  s.take<float>((size_t)B * C * H * W);  // proj output
  s.take<float>((size_t)ntok * C);       // S
  s.take<float>((size_t)ntok * C);       // U / O
  s.take<float>((size_t)ntok * 3 * C);   // QKV (decomposed path)
  s.take<float>((size_t)ntok * C);       // Z
  s.take<float>((size_t)ntok * 2);       // LayerNorm row statistics
  s.take<char>(yolosod_a2_fused_prep_bytes(C));  // per-call weight preparation of the fused LN / QKV / attention kernel
  return s.off;
}

// Size of the prepared-parameter block of the fused kernels (0: the shape takes neither). The proj + SiLU + pooling
// kernel takes it for any sequence length (its area groups bound the tile, checked per call with H), the LN / QKV /
// attention kernel for L = num_areas * W <= 160.
YS_EXPORT size_t yolosod_a2_prep_bytes(int C, int num_heads, int num_areas, int W) {
  const bool attn = yolosod_a2_fused_ok(C, num_heads, num_areas * W);
  const bool pool = yolosod_a2_fused_ok(C, num_heads, 1) && num_areas > 0 && W > 0;
  return (attn || pool) ? yolosod_a2_fused_prep_bytes(C) : 0;
}

// Weight preparation for yolosod_a2_forward_prepared: in_proj with the LayerNorm affine folded and the proj 1x1 conv
// (BN folded, as passed to the forward), split into fp16 planes; re-run whenever one of them changes.
YS_EXPORT int yolosod_a2_prepare(int C, const float* proj_w, const float* ln_w, const float* ln_b,
                                 const float* in_proj_w, const float* in_proj_b, void* prep, size_t prep_bytes,
                                 void* stream) {
  YS_CHECK_ARG(proj_w && ln_w && ln_b && in_proj_w && in_proj_b && prep, "a2_prepare: null pointer");
  YS_CHECK_ARG(C > 0 && C % 64 == 0 && C <= 1024, "a2_prepare: C=%d unsupported", C);
  return yolosod_a2_fused_prepare(C, proj_w, ln_w, ln_b, in_proj_w, in_proj_b, prep, prep_bytes,
                                  (hipStream_t)stream);
}

static int a2_forward_impl(const float* x, float* y, int B, int C, int H, int W, int num_areas, int num_heads,
                           const float* proj_w, const float* proj_b, const float* ln_w, const float* ln_b,
                           float ln_eps, const float* in_proj_w, const float* in_proj_b, const float* mha_out_w,
                           const float* mha_out_b, const float* oproj_w, const float* oproj_b, const void* prep,
                           size_t prep_bytes, void* workspace, size_t workspace_bytes, hipStream_t st);

YS_EXPORT int yolosod_a2_forward(const float* x, float* y, int B, int C, int H, int W, int num_areas, int num_heads,
                                 const float* proj_w, const float* proj_b, const float* ln_w, const float* ln_b,
                                 float ln_eps, const float* in_proj_w, const float* in_proj_b,
                                 const float* mha_out_w, const float* mha_out_b, const float* oproj_w,
                                 const float* oproj_b, void* workspace, size_t workspace_bytes, void* stream) {
  return a2_forward_impl(x, y, B, C, H, W, num_areas, num_heads, proj_w, proj_b, ln_w, ln_b, ln_eps, in_proj_w,
                         in_proj_b, mha_out_w, mha_out_b, oproj_w, oproj_b, nullptr, 0, workspace, workspace_bytes,
                         (hipStream_t)stream);
}

// The same forward on a prepared block (yolosod_a2_prepare of these LN / in_proj parameters) kept by the caller.
YS_EXPORT int yolosod_a2_forward_prepared(const float* x, float* y, int B, int C, int H, int W, int num_areas,
                                          int num_heads, const float* proj_w, const float* proj_b, const float* ln_w,
                                          const float* ln_b, float ln_eps, const float* in_proj_w,
                                          const float* in_proj_b, const float* oproj_w, const float* oproj_b,
                                          const void* prep, size_t prep_bytes, void* workspace,
                                          size_t workspace_bytes, void* stream) {
  YS_CHECK_ARG(prep, "a2_prepared: null prepared block");
  return a2_forward_impl(x, y, B, C, H, W, num_areas, num_heads, proj_w, proj_b, ln_w, ln_b, ln_eps, in_proj_w,
                         in_proj_b, nullptr, nullptr, oproj_w, oproj_b, prep, prep_bytes, workspace, workspace_bytes,
                         (hipStream_t)stream);
}

static int a2_forward_impl(const float* x, float* y, int B, int C, int H, int W, int num_areas, int num_heads,
                           const float* proj_w, const float* proj_b, const float* ln_w, const float* ln_b,
                           float ln_eps, const float* in_proj_w, const float* in_proj_b, const float* mha_out_w,
                           const float* mha_out_b, const float* oproj_w, const float* oproj_b, const void* prep,
                           size_t prep_bytes, void* workspace, size_t workspace_bytes, hipStream_t st) {
  YS_CHECK_ARG(x && y && proj_w && proj_b && ln_w && ln_b && in_proj_w && in_proj_b && oproj_w && oproj_b &&
                   (mha_out_w != nullptr) == (mha_out_b != nullptr),
               "a2: null pointer");
  const bool premul = mha_out_w == nullptr;  // oproj_w / oproj_b already include the MHA out-projection
  YS_CHECK_ARG(B >= 0 && C > 0 && H > 0 && W > 0 && num_areas > 0, "a2: bad shape");
  YS_CHECK_ARG(C % 32 == 0, "a2: C must be a multiple of 32");
  if (B == 0) return 0;
  const int A = num_areas;
  const long HW = (long)H * W;
  const long ntok = (long)B * A * W;
  Carver cv(workspace, workspace_bytes);
  float* XP = cv.take<float>((size_t)B * C * HW);
  float* S = cv.take<float>((size_t)ntok * C);
  float* U = cv.take<float>((size_t)ntok * C);
  float* Q = cv.take<float>((size_t)ntok * 3 * C);
  float* Z = cv.take<float>((size_t)ntok * C);
  float* lns = cv.take<float>((size_t)ntok * 2);
  const size_t fpb = yolosod_a2_fused_prep_bytes(C);
  char* fprep = cv.take<char>(fpb);
  YS_CHECK_ARG(fprep, "a2: workspace too small (%zu)", workspace_bytes);
  int rc;
  const bool x2 = a2_x2();
  const bool fused = x2 && yolosod_a2_fused_ok(C, num_heads, A * W);
  if (fused && !prep) {  // per-call weight preparation (callers that keep a block use yolosod_a2_forward_prepared)
    if ((rc = yolosod_a2_fused_prepare(C, proj_w, ln_w, ln_b, in_proj_w, in_proj_b, fprep, fpb, st))) return rc;
    prep = fprep;
    prep_bytes = fpb;
  }
  GemmArgs ga{};
  // the proj / pool kernel needs the prepared proj planes: a caller's block, or the per-call one of the fused path
  if (x2 && prep && yolosod_a2_proj_pool_ok(C, H, W, A) && ((uintptr_t)x & 15) == 0) {
    // proj + SiLU + row pooling in one kernel (a2_fused.hip): x -> S; the projected map never reaches HBM
    if ((rc = yolosod_a2_proj_pool_run(x, proj_b, S, B, C, H, W, A, prep, prep_bytes, st))) return rc;
  } else {
    // XP = SiLU(Wp x + bp)  (Conv with folded BN, a2_attn.py:39): M = Cout, N = HW, batched over images
    ga.A = proj_w; ga.lda = C; ga.B = x; ga.b_bs = C * HW; ga.ldb = (int)HW; ga.M = C; ga.N = (int)HW; ga.K = C;
    ga.epi = epi_plain(XP, C * HW, (int)HW);
    ga.epi.bias = proj_b; ga.epi.bias_mode = 1; ga.epi.act = 1;
    ga.x2 = x2; ga.x2_sa = 64.f;
    if ((rc = launch_gemm(ga, B, false, st))) return rc;
    YS_CHECK_ARG((size_t)64 * (W + 1) * sizeof(float) <= 64 * 1024, "a2: W=%d too large for the pooling kernel", W);
    hipLaunchKernelGGL(a2_pool_tokens_kernel, dim3(B * A, (C + 63) / 64), dim3(256),
                       (size_t)64 * (W + 1) * sizeof(float), st, XP, S, C, H, W, A);
    YS_CHECK_LAUNCH("a2_pool");
  }
  ga = GemmArgs{};
  if (fused) {
    // LN -> QKV -> attention per (image, head) in one kernel (a2_fused.hip): S + row statistics -> U
    if ((rc = launch_row_stats(S, C, ntok, C, ln_eps, lns, st))) return rc;
    if ((rc = yolosod_a2_fused_run(S, lns, U, B, A * W, C, num_heads, prep, prep_bytes, st))) return rc;
  } else {
    // LN(S) -> U once (U is free until the attention writes it), then the QKV GEMM without an LN prologue
    if ((rc = launch_ln_rows(S, C, ntok, C, ln_eps, ln_w, ln_b, U, C, st))) return rc;
    ga.A = U; ga.lda = C; ga.B = in_proj_w; ga.ldb = C; ga.M = (int)ntok; ga.N = 3 * C; ga.K = C;
    ga.epi = epi_plain(Q, 0, 3 * C);
    ga.epi.bias = in_proj_b; ga.epi.bias_mode = 2;
    ga.x2 = x2; ga.x2_sb = 64.f;
    if ((rc = launch_gemm(ga, 1, true, st))) return rc;
    if ((rc = launch_attention(Q, U, B, A * W, C, num_heads, st))) return rc;
  }
  if (!premul) {
    ga = GemmArgs{};
    ga.A = U; ga.lda = C; ga.B = mha_out_w; ga.ldb = C; ga.M = (int)ntok; ga.N = C; ga.K = C;
    ga.epi = epi_plain(Z, 0, C);
    ga.epi.bias = mha_out_b; ga.epi.bias_mode = 2;
    ga.x2 = x2; ga.x2_sb = 64.f;
    if ((rc = launch_gemm(ga, 1, true, st))) return rc;
  }
  // T[img][n][t] = sum_c Wout[n][c] Z[img*AW + t][c]   (reuse S as T: B*C*A*W floats == ntok*C)
  float* T = S;
  ga = GemmArgs{};
  ga.A = oproj_w; ga.lda = C; ga.B = premul ? U : Z; ga.b_bs = (long)A * W * C; ga.ldb = C; ga.M = C; ga.N = A * W; ga.K = C;
  ga.epi = epi_plain(T, (long)C * A * W, A * W);
  ga.x2 = x2; ga.x2_sa = 64.f;
  if ((rc = launch_gemm(ga, B, true, st))) return rc;
  if (W % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0) {
    const long total4 = (long)B * C * HW / 4;
    hipLaunchKernelGGL(a2_upsample_out4w_kernel, dim3((unsigned)((total4 + 255) / 256)), dim3(256), 0, st, x, T,
                       oproj_b, y, C, H, W, A, total4);
  } else if (HW % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0) {
    const long total4 = (long)B * C * HW / 4;
    hipLaunchKernelGGL(a2_upsample_out4_kernel, dim3((unsigned)((total4 + 255) / 256)), dim3(256), 0, st, x, T, oproj_b,
                       y, C, H, W, A, total4);
  } else {
    hipLaunchKernelGGL(a2_upsample_out_kernel, dim3((unsigned)(B * C), (unsigned)((HW + 255) / 256)), dim3(256), 0,
                       st, x, T, oproj_b, y, C, H, W, A);
  }
  YS_CHECK_LAUNCH("a2_upsample");
  return 0;
}
