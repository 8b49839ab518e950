// Fused SwinBlock for small channel counts (C <= 128: the P2 instance L28, C = 64 in the paper model).
//
// One 256-thread workgroup = one 7x7 window. The window's tokens never leave LDS between the depthwise conv and
// the final pw1x1+BN+SiLU+residual, so the per-token HBM traffic is read x (+ halo) once and write y once, against
// ~5.5 GB of token-major scratch for the decomposed path at 640^2 bs=32.
//
// Stages (ultralytics/nn/modules/blocks_transformer.py):
//   0 dw3x3 (pad 1, no bias) on the (wh+2)x(ww+2) halo patch -> T[tok][c]; tokens of the bottom/right zero pad = 0
//     (:160, window_partition :31-46)
//   1 U = LN1(T)                                   (:112)
//   2 QKV = U Win^T + b_in                         (MHA in_proj, :116)
//   3 per head: S^T = K Q^T * scale, softmax over keys (keys >= L masked), O^T = V^T P^T  (:116)
//   4 T += O Wo^T + bo                             (out_proj + residual, :119)
//   5 U = LN2(T); 6 Hd = GELU(U W1^T + b1); 7 T += Hd W2^T + b2   (:122)
//   8 y = x + SiLU(BN(Wpw T^T)) on the valid (cropped) tokens, NCHW   (window_reverse + crop :125-129, :166-171)
// All GEMMs run on v_mfma_f32_16x16x4_f32 (exact fp32). A wave owns a slice of output columns for all 64
// (padded) token rows; the MFMA k index is permuted (lane group g takes k in [g*K/4, (g+1)*K/4)) so operands are
// 16-byte loads: A from LDS, weights straight from global (L2-resident, each weight element read once per
// window). Attention computes S^T so that its accumulator registers are directly the B operand of O^T = V^T P^T
// (keys permuted consistently), so P never touches LDS.
// Padding rows: only 49 token rows + 1 zero row are stored; MFMA rows >= 49 read the zero row and their outputs
// are discarded.
#include "common.h"
#include <math.h>
#include <stdlib.h>

namespace ys {

constexpr int SW_ROWS = 50;  // 49 tokens + zero row

struct SwinFusedArgs {
  const float* x;
  float* y;
  int B, H, W, wh, ww, nWx, nWin, L;
  const float* dw;
  const float* ln1_w;
  const float* ln1_b;
  float ln1_eps;
  const float* win;
  const float* bin;
  const float* wo;
  const float* bo;
  const float* ln2_w;
  const float* ln2_b;
  float ln2_eps;
  const float* w1;
  const float* b1;
  const float* w2;
  const float* b2;
  const float* wpw;
  const float* bn_scale;
  const float* bn_shift;
  float scale;
  int abl;  // timing ablation (debug only): 1 skip halo loads, 2 skip weight loads, 4 skip residual loads
  unsigned long long* stamps;  // diagnostic build only: per-stage s_memtime of wave 0 ([grid][16]) or nullptr
};

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// acc[rb][j] = A'[rows of block rb][K] . W[n][K]^T for this wave's column blocks cb = wid + 4*j (NCB % 4 == 0).
// A: LDS [SW_ROWS][lda], row index clamped to the zero row (SW_ROWS-1). With LN, A' = (A - mean_r)*rstd_r*w + b
// (row statistics from `stats`, LN affine parameters from LDS) is applied to the fragments as they are read, so no
// normalised copy of the tile is stored. W: global [N][K], fragments loaded up front. MFMAs are issued
// component-outer so 4*NJ independent accumulators separate dependent ones.
template <int K, int NCB, bool LN>
__device__ __forceinline__ void wave_gemm_rows(const float* __restrict__ As, int lda, const float* __restrict__ Wg,
                                               f32x4 (&acc)[4][NCB / 4], const float* stats, const float* lnw,
                                               const float* lnb, int abl) {
  constexpr int NJ = NCB / 4;
  static_assert(NCB % 4 == 0, "column blocks must split evenly over the 4 waves");
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int l15 = lane & 15, g = lane >> 4;
  constexpr int KQ = K / 4;  // k range per lane group
  float4 bw[NJ][KQ / 4];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const float* wr = Wg + (long)((wid + 4 * j) * 16 + l15) * K + g * KQ;
#pragma unroll
    for (int t = 0; t < KQ / 4; ++t)
      bw[j][t] = (abl & 2) ? make_float4(0.f, 0.f, 0.f, 0.f) : *reinterpret_cast<const float4*>(wr + 4 * t);
  }
  const float* arow[4];
  float mu[4], rs[4];
#pragma unroll
  for (int rb = 0; rb < 4; ++rb) {
    int r = rb * 16 + l15;
    r = r < SW_ROWS - 1 ? r : SW_ROWS - 1;
    arow[rb] = As + r * lda + g * KQ;
    if (LN) {
      mu[rb] = stats[2 * r];
      rs[rb] = stats[2 * r + 1];
    }
  }
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[rb][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < KQ / 4; ++t) {
    float4 a[4];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) a[rb] = *reinterpret_cast<const float4*>(arow[rb] + 4 * t);
    if (LN) {
      const float4 w = *reinterpret_cast<const float4*>(lnw + g * KQ + 4 * t);
      const float4 bb = *reinterpret_cast<const float4*>(lnb + g * KQ + 4 * t);
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        a[rb].x = (a[rb].x - mu[rb]) * rs[rb] * w.x + bb.x;
        a[rb].y = (a[rb].y - mu[rb]) * rs[rb] * w.y + bb.y;
        a[rb].z = (a[rb].z - mu[rb]) * rs[rb] * w.z + bb.z;
        a[rb].w = (a[rb].w - mu[rb]) * rs[rb] * w.w + bb.w;
      }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const float av = c == 0 ? a[rb].x : c == 1 ? a[rb].y : c == 2 ? a[rb].z : a[rb].w;
          const float bv = c == 0 ? bw[j][t].x : c == 1 ? bw[j][t].y : c == 2 ? bw[j][t].z : bw[j][t].w;
          acc[rb][j] = mfma4(av, bv, acc[rb][j]);
        }
  }
}

// Row statistics (mean, rstd) of rows [0, SW_ROWS) of S[SW_ROWS][lds] over C: 4 threads per row (all rows at
// once), each with C/4 values from float4 LDS reads, two-pass, DPP quad reductions; rows >= L get (0, 0).
template <int C>
__device__ __forceinline__ void lds_row_stats(const float* S, int lds, float* stats, int L, float eps) {
  constexpr int CP = C / 4;
  const int tid = threadIdx.x;
  const int r = tid >> 2, qd = tid & 3;
  const bool valid = r < L;
  float4 v[CP / 4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < CP / 4; ++i) {
    v[i] = valid ? *reinterpret_cast<const float4*>(S + r * lds + qd * CP + 4 * i) : make_float4(0.f, 0.f, 0.f, 0.f);
    s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  }
  const float mean = quad_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < CP / 4; ++i) {
    const float a0 = v[i].x - mean, a1 = v[i].y - mean, a2 = v[i].z - mean, a3 = v[i].w - mean;
    q += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
  }
  const float var = quad_sum(q) / (float)C;
  if (qd == 0 && r < SW_ROWS) {
    stats[2 * r] = valid ? mean : 0.f;
    stats[2 * r + 1] = valid ? 1.0f / sqrtf(var + eps) : 0.f;
  }
}

#define YS_STAMP(k)                                                                  \
  if (p.stamps && tid == 0) p.stamps[gw * 16 + (k)] = __builtin_amdgcn_s_memtime();

template <int C, int NH, bool W7>
__global__ __launch_bounds__(256, 3) void swin_fused_kernel(SwinFusedArgs p) {
  constexpr int HD = C / NH;
  constexpr int HID = 2 * C;
  constexpr int LT = C + 4;          // T row stride (== 4 mod 64 floats: conflict-free b128 row reads)
  constexpr int LQ = 3 * C + 4;      // QKV row stride (also holds the attention output and the MLP hidden)
  constexpr int LH = HID + 4;
  constexpr int NR = (C * 9 + 255) / 256;  // halo rows (of <= 9 floats) per thread
  static_assert(HD % 16 == 0 && HD <= 64, "head dim");
  static_assert(LH <= LQ, "MLP hidden must fit the QKV region");
  // T: residual stream; Q: x halo patch (stage 0) -> QKV (O overwrites each wave's own query columns) -> hidden;
  // stats: per-row (mean, rstd); lnp: LN1/LN2 affine parameters
  __shared__ __attribute__((aligned(16))) float smem[SW_ROWS * LT + SW_ROWS * LQ + 2 * SW_ROWS + 4 * C];
  float* T = smem;
  float* Q = smem + SW_ROWS * LT;
  float* stats = Q + SW_ROWS * LQ;
  float* lnp = stats + 2 * SW_ROWS;  // [ln1_w | ln1_b | ln2_w | ln2_b]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l15 = lane & 15, g = lane >> 4;
  const int wh = W7 ? 7 : p.wh, ww = W7 ? 7 : p.ww, L = W7 ? 49 : p.L;
  const int H = p.H, W = p.W;
  const long HWl = (long)H * W;
  const int PH = wh + 2, PW = ww + 2, PP = PH * PW;
  const long total = (long)p.B * p.nWin;

  // persistent: loop-invariant LN parameters (LDS) and depthwise taps (registers)
  for (int e = tid; e < 4 * C; e += 256) {
    const int which = e / C, c = e - which * C;
    const float* src = which == 0 ? p.ln1_w : which == 1 ? p.ln1_b : which == 2 ? p.ln2_w : p.ln2_b;
    lnp[e] = src[c];
  }
  constexpr int TG = 256 / C;
  const int dw_c = tid % C, dw_tg = tid / C;
  float dwk[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) dwk[i] = p.dw[dw_c * 9 + i];

  // halo patch [C][PH][PW] of window gwin into registers, row-wise: thread -> (c, py) rows of PW floats
  float hv[NR][9];
  auto load_halo = [&](long gwin) {
    const int im = (int)(gwin / p.nWin), wn = (int)(gwin % p.nWin);
    const int wy_ = wn / p.nWx, wx_ = wn % p.nWx;
    const int h0 = wy_ * wh - 1, w0 = wx_ * ww - 1;
    const float* xb_ = p.x + (long)im * C * HWl;
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int rr = tid + 256 * i;
      const int c = rr / PH, py = rr - c * PH;
      const int hh = h0 + py;
      const bool rowok = rr < C * PH && hh >= 0 && hh < H && !(p.abl & 1);
      const float* src = xb_ + (long)c * HWl + (long)hh * W + w0;
#pragma unroll
      for (int px = 0; px < 9; ++px) {
        const int wc = w0 + px;
        hv[i][px] = (rowok && px < PW && wc >= 0 && wc < W) ? src[px] : 0.f;
      }
    }
  };
  // one window per workgroup, XCD-aware: workgroup i runs on XCD i % 8, so each XCD gets a contiguous range of
  // windows and neighbouring windows (which share 128-B lines of x and y: a window row is only 28 B wide) meet in
  // the same L2 instead of each XCD fetching / partially writing back the same lines.
  const long nwin_total = (long)p.B * p.nWin;
  const long per_xcd = (nwin_total + 7) >> 3;
  const long gw = (long)(blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  if (gw >= nwin_total) return;
  load_halo(gw);
  const float* w_in = p.win;
  const float* w_o = p.wo;
  const float* w_1 = p.w1;
  const float* w_2 = p.w2;
  const float* w_pw = p.wpw;
  const int img = (int)(gw / p.nWin), win = (int)(gw % p.nWin);
  const int wy = win / p.nWx, wx = win % p.nWx;
  const float* xb = p.x + (long)img * C * HWl;
  YS_STAMP(0)

  // ---- stage 0: halo patch (prefetched) -> LDS -> dw conv -> T (rows >= L and the zero row are 0) ----
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int rr = tid + 256 * i;
    if (rr < C * PH) {
#pragma unroll
      for (int px = 0; px < 9; ++px)
        if (px < PW) Q[rr * PW + px] = hv[i][px];
    }
  }
  __syncthreads();
  YS_STAMP(1)
  {
    // thread -> channel c (taps in registers), tokens tok = tg, tg + TG, ...
    const float* pcb = Q + dw_c * PP;
    for (int tok = dw_tg; tok < SW_ROWS; tok += TG) {
      float v = 0.f;
      if (tok < L) {
        const int iy = tok / ww, ix = tok - iy * ww;
        const int hh = wy * wh + iy, wc = wx * ww + ix;
        if (hh < H && wc < W) {
          const float* pc = pcb + iy * PW + ix;
          v = dwk[0] * pc[0] + dwk[1] * pc[1] + dwk[2] * pc[2] + dwk[3] * pc[PW] + dwk[4] * pc[PW + 1] +
              dwk[5] * pc[PW + 2] + dwk[6] * pc[2 * PW] + dwk[7] * pc[2 * PW + 1] + dwk[8] * pc[2 * PW + 2];
        }
      }
      T[tok * LT + dw_c] = v;
    }
  }
  __syncthreads();
  YS_STAMP(2)

  // ---- stage 1: LN1 row statistics; zero row of Q ----
  lds_row_stats<C>(T, LT, stats, L, p.ln1_eps);
  for (int c = tid; c < LQ; c += 256) Q[(SW_ROWS - 1) * LQ + c] = 0.f;
  __syncthreads();
  YS_STAMP(3)

  // ---- stage 2: QKV = LN1(T) Win^T + b_in ----
  {
    constexpr int NCB = 3 * C / 16;
    constexpr int NJ = NCB / 4;
    f32x4 acc[4][NJ];
    wave_gemm_rows<C, NCB, true>(T, LT, w_in, acc, stats, lnp, lnp + C, p.abl);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = (wid + 4 * j) * 16 + l15;
      const float bias = p.bin[n];
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rb * 16 + g * 4 + r;
          if (row < SW_ROWS - 1) Q[row * LQ + n] = acc[rb][j][r] + bias;
        }
    }
  }
  __syncthreads();
  YS_STAMP(4)

  // ---- stage 3: attention, wave = query block (16 queries), all heads interleaved ----
  // The output O[q][h*HD + d] overwrites the query columns of the wave's own rows (read only by this wave).
  {
    const int qb = wid;
    int qrow = qb * 16 + l15;
    qrow = qrow < SW_ROWS - 1 ? qrow : SW_ROWS - 1;
    constexpr int DQ = HD / 4;  // d range per lane group
    f32x4 st[NH][4];
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) st[h][kb] = f32x4{0.f, 0.f, 0.f, 0.f};
    int krow[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const int kr = kb * 16 + l15;
      krow[kb] = kr < SW_ROWS - 1 ? kr : SW_ROWS - 1;
    }
#pragma unroll
    for (int t = 0; t < DQ / 4; ++t) {
      float4 qv[NH], kv[NH][4];
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        qv[h] = *reinterpret_cast<const float4*>(Q + qrow * LQ + h * HD + g * DQ + 4 * t);
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
          kv[h][kb] = *reinterpret_cast<const float4*>(Q + krow[kb] * LQ + C + h * HD + g * DQ + 4 * t);
      }
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int h = 0; h < NH; ++h)
#pragma unroll
          for (int kb = 0; kb < 4; ++kb) {
            const float kk = c == 0 ? kv[h][kb].x : c == 1 ? kv[h][kb].y : c == 2 ? kv[h][kb].z : kv[h][kb].w;
            const float qq = c == 0 ? qv[h].x : c == 1 ? qv[h].y : c == 2 ? qv[h].z : qv[h].w;
            st[h][kb] = mfma4(kk, qq, st[h][kb]);
          }
    }
    // lane holds S^T[key = kb*16 + 4g + r][q = l15] per head: softmax over keys (in-lane, then lane groups)
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      float mx = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kb * 16 + 4 * g + r;
          const float sv = (key < L) ? st[h][kb][r] * p.scale : -INFINITY;
          st[h][kb][r] = sv;
          mx = fmaxf(mx, sv);
        }
      mx = xor32_max(xor16_max(mx));
      float sum = 0.f;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __expf(st[h][kb][r] - mx);
          st[h][kb][r] = e;
          sum += e;
        }
      sum = xor32_sum(xor16_sum(sum));
      const float inv = 1.0f / sum;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) st[h][kb][r] *= inv;
    }
    // O^T[d][q] = sum_key V[key][d] P[q][key]; MFMA (kb, r) consumes keys {kb*16 + 4g' + r}
    f32x4 o[NH][HD / 16];
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
      for (int db = 0; db < HD / 16; ++db) o[h][db] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int key = kb * 16 + 4 * g + r;
        key = key < SW_ROWS - 1 ? key : SW_ROWS - 1;
        const float* vrow = Q + key * LQ + 2 * C + l15;
#pragma unroll
        for (int h = 0; h < NH; ++h)
#pragma unroll
          for (int db = 0; db < HD / 16; ++db) o[h][db] = mfma4(vrow[h * HD + db * 16], st[h][kb][r], o[h][db]);
      }
    // lane holds O^T[d = db*16 + 4g + r][q = l15] -> O[q][h*HD + d] (4 consecutive d) into the q columns
    const int q = qb * 16 + l15;
    if (q < L) {
#pragma unroll
      for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int db = 0; db < HD / 16; ++db)
          *reinterpret_cast<f32x4*>(Q + q * LQ + h * HD + db * 16 + 4 * g) = o[h][db];
    }
  }
  __syncthreads();
  YS_STAMP(5)

  // ---- stage 4: T += O Wo^T + bo ----
  {
    constexpr int NCB = C / 16;
    constexpr int NJ = NCB / 4;
    f32x4 acc[4][NJ];
    wave_gemm_rows<C, NCB, false>(Q, LQ, w_o, acc, nullptr, nullptr, nullptr, p.abl);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = (wid + 4 * j) * 16 + l15;
      const float bias = p.bo[n];
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rb * 16 + g * 4 + r;
          if (row < L) T[row * LT + n] += acc[rb][j][r] + bias;
        }
    }
  }
  __syncthreads();
  YS_STAMP(6)

  // ---- stage 5: LN2 row statistics ----
  lds_row_stats<C>(T, LT, stats, L, p.ln2_eps);
  __syncthreads();
  YS_STAMP(7)

  // ---- stage 6: Hd = GELU(LN2(T) W1^T + b1) -> Q region [rows][LH] ----
  float* Hd = Q;
  {
    constexpr int NCB = HID / 16;
    constexpr int NJ = NCB / 4;
    f32x4 acc[4][NJ];
    wave_gemm_rows<C, NCB, true>(T, LT, w_1, acc, stats, lnp + 2 * C, lnp + 3 * C, p.abl);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = (wid + 4 * j) * 16 + l15;
      const float bias = p.b1[n];
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rb * 16 + g * 4 + r;
          if (row < SW_ROWS - 1) Hd[row * LH + n] = gelu_fast_(acc[rb][j][r] + bias);
        }
    }
    for (int c = tid; c < LH; c += 256) Hd[(SW_ROWS - 1) * LH + c] = 0.f;
  }
  __syncthreads();
  YS_STAMP(8)

  // ---- stage 7: T += Hd W2^T + b2 ----
  {
    constexpr int NCB = C / 16;
    constexpr int NJ = NCB / 4;
    f32x4 acc[4][NJ];
    wave_gemm_rows<HID, NCB, false>(Hd, LH, w_2, acc, nullptr, nullptr, nullptr, p.abl);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = (wid + 4 * j) * 16 + l15;
      const float bias = p.b2[n];
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rb * 16 + g * 4 + r;
          if (row < L) T[row * LT + n] += acc[rb][j][r] + bias;
        }
    }
  }
  __syncthreads();
  YS_STAMP(9)

  // ---- stage 8: y = x + SiLU(BN(Wpw T^T)); output tile Y^T[c][tok] (lanes over tokens) ----
  {
    constexpr int NCB = C / 16;
    constexpr int CQ = C / 4;
    float* yb = p.y + (long)img * C * HWl;
    for (int cb = wid; cb < NCB; cb += 4) {
      const float* wrow = w_pw + (long)(cb * 16 + l15) * C + g * CQ;
      // residual x and BN terms first (their latency overlaps the MFMAs)
      long pix[4];
      float xr[4][4];
#pragma unroll
      for (int tb = 0; tb < 4; ++tb) {
        const int tok = tb * 16 + l15;
        const int iy = tok / ww, ix = tok - iy * ww;
        const int hh = wy * wh + iy, wc = wx * ww + ix;
        pix[tb] = (tok < L && hh < H && wc < W) ? (long)hh * W + wc : -1;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          xr[tb][r] = (pix[tb] >= 0 && !(p.abl & 4)) ? xb[(long)(cb * 16 + 4 * g + r) * HWl + pix[tb]] : 0.f;
      }
      float bsc[4], bsh[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        bsc[r] = p.bn_scale[cb * 16 + 4 * g + r];
        bsh[r] = p.bn_shift[cb * 16 + 4 * g + r];
      }
      f32x4 acc[4];
#pragma unroll
      for (int tb = 0; tb < 4; ++tb) acc[tb] = f32x4{0.f, 0.f, 0.f, 0.f};
      float4 wa[CQ / 4];
#pragma unroll
      for (int t = 0; t < CQ / 4; ++t) wa[t] = *reinterpret_cast<const float4*>(wrow + 4 * t);
#pragma unroll
      for (int t = 0; t < CQ / 4; ++t) {
        float4 bt[4];
#pragma unroll
        for (int tb = 0; tb < 4; ++tb) {
          int tr = tb * 16 + l15;
          tr = tr < SW_ROWS - 1 ? tr : SW_ROWS - 1;
          bt[tb] = *reinterpret_cast<const float4*>(T + tr * LT + g * CQ + 4 * t);
        }
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int tb = 0; tb < 4; ++tb) {
            const float av = c == 0 ? wa[t].x : c == 1 ? wa[t].y : c == 2 ? wa[t].z : wa[t].w;
            const float bv = c == 0 ? bt[tb].x : c == 1 ? bt[tb].y : c == 2 ? bt[tb].z : bt[tb].w;
            acc[tb] = mfma4(av, bv, acc[tb]);
          }
      }
      // lane holds Y^T[c = cb*16 + 4g + r][tok = tb*16 + l15]
#pragma unroll
      for (int tb = 0; tb < 4; ++tb) {
        if (pix[tb] < 0) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = cb * 16 + 4 * g + r;
          yb[(long)c * HWl + pix[tb]] = xr[tb][r] + silu_fast_(acc[tb][r] * bsc[r] + bsh[r]);
        }
      }
    }
  }
  YS_STAMP(15)
}

}  // namespace ys

using namespace ys;

static unsigned long long* g_stamps = nullptr;  // diagnostic build only (YOLOSOD_SWIN_STAMPS)
static size_t g_stamp_cap = 0, g_stamp_n = 0;

// Diagnostic: average cycles between consecutive per-stage stamps of the last fused launch (synchronous).
YS_EXPORT int yolosod_debug_swin_stage_cycles(double* out, int n) {
  if (!g_stamps || n > 16) return -1;
  const size_t cnt = g_stamp_n;
  unsigned long long* h = (unsigned long long*)malloc(cnt * sizeof(unsigned long long));
  if (hipMemcpy(h, g_stamps, cnt * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) { free(h); return -1; }
  for (int k = 0; k < n; ++k) out[k] = 0.0;
  size_t blocks = cnt / 16;
  for (size_t b = 0; b < blocks; ++b) {
    unsigned long long* r = h + b * 16;
    unsigned long long prev = r[0];
    for (int k = 1; k < 16; ++k) {
      if (!r[k]) continue;
      if (k < n) out[k] += (double)(r[k] - prev);
      prev = r[k];
    }
  }
  for (int k = 0; k < n; ++k) out[k] /= (double)blocks;
  free(h);
  return 0;
}

// returns 1 if launched, 0 if the shape is not handled by the fused kernel, <0 on error
int yolosod_swin_fused_launch(const float* x, float* y, int B, int C, int H, int W, int num_heads, int wh, int ww,
                              int nWx, int nWin, const float* dw_w, const float* ln1_w, const float* ln1_b,
                              float ln1_eps, const float* in_proj_w, const float* in_proj_b, const float* out_proj_w,
                              const float* out_proj_b, const float* ln2_w, const float* ln2_b, float ln2_eps,
                              const float* mlp1_w, const float* mlp1_b, int mlp_hidden, const float* mlp2_w,
                              const float* mlp2_b, const float* pw_w, const float* bn_scale, const float* bn_shift,
                              hipStream_t st) {
  const int L = wh * ww;
  if (L > SW_ROWS - 1 || (wh + 2) * (ww + 2) * C > SW_ROWS * (3 * C + 4) || mlp_hidden != 2 * C) return 0;
  SwinFusedArgs a{x, y, B, H, W, wh, ww, nWx, nWin, L, dw_w, ln1_w, ln1_b, ln1_eps, in_proj_w, in_proj_b,
                  out_proj_w, out_proj_b, ln2_w, ln2_b, ln2_eps, mlp1_w, mlp1_b, mlp2_w, mlp2_b, pw_w,
                  bn_scale, bn_shift, 1.0f / sqrtf((float)(C / num_heads)), 0, nullptr};
  if (const char* e = getenv("YOLOSOD_SWIN_ABL")) a.abl = atoi(e);
  a.stamps = nullptr;
  if (getenv("YOLOSOD_SWIN_STAMPS")) {
    const size_t need = (size_t)B * nWin * 16;
    if (need > g_stamp_cap) {
      if (g_stamps) (void)hipFree(g_stamps);
      g_stamps = nullptr;
      if (hipMalloc((void**)&g_stamps, need * sizeof(unsigned long long)) != hipSuccess) return -1;
      g_stamp_cap = need;
    }
    (void)hipMemsetAsync(g_stamps, 0, need * sizeof(unsigned long long), st);
    g_stamp_n = need;
    a.stamps = g_stamps;
  }
  // one window per workgroup (XCD-aware order, padded to a multiple of 8); 3 resident per CU (LDS 53 KB, 168 VGPRs)
  dim3 grid((unsigned)(8 * (((long)B * nWin + 7) / 8)));
  const bool w7 = (wh == 7 && ww == 7);
#define YS_SWF(CC, NHH)                                                                                  \
  if (C == CC && num_heads == NHH) {                                                                     \
    if (w7) hipLaunchKernelGGL((swin_fused_kernel<CC, NHH, true>), grid, dim3(256), 0, st, a);           \
    else hipLaunchKernelGGL((swin_fused_kernel<CC, NHH, false>), grid, dim3(256), 0, st, a);             \
  } else
  YS_SWF(64, 2) YS_SWF(64, 4) YS_SWF(128, 2) YS_SWF(128, 4) return 0;
#undef YS_SWF
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("swin_fused: launch failed: %s", hipGetErrorString(e));
    return -1;
  }
  return 1;
}
