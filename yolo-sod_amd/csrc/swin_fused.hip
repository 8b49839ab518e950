// Fused SwinBlock for small channel counts (C <= 128: the P2 instance L28, C = 64 in the paper model).
//
// One 256-thread workgroup processes one 7x7 window. The window's tokens never leave LDS between the depthwise conv and the final pw1x1+BN+SiLU+residual,
// so the per-token HBM traffic is read x (+ halo) once and write y once, against ~5.5 GB of token-major scratch
// for the decomposed path at 640^2 bs=32.
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
// GEMMs run on v_mfma_f32_16x16x4_f32 (exact fp32). A wave owns a slice of output columns for all token rows;
// the MFMA k index is permuted (lane group g takes k in [g*K/4, (g+1)*K/4)) so operands are 16-byte loads: A
// from LDS, weights straight from global (L2-resident). 49 tokens = three 16-row MFMA blocks (rows 0..47) + row
// 48 on the VALU from the weight fragments already in registers (a fourth MFMA block would be 15/16 padding:
// this removes 25% of the MFMAs). Attention computes S^T so that its accumulator registers are directly the B
// operand of O^T = V^T P^T (keys permuted consistently), so P never touches LDS; key 48 is a VALU rank-1 term.
#include "common.h"
#include <math.h>
#include <stdlib.h>

namespace ys {

constexpr int SW_ROWS = 49;  // token rows stored per window (7x7)
constexpr int XR = 48;       // the token row computed on the VALU (rows 0..47 = three 16-row MFMA blocks)
constexpr int HPW = 12;      // halo patch row stride in LDS (9 used; 16-byte aligned rows)

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
};

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float dot4_acc(float4 a, float4 b, float acc) {
  acc = fmaf(a.x, b.x, acc);
  acc = fmaf(a.y, b.y, acc);
  acc = fmaf(a.z, b.z, acc);
  return fmaf(a.w, b.w, acc);
}

// sum over the four lane groups g = lane >> 4 (lanes l, l^16, l^32, l^48)
__device__ __forceinline__ float group4_sum(float v) { return xor32_sum(xor16_sum(v)); }

// Weight fragments of one GEMM stage for this wave: column blocks cb = wid + 4*j, lane (g, l15) holds
// W[cb*16 + l15][g*K/4 .. (g+1)*K/4) as float4s. Loaded one stage ahead (issued before the previous stage's
// barrier) so the L2 latency overlaps that stage instead of stalling the first MFMAs.
template <int K, int NCB>
struct WFrag {
  float4 v[NCB / 4][K / 16];
};

template <int K, int NCB>
__device__ __forceinline__ void load_wfrag(const float* __restrict__ Wg, WFrag<K, NCB>& f, int tid) {
  const int lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, g = lane >> 4;
#pragma unroll
  for (int t = 0; t < K / 16; ++t)
#pragma unroll
    for (int j = 0; j < NCB / 4; ++j) {
      const float* wr = Wg + (long)((wid + 4 * j) * 16 + l15) * K + g * (K / 4);
      f.v[j][t] = *reinterpret_cast<const float4*>(wr + 4 * t);
    }
}

// Transposed output tiles: acc[rb][j] = (A[rows rb*16 .. +15][K] . W[n][K]^T)^T for this wave's column blocks
// cb = wid + 4*j (NCB % 4 == 0): the W fragment is the MFMA A operand and the token rows the B operand, so lane
// (g, l15) holds out[token rb*16 + l15][n = cb*16 + 4g .. +3] - four consecutive columns of one row, stored as one
// 16-byte LDS write (and residual-added with one 16-byte read) instead of four 4-byte ones. The accumulators start
// from the bias (the MFMA's C operand), so no epilogue add. ext[j] = the same for token row 48 on the VALU, column
// n = cb*16 + l15, without bias.
// The MFMA k index is permuted: lane group g owns k in [g*K/4, (g+1)*K/4), so A and W fragments are 16-byte loads;
// the row-48 dot products reuse the W fragments already in registers (partial over the lane's k quarter, then a
// cross-group sum), so the fourth 16-row block - 15 of its 16 rows padding - is never issued.
// A: LDS [SW_ROWS][lda]. W: the stage's prefetched fragments.
template <int K, int NCB>
__device__ __forceinline__ void wave_gemm_rows(const float* __restrict__ As, int lda, const WFrag<K, NCB>& wf,
                                               const f32x4 (&bias)[NCB / 4], f32x4 (&acc)[3][NCB / 4],
                                               float (&ext)[NCB / 4], int tid) {
  constexpr int NJ = NCB / 4;
  static_assert(NCB % 4 == 0, "column blocks must split evenly over the 4 waves");
  const int lane = tid & 63;
  const int l15 = lane & 15, g = lane >> 4;
  constexpr int KQ = K / 4;  // k range per lane group
  const auto& bw = wf.v;
  const float* arow[4];
#pragma unroll
  for (int rb = 0; rb < 4; ++rb) arow[rb] = As + (rb < 3 ? rb * 16 + l15 : XR) * lda + g * KQ;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    ext[j] = 0.f;
#pragma unroll
    for (int rb = 0; rb < 3; ++rb) acc[rb][j] = bias[j];
  }
#pragma unroll
  for (int t = 0; t < KQ / 4; ++t) {
    float4 a[4];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) a[rb] = *reinterpret_cast<const float4*>(arow[rb] + 4 * t);
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int rb = 0; rb < 3; ++rb)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const float av = c == 0 ? a[rb].x : c == 1 ? a[rb].y : c == 2 ? a[rb].z : a[rb].w;
          const float bv = c == 0 ? bw[j][t].x : c == 1 ? bw[j][t].y : c == 2 ? bw[j][t].z : bw[j][t].w;
          acc[rb][j] = mfma4(bv, av, acc[rb][j]);
        }
#pragma unroll
    for (int j = 0; j < NJ; ++j) ext[j] = dot4_acc(a[3], bw[j][t], ext[j]);
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) ext[j] = group4_sum(ext[j]);
}

// biases of this wave's column blocks: bias4[j] = b[cb*16 + 4g .. +3] (the transposed tiles' rows), b48[j] =
// b[cb*16 + l15] (token 48's column)
template <int NJ>
__device__ __forceinline__ void load_bias(const float* __restrict__ b, f32x4 (&bias4)[NJ], float (&b48)[NJ],
                                          int wid, int lane) {
  const int l15 = lane & 15, g = lane >> 4;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    bias4[j] = *reinterpret_cast<const f32x4*>(b + (wid + 4 * j) * 16 + 4 * g);
    b48[j] = b[(wid + 4 * j) * 16 + l15];
  }
}

// LayerNorm of rows [0, SW_ROWS) of S[SW_ROWS][lds] over C into U[SW_ROWS][ldu]: 4 threads per row (all rows at
// once), each holding C/4 values in registers from float4 LDS reads, two-pass statistics with DPP quad reductions,
// then U = (S - mean) * rstd * w + b written straight from those registers. Rows >= L (padding of a small global
// window) get U = b. The GEMMs read U as plain A fragments: the normalisation is done once per element instead of
// once per element per wave (all four waves read every A row).
template <int C>
__device__ __forceinline__ void lds_row_layernorm(const float* S, int lds, float* U, int ldu, const float* lnw,
                                                  const float* lnb, int L, float eps, int tid) {
  constexpr int CP = C / 4;
  const int r = tid >> 2, qd = tid & 3;
  const bool valid = r < L;
  float4 v[CP / 4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < CP / 4; ++i) {
    v[i] = valid ? *reinterpret_cast<const float4*>(S + r * lds + qd * CP + 4 * i) : make_float4(0.f, 0.f, 0.f, 0.f);
    s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  }
  const float mean = quad_sum(s) * (1.0f / (float)C);  // C is a power of two: exact
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < CP / 4; ++i) {  // centred values kept for the output pass
    v[i].x -= mean; v[i].y -= mean; v[i].z -= mean; v[i].w -= mean;
    q += (v[i].x * v[i].x + v[i].y * v[i].y) + (v[i].z * v[i].z + v[i].w * v[i].w);
  }
  const float var = quad_sum(q) * (1.0f / (float)C);
  const float rs = valid ? __builtin_amdgcn_rsqf(var + eps) : 0.f;  // v_rsq_f32 (1 ulp)
  if (r < SW_ROWS) {
#pragma unroll
    for (int i = 0; i < CP / 4; ++i) {
      const float4 w = *reinterpret_cast<const float4*>(lnw + qd * CP + 4 * i);
      const float4 b = *reinterpret_cast<const float4*>(lnb + qd * CP + 4 * i);
      float4 u;
      u.x = v[i].x * rs * w.x + b.x;
      u.y = v[i].y * rs * w.y + b.y;
      u.z = v[i].z * rs * w.z + b.z;
      u.w = v[i].w * rs * w.w + b.w;
      *reinterpret_cast<float4*>(U + r * ldu + qd * CP + 4 * i) = u;
    }
  }
}

// Workgroup i runs on XCD i % 8 and takes its window from that XCD's contiguous window range (neighbouring windows
// share 128-B lines of x and y - a window row is 28 B - so they meet in one L2).
template <int C, int NH, bool W7>
__global__ __launch_bounds__(256, 3) void swin_fused_kernel(SwinFusedArgs p) {
  constexpr int HD = C / NH;
  constexpr int HID = 2 * C;
  constexpr int LT = C + 4;          // T row stride (== 4 mod 64 floats: conflict-free b128 row reads)
  constexpr int LQ = 3 * C + 4;      // QKV row stride (also holds the attention output and the MLP hidden)
  constexpr int LH = HID + 4;
  constexpr int NHL = (C * 9 + 27) / 28;  // halo loads per lane: a wave-instruction covers 7 rows x 9 columns
  static_assert(HD % 16 == 0 && HD <= 64, "head dim");
  static_assert(LH <= LQ, "MLP hidden must fit the QKV region");
  static_assert(256 % C == 0 || C % 256 == 0, "depthwise channel mapping");
  static_assert(3 * ((C + 2) / 3) * 9 * HPW <= SW_ROWS * LQ, "halo patch must fit the QKV region");
  // T: residual stream; Q: x halo patch [C][PH][HPW] (stage 0) -> QKV (O overwrites each wave's own query
  // columns) -> MLP hidden; stats: per-row (mean, rstd); lnp: LN1/LN2 affine parameters
  // LN2 output U2 [SW_ROWS][LT] sits after the MLP hidden [SW_ROWS][LH] in the Q region (MLP1 reads U2 and
  // writes the hidden: disjoint); LN1 output U1 sits in the V columns of the QKV tile (QKV's epilogue waits)
  constexpr int QREG = (SW_ROWS * LQ > SW_ROWS * (LH + LT)) ? SW_ROWS * LQ : SW_ROWS * (LH + LT);
  __shared__ __attribute__((aligned(16))) float smem[SW_ROWS * LT + QREG + 4 * C];
  float* T = smem;
  float* Q = smem + SW_ROWS * LT;
  float* lnp = Q + QREG;  // [ln1_w | ln1_b | ln2_w | ln2_b]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l15 = lane & 15, g = lane >> 4;
  const int wh = W7 ? 7 : p.wh, ww = W7 ? 7 : p.ww, L = W7 ? 49 : p.L;
  const int H = p.H, W = p.W;
  const long HWl = (long)H * W;
  const int HWi = H * W;  // per-image offsets are 32-bit (launcher checks C*H*W < 2^30): cheap addressing
  const int PH = wh + 2, PW = ww + 2;

  const long nwin_total = (long)p.B * p.nWin;
  const long per_xcd = (nwin_total + 7) >> 3;
  const long xbeg = (long)(blockIdx.x & 7) * per_xcd;
  const long xend = (xbeg + per_xcd < nwin_total) ? xbeg + per_xcd : nwin_total;
  long gw = xbeg + (blockIdx.x >> 3);
  if (gw >= xend) return;

  // loop-invariant: LN parameters (LDS), depthwise taps of this thread's channel (registers)
  for (int e = tid; e < 4 * C; e += 256) {
    const int which = e / C, c = e - which * C;
    const float* src = which == 0 ? p.ln1_w : which == 1 ? p.ln1_b : which == 2 ? p.ln2_w : p.ln2_b;
    lnp[e] = src[c];
  }
  const int dw_c = tid % C;
  float dwk[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) dwk[i] = p.dw[dw_c * 9 + i];

  // halo patch [C][PH][PW] of window gwin into registers: lane = 9 * row + column (lane 63 idle), so one
  // wave-instruction reads 7 row segments of 9 floats (~14 cache lines) instead of 64 rows of one float each.
  // W7 (PH = 9): row slot s = 7*wid + row < 27 is (channel 3i + s/9, patch row s%9) at step i, so a lane's offset
  // is fixed across steps (the step advances the scalar soffset by 3 planes) and out-of-image lanes get an
  // out-of-range voffset that the buffer load returns as 0: no per-load VALU. Slot 27 idles.
  constexpr int NHS = (C + 2) / 3;                 // W7 steps (3 channels each)
  constexpr int NHV = NHS > NHL ? NHS : NHL;
  float hv[NHV];
  const int hl_r = lane / 9, hl_px = lane - (lane / 9) * 9;
  const int hslot = 7 * wid + hl_r;                 // W7 row slot (valid < 27)
  const int hcs = hslot / 9, hpy = hslot - (hslot / 9) * 9;
  constexpr unsigned OOB = 0x80000000u;             // > any image's byte size (< 2^32 with the largest soffset)
  auto load_halo = [&](long gwin) {
    const int gwi = __builtin_amdgcn_readfirstlane((int)gwin);  // window counts are < 2^31 (launcher)
    const int im = gwi / p.nWin, wn = gwi - (gwi / p.nWin) * p.nWin;
    const int wy_ = wn / p.nWx, wx_ = wn - (wn / p.nWx) * p.nWx;
    const int h0 = wy_ * wh - 1, w0 = wx_ * ww - 1;
    const float* xb_ = p.x + (long)im * C * HWl;
    const int wc = w0 + hl_px;
    const bool colok = hl_r < 7 && hl_px < PW && wc >= 0 && wc < W;
    if (W7) {
      // descriptor from provably wave-uniform words (otherwise every load becomes a readfirstlane waterfall)
      const unsigned long long xa = (unsigned long long)xb_;
      const unsigned long long xu = ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(xa >> 32)) << 32) |
                                    (unsigned)__builtin_amdgcn_readfirstlane((unsigned)xa);
      const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
          (void*)xu, (short)0, __builtin_amdgcn_readfirstlane(C * HWi * 4), 0x00020000);
      const int hh = h0 + hpy;
      const bool ok = colok && hslot < 27 && (unsigned)hh < (unsigned)H;
      const unsigned voff = ok ? (unsigned)((hcs * HWi + hh * W + wc) * 4) : OOB;
      const unsigned vlast = (3 * (NHS - 1) + hcs < C) ? voff : OOB;  // channel bound of the last step
#pragma unroll
      for (int i = 0; i < NHS; ++i)
        hv[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, i == NHS - 1 ? vlast : voff,
                                                                              i * 3 * HWi * 4, 0));
    } else {
#pragma unroll
      for (int i = 0; i < NHL; ++i) {
        const int rr = (i * 4 + wid) * 7 + hl_r;
        const int c = rr / PH, py = rr - c * PH;
        const int hh = h0 + py;
        const bool ok = colok && rr < C * PH && hh >= 0 && hh < H;
        const float v = xb_[ok ? c * HWi + hh * W + wc : 0];  // branch-free: out-of-window lanes read element 0
        hv[i] = ok ? v : 0.f;
      }
    }
  };
  load_halo(gw);

  for (;;) {
    const int gwc = __builtin_amdgcn_readfirstlane((int)gw);
    const int img = gwc / p.nWin, win = gwc - (gwc / p.nWin) * p.nWin;
    const int wy = win / p.nWx, wx = win - (win / p.nWx) * p.nWx;
    const float* xb = p.x + (long)img * C * HWl;
    // parameter pointers laundered per window: otherwise the compiler hoists every (loop-invariant) weight
    // fragment and bias load out of the window loop and spills them
    const float *w_in = p.win, *b_in = p.bin, *w_o = p.wo, *b_o = p.bo, *w_1 = p.w1, *b_1 = p.b1, *w_2 = p.w2,
                *b_2 = p.b2, *w_pw = p.wpw, *bn_sc = p.bn_scale, *bn_sh = p.bn_shift;
    // QKV weight fragments: in flight during the halo store, the depthwise conv and the LN1 statistics
    WFrag<C, 3 * C / 16> f_in;
    load_wfrag(w_in, f_in, tid);
    // each epilogue's biases are loaded with that stage's weight fragments: a bias load issued after the GEMM sat
    // behind nothing but still cost an exposed L2 round trip (s_waitcnt vmcnt(0)) per stage
    f32x4 bq[3 * C / 64];
    float bq48[3 * C / 64];
    load_bias(b_in, bq, bq48, wid, lane);

    // ---- stage 0: halo patch (registers) -> LDS [c][py][HPW] -> dw conv, one output row of 7 tokens per item ----
    if (W7) {
      if (hl_r < 7 && hslot < 27) {  // patch row 9*(3i + hcs) + hpy = 27i + hslot; rows of channels >= C are unused
#pragma unroll
        for (int i = 0; i < NHS; ++i) Q[(27 * i + hslot) * HPW + hl_px] = hv[i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < NHL; ++i) {
        const int rr = (i * 4 + wid) * 7 + hl_r;
        if (hl_r < 7 && rr < C * PH) Q[rr * HPW + hl_px] = hv[i];  // columns 9..11 of a row are never read
      }
    }
    __syncthreads();
    for (int item = tid; item < C * wh; item += 256) {
      const int iy = item / C;  // item % C == dw_c (256 % C == 0)
      const float* hp = Q + (dw_c * PH + iy) * HPW;
      float r[3][12];
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int q4 = 0; q4 < 3; ++q4) {
          const float4 v = *reinterpret_cast<const float4*>(hp + ky * HPW + 4 * q4);
          r[ky][4 * q4] = v.x; r[ky][4 * q4 + 1] = v.y; r[ky][4 * q4 + 2] = v.z; r[ky][4 * q4 + 3] = v.w;
        }
      const bool rowok = wy * wh + iy < H;
#pragma unroll
      for (int ix = 0; ix < 7; ++ix) {
        if (!W7 && ix >= ww) break;
        const float v = dwk[0] * r[0][ix] + dwk[1] * r[0][ix + 1] + dwk[2] * r[0][ix + 2] + dwk[3] * r[1][ix] +
                        dwk[4] * r[1][ix + 1] + dwk[5] * r[1][ix + 2] + dwk[6] * r[2][ix] + dwk[7] * r[2][ix + 1] +
                        dwk[8] * r[2][ix + 2];
        T[(iy * ww + ix) * LT + dw_c] = (rowok && wx * ww + ix < W) ? v : 0.f;
      }
    }
    if (!W7 && L < SW_ROWS)
      for (int e = tid; e < (SW_ROWS - L) * C; e += 256) T[(L + e / C) * LT + e % C] = 0.f;
    __syncthreads();

    // ---- stage 1: LN1 row statistics ----
    lds_row_layernorm<C>(T, LT, Q + 2 * C, LQ, lnp, lnp + C, L, p.ln1_eps, tid);
    __syncthreads();

    // ---- stage 2: QKV = LN1(T) Win^T + b_in ----
    {
      constexpr int NCB = 3 * C / 16;
      constexpr int NJ = NCB / 4;
      f32x4 acc[3][NJ];
      float ext[NJ];
      wave_gemm_rows<C, NCB>(Q + 2 * C, LQ, f_in, bq, acc, ext, tid);
      __syncthreads();  // every wave has read U1 (the V columns) before any wave writes V
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n4 = (wid + 4 * j) * 16 + 4 * g;
#pragma unroll
        for (int rb = 0; rb < 3; ++rb) *reinterpret_cast<f32x4*>(Q + (rb * 16 + l15) * LQ + n4) = acc[rb][j];
        if (g == 0) Q[XR * LQ + (wid + 4 * j) * 16 + l15] = ext[j] + bq48[j];
      }
    }
    WFrag<C, C / 16> f_o;  // out-proj weights: in flight during attention
    load_wfrag(w_o, f_o, tid);
    f32x4 bo_[C / 64];
    float bo48[C / 64];
    load_bias(b_o, bo_, bo48, wid, lane);
    __syncthreads();

    // ---- stage 3: attention, wave = query block (16 queries), all heads interleaved ----
    // Keys 0..47 on MFMA (S^T accumulators reused as the B operand of O^T = V^T P^T), key 48 on the VALU. The
    // output O[q][h*HD + d] overwrites the query columns of the wave's own rows (read only by this wave).
    {
      const int qb = wid;
      int qrow = qb * 16 + l15;
      qrow = qrow < XR ? qrow : XR;
      constexpr int DQ = HD / 4;  // d range per lane group
      f32x4 st[NH][3];
      float s48[NH];
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        s48[h] = 0.f;
#pragma unroll
        for (int kb = 0; kb < 3; ++kb) st[h][kb] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int t = 0; t < DQ / 4; ++t) {
        float4 qv[NH], kv[NH][3], k48[NH];
#pragma unroll
        for (int h = 0; h < NH; ++h) {
          qv[h] = *reinterpret_cast<const float4*>(Q + qrow * LQ + h * HD + g * DQ + 4 * t);
#pragma unroll
          for (int kb = 0; kb < 3; ++kb)
            kv[h][kb] = *reinterpret_cast<const float4*>(Q + (kb * 16 + l15) * LQ + C + h * HD + g * DQ + 4 * t);
          k48[h] = *reinterpret_cast<const float4*>(Q + XR * LQ + C + h * HD + g * DQ + 4 * t);
        }
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int h = 0; h < NH; ++h)
#pragma unroll
            for (int kb = 0; kb < 3; ++kb) {
              const float kk = c == 0 ? kv[h][kb].x : c == 1 ? kv[h][kb].y : c == 2 ? kv[h][kb].z : kv[h][kb].w;
              const float qq = c == 0 ? qv[h].x : c == 1 ? qv[h].y : c == 2 ? qv[h].z : qv[h].w;
              st[h][kb] = mfma4(kk, qq, st[h][kb]);
            }
#pragma unroll
        for (int h = 0; h < NH; ++h) s48[h] = dot4_acc(k48[h], qv[h], s48[h]);
      }
      // lane holds S^T[key = kb*16 + 4g + r][q = l15] per head (+ key 48 after the group sum): softmax over keys
      // on the raw scores (scale > 0 commutes with the max), exp2 with scale*log2(e) folded into one FMA; the
      // 1/sum normalisation is applied to O (per query = per lane) instead of to the 49 probabilities
      const float c2 = p.scale * 1.44269504088896341f;
      float p48[NH], inv[NH];
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        const bool k48ok = XR < L;
        const float sv48 = k48ok ? group4_sum(s48[h]) : -INFINITY;
        float mx = sv48;
#pragma unroll
        for (int kb = 0; kb < 3; ++kb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = kb * 16 + 4 * g + r;
            const float sv = (key < L) ? st[h][kb][r] : -INFINITY;
            st[h][kb][r] = sv;
            mx = fmaxf(mx, sv);
          }
        mx = xor32_max(xor16_max(mx));
        const float mc = -mx * c2;
        float sum = 0.f;
#pragma unroll
        for (int kb = 0; kb < 3; ++kb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float e = __builtin_amdgcn_exp2f(fmaf(st[h][kb][r], c2, mc));
            st[h][kb][r] = e;
            sum += e;
          }
        const float e48 = __builtin_amdgcn_exp2f(fmaf(sv48, c2, mc));
        sum += (g == 0) ? e48 : 0.f;
        inv[h] = __builtin_amdgcn_rcpf(group4_sum(sum));
        p48[h] = e48;
      }
      // O^T[d][q] = sum_key V[key][d] P[q][key]; MFMA (kb, r) consumes keys {kb*16 + 4g' + r}; key 48 rank-1 update
      f32x4 o[NH][HD / 16];
#pragma unroll
      for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int db = 0; db < HD / 16; ++db) o[h][db] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < 3; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float* vrow = Q + (kb * 16 + 4 * g + r) * LQ + 2 * C + l15;
#pragma unroll
          for (int h = 0; h < NH; ++h)
#pragma unroll
            for (int db = 0; db < HD / 16; ++db) o[h][db] = mfma4(vrow[h * HD + db * 16], st[h][kb][r], o[h][db]);
        }
#pragma unroll
      for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int db = 0; db < HD / 16; ++db) {
          const float4 v48 = *reinterpret_cast<const float4*>(Q + XR * LQ + 2 * C + h * HD + db * 16 + 4 * g);
          o[h][db][0] = fmaf(v48.x, p48[h], o[h][db][0]) * inv[h];
          o[h][db][1] = fmaf(v48.y, p48[h], o[h][db][1]) * inv[h];
          o[h][db][2] = fmaf(v48.z, p48[h], o[h][db][2]) * inv[h];
          o[h][db][3] = fmaf(v48.w, p48[h], o[h][db][3]) * inv[h];
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

    // ---- stage 4: T += O Wo^T + bo ----
    {
      constexpr int NCB = C / 16;
      constexpr int NJ = NCB / 4;
      f32x4 acc[3][NJ];
      float ext[NJ];
      wave_gemm_rows<C, C / 16>(Q, LQ, f_o, bo_, acc, ext, tid);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n4 = (wid + 4 * j) * 16 + 4 * g;
#pragma unroll
        for (int rb = 0; rb < 3; ++rb) {
          f32x4* tp = reinterpret_cast<f32x4*>(T + (rb * 16 + l15) * LT + n4);
          *tp = *tp + acc[rb][j];
        }
        if (g == 0 && XR < L) T[XR * LT + (wid + 4 * j) * 16 + l15] += ext[j] + bo48[j];
      }
    }
    WFrag<C, HID / 16> f_1;  // MLP1 weights: in flight during the LN2 statistics
    load_wfrag(w_1, f_1, tid);
    f32x4 b1_[HID / 64];
    float b1_48[HID / 64];
    load_bias(b_1, b1_, b1_48, wid, lane);
    __syncthreads();

    // ---- stage 5: LN2 row statistics ----
    lds_row_layernorm<C>(T, LT, Q + SW_ROWS * LH, LT, lnp + 2 * C, lnp + 3 * C, L, p.ln2_eps, tid);
    __syncthreads();

    // ---- stage 6: Hd = GELU(LN2(T) W1^T + b1) -> Q region [rows][LH] ----
    float* Hd = Q;
    {
      constexpr int NCB = HID / 16;
      constexpr int NJ = NCB / 4;
      f32x4 acc[3][NJ];
      float ext[NJ];
      wave_gemm_rows<C, HID / 16>(Q + SW_ROWS * LH, LT, f_1, b1_, acc, ext, tid);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n4 = (wid + 4 * j) * 16 + 4 * g;
#pragma unroll
        for (int rb = 0; rb < 3; ++rb) {
          const f32x2 lo = gelu2_fast_(f32x2{acc[rb][j][0], acc[rb][j][1]});
          const f32x2 hi = gelu2_fast_(f32x2{acc[rb][j][2], acc[rb][j][3]});
          *reinterpret_cast<f32x4*>(Hd + (rb * 16 + l15) * LH + n4) = f32x4{lo.x, lo.y, hi.x, hi.y};
        }
        if (g == 0) Hd[XR * LH + (wid + 4 * j) * 16 + l15] = gelu_fast_(ext[j] + b1_48[j]);
      }
    }
    WFrag<HID, C / 16> f_2;  // MLP2 weights
    load_wfrag(w_2, f_2, tid);
    f32x4 b2_[C / 64];
    float b2_48[C / 64];
    load_bias(b_2, b2_, b2_48, wid, lane);
    __syncthreads();

    // stage-8 residual x (L2-hot: this window's halo) and BN terms of this wave's first channel block, loaded
    // here so their latency overlaps MLP2. Residual loads and y stores are buffer ops on per-image descriptors:
    // a lane's voffset is fixed (its token, channel row 4g (+ l15 for token 48) of the wave's first block; out-of-
    // image tokens get an out-of-range voffset: loads return 0, stores are dropped) and the channel
    // ((cb - wid)*16 + r planes) goes into the scalar soffset.
    const int iy48 = XR / ww, ix48 = XR - (XR / ww) * ww;
    const int pix48 = (XR < L && wy * wh + iy48 < H && wx * ww + ix48 < W)
                          ? (wy * wh + iy48) * W + wx * ww + ix48 : -1;
    const unsigned long long ya = (unsigned long long)(p.y + (long)img * C * HWl);
    const unsigned long long xa8 = (unsigned long long)xb;
    const __amdgpu_buffer_rsrc_t rx8 = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(xa8 >> 32)) << 32) |
                (unsigned)__builtin_amdgcn_readfirstlane((unsigned)xa8)),
        (short)0, __builtin_amdgcn_readfirstlane(C * HWi * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t ry8 = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(ya >> 32)) << 32) |
                (unsigned)__builtin_amdgcn_readfirstlane((unsigned)ya)),
        (short)0, __builtin_amdgcn_readfirstlane(C * HWi * 4), 0x00020000);
    unsigned vtok[3];  // byte offset of (channel wid*16 + 4g, token tb*16 + l15), or OOB
#pragma unroll
    for (int tb = 0; tb < 3; ++tb) {
      const int tok = tb * 16 + l15;
      const int iy = tok / ww, ix = tok - iy * ww;
      const int hh = wy * wh + iy, wc = wx * ww + ix;
      const bool ok = tok < L && hh < H && wc < W;
      vtok[tb] = ok ? (unsigned)(((wid * 16 + 4 * g) * HWi + hh * W + wc) * 4) : OOB;
    }
    const unsigned v48 = (pix48 >= 0 && g == 0) ? (unsigned)(((wid * 16 + l15) * HWi + pix48) * 4) : OOB;
    float xr[3][4], x48, bsc[4], bsh[4], sc48, sh48;
    auto load_resid = [&](int cb) {
      const int sb = (cb - wid) * 16 * HWi * 4;
#pragma unroll
      for (int tb = 0; tb < 3; ++tb)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          xr[tb][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx8, vtok[tb],
                                                                                    sb + r * HWi * 4, 0));
      x48 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx8, v48, sb, 0));
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        bsc[r] = bn_sc[cb * 16 + 4 * g + r];
        bsh[r] = bn_sh[cb * 16 + 4 * g + r];
      }
      sc48 = bn_sc[cb * 16 + l15];
      sh48 = bn_sh[cb * 16 + l15];
    };
    load_resid(wid);

    // ---- stage 7: T += Hd W2^T + b2 ----
    {
      constexpr int NCB = C / 16;
      constexpr int NJ = NCB / 4;
      f32x4 acc[3][NJ];
      float ext[NJ];
      wave_gemm_rows<HID, C / 16>(Hd, LH, f_2, b2_, acc, ext, tid);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n4 = (wid + 4 * j) * 16 + 4 * g;
#pragma unroll
        for (int rb = 0; rb < 3; ++rb) {
          f32x4* tp = reinterpret_cast<f32x4*>(T + (rb * 16 + l15) * LT + n4);
          *tp = *tp + acc[rb][j];
        }
        if (g == 0 && XR < L) T[XR * LT + (wid + 4 * j) * 16 + l15] += ext[j] + b2_48[j];
      }
    }
    // pw weights of this wave's first output-channel block
    constexpr int CQ = C / 4;
    float4 wa[CQ / 4];
    {
      const float* wrow = w_pw + (long)(wid * 16 + l15) * C + g * CQ;
#pragma unroll
      for (int t = 0; t < CQ / 4; ++t) wa[t] = *reinterpret_cast<const float4*>(wrow + 4 * t);
    }
    __syncthreads();

    // next window's halo: in flight during the last stage

    // ---- stage 8: y = x + SiLU(BN(Wpw T^T)); output tile Y^T[c][tok] (lanes over tokens), token 48 on the VALU ----
    {
      constexpr int NCB = C / 16;
      for (int cb = wid; cb < NCB; cb += 4) {
        const float* wrow = w_pw + (long)(cb * 16 + l15) * C + g * CQ;
        if (cb != wid) load_resid(cb);
        f32x4 acc[3];
#pragma unroll
        for (int tb = 0; tb < 3; ++tb) acc[tb] = f32x4{0.f, 0.f, 0.f, 0.f};
        float e48 = 0.f;
        if (cb != wid) {
#pragma unroll
          for (int t = 0; t < CQ / 4; ++t) wa[t] = *reinterpret_cast<const float4*>(wrow + 4 * t);
        }
#pragma unroll
        for (int t = 0; t < CQ / 4; ++t) {
          float4 bt[3];
#pragma unroll
          for (int tb = 0; tb < 3; ++tb)
            bt[tb] = *reinterpret_cast<const float4*>(T + (tb * 16 + l15) * LT + g * CQ + 4 * t);
          const float4 t48 = *reinterpret_cast<const float4*>(T + XR * LT + g * CQ + 4 * t);
#pragma unroll
          for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int tb = 0; tb < 3; ++tb) {
              const float av = c == 0 ? wa[t].x : c == 1 ? wa[t].y : c == 2 ? wa[t].z : wa[t].w;
              const float bv = c == 0 ? bt[tb].x : c == 1 ? bt[tb].y : c == 2 ? bt[tb].z : bt[tb].w;
              acc[tb] = mfma4(av, bv, acc[tb]);
            }
          e48 = dot4_acc(wa[t], t48, e48);
        }
        e48 = group4_sum(e48);
        // lane holds Y^T[c = cb*16 + 4g + r][tok = tb*16 + l15]
        const int sb = (cb - wid) * 16 * HWi * 4;
#pragma unroll
        for (int tb = 0; tb < 3; ++tb)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            __builtin_amdgcn_raw_buffer_store_b32(
                __builtin_bit_cast(unsigned, xr[tb][r] + silu_fast_(acc[tb][r] * bsc[r] + bsh[r])), ry8, vtok[tb],
                sb + r * HWi * 4, 0);
        __builtin_amdgcn_raw_buffer_store_b32(
            __builtin_bit_cast(unsigned, x48 + silu_fast_(e48 * sc48 + sh48)), ry8, v48, sb, 0);
      }
    }
    break;  // one window per workgroup
  }
}

}  // namespace ys

using namespace ys;

// returns 1 if launched, 0 if the shape is not handled by the fused kernel, <0 on error
int yolosod_swin_fused_launch(const float* x, float* y, int B, int C, int H, int W, int num_heads, int wh, int ww,
                              int nWx, int nWin, const float* dw_w, const float* ln1_w, const float* ln1_b,
                              float ln1_eps, const float* in_proj_w, const float* in_proj_b, const float* out_proj_w,
                              const float* out_proj_b, const float* ln2_w, const float* ln2_b, float ln2_eps,
                              const float* mlp1_w, const float* mlp1_b, int mlp_hidden, const float* mlp2_w,
                              const float* mlp2_b, const float* pw_w, const float* bn_scale, const float* bn_shift,
                              hipStream_t st) {
  const int L = wh * ww;
  if (L > SW_ROWS || wh > 7 || ww > 7 || mlp_hidden != 2 * C) return 0;
  if ((long)C * H * W >= (1L << 30)) return 0;  // per-image byte offsets are 32-bit (buffer loads) in the kernel
  if ((long)B * nWin >= (1L << 31)) return 0;    // window indices are 32-bit
  SwinFusedArgs a{x, y, B, H, W, wh, ww, nWx, nWin, L, dw_w, ln1_w, ln1_b, ln1_eps, in_proj_w, in_proj_b,
                  out_proj_w, out_proj_b, ln2_w, ln2_b, ln2_eps, mlp1_w, mlp1_b, mlp2_w, mlp2_b, pw_w,
                  bn_scale, bn_shift, 1.0f / sqrtf((float)(C / num_heads))};
  const bool w7 = (wh == 7 && ww == 7);
  const long nwin = (long)B * nWin;
  auto grid_of = [&](long n) {
    const long cap = 8 * ((nwin + 7) / 8);
    if (n > cap) n = cap;
    return dim3((unsigned)(8 * ((n + 7) / 8)));
  };
#define YS_SWF(CC, NHH)                                                                                  \
  if (C == CC && num_heads == NHH) {                                                                     \
    if (w7) {                                                                                            \
      hipLaunchKernelGGL((swin_fused_kernel<CC, NHH, true>), grid_of(nwin), dim3(256), 0, st, a);        \
    } else {                                                                                             \
      hipLaunchKernelGGL((swin_fused_kernel<CC, NHH, false>), grid_of(nwin), dim3(256), 0, st, a);       \
    }                                                                                                    \
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
