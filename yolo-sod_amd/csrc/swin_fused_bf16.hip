// Fused SwinBlock for the bf16 config at C = 64 / 128 (the P2 instance L28: C = 128 at the m scale), 7x7 windows.
//
// One 256-thread workgroup processes one window; two workgroups per CU (LDS ~73 KB at C = 128). The window's tokens
// stay in LDS from the depthwise conv to the pw1x1 + BN + SiLU + residual store, so the per-window HBM traffic is
// the x halo read and the y write; the GEMM weights (bf16, 288 KB at C = 128) stream from L2.
//
// Stages (ultralytics/nn/modules/blocks_transformer.py), activations bf16 in LDS, fp32 accumulation:
//   0 dw3x3 (pad 1, no bias) on the 9x9 halo -> T[tok][c]; tokens of the bottom/right zero pad = 0  (:160, :31-46)
//   1 U = LN1(T)                                   (:112)
//   2 [Q | K] = U Win^T + b_in, V stored transposed (V^T[d][key])   (MHA in_proj, :116)
//   3 per head: S^T = K Q^T, softmax over keys (fp32, keys >= 49 masked), O^T = V^T P^T     (:116)
//   4 T += O Wo^T + bo                             (out_proj + residual, :119)
//   5 U = LN2(T); 6 H = GELU(U W1^T + b1); 7 T += H W2^T + b2        (:122)
//   8 y = x + SiLU(BN(Wpw T^T)) on the valid (cropped) tokens, NCHW  (window_reverse + crop :125-129, :166-171)
// MFMA: v_mfma_f32_16x16x32_bf16 (lane l: A[row l&15][k = 8(l>>4)+j], B[k = 8(l>>4)+j][col l&15], D[row 4(l>>4)+r]
// [col l&15]). GEMM tiles cover token rows 0..63 (four 16-row blocks; rows 49..63 are padding: their A rows read
// past the 49-row buffers into the next LDS region - finite values - and their outputs are never stored).
// Attention computes S^T so that its accumulators ARE the P^T operand of O^T = V^T P^T: for a 32-key step the B
// fragment element j is key 4g + j of the first 16-key block (j < 4) and 16 + 4g + (j - 4) of the second, and the
// V^T fragment is read in that key order (two 8-byte LDS reads). P is rounded to bf16 like the bf16 model's P.
#include "common.h"
#include <math.h>

namespace ys {

constexpr int SB_NR = 49;  // tokens per window

struct SwinBArgs {
  const bf16_t* x;
  bf16_t* y;
  int B, H, W, nWx, nWin;
  const float* dw;
  const float* ln1_w;
  const float* ln1_b;
  float ln1_eps;
  const bf16_t* win;
  const float* bin;
  const bf16_t* wo;
  const float* bo;
  const float* ln2_w;
  const float* ln2_b;
  float ln2_eps;
  const bf16_t* w1;
  const float* b1;
  const bf16_t* w2;
  const float* b2;
  const bf16_t* wpw;
  const float* bn_scale;
  const float* bn_shift;
  float scale;
};

// GELU(x) = 0.5 x (1 + erf(x / sqrt 2)) for bf16 outputs: erf by Abramowitz & Stegun 7.1.25 (|error| <= 2.5e-5,
// 100x below the 2^-8 relative rounding of the bf16 result), with x erf(x/sqrt2) = |x| erf(|x|/sqrt2) so no sign
// fix-up is needed: GELU = 0.5 (x + |x|) - 0.5 |x| poly(t) exp(-x^2/2), t = 1 / (1 + p |x| / sqrt2)
__device__ __forceinline__ f32x2 gelu2_bf16_(f32x2 x) {
  const f32x2 ax = {fabsf(x.x), fabsf(x.y)};
  const f32x2 den = __builtin_elementwise_fma(ax, f32x2{0.47047f * 0.70710678f, 0.47047f * 0.70710678f},
                                              f32x2{1.0f, 1.0f});
  const f32x2 t = {__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
  // 0.5 * (a1 t + a2 t^2 + a3 t^3)
  f32x2 poly = __builtin_elementwise_fma(t, f32x2{0.5f * 0.7478556f, 0.5f * 0.7478556f},
                                         f32x2{0.5f * -0.0958798f, 0.5f * -0.0958798f});
  poly = __builtin_elementwise_fma(t, poly, f32x2{0.5f * 0.3480242f, 0.5f * 0.3480242f});
  poly = poly * t;
  const f32x2 m = ax * (ax * -0.72134752044448170f);  // -x^2/2 log2(e)
  const f32x2 e = {__builtin_amdgcn_exp2f(m.x), __builtin_amdgcn_exp2f(m.y)};
  const f32x2 q = (ax * poly) * e;
  return __builtin_elementwise_fma(x + ax, f32x2{0.5f, 0.5f}, -q);
}

__device__ __forceinline__ f32x4 mfma_b(bf16x8_t a, bf16x8_t b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// weight fragments of W [N][K] for this wave's column blocks cb = wid + 4j: lane (g, l15) holds
// W[cb*16 + l15][32s + 8g .. +7] for every k-step s. W is the fragment-major copy swin_wfrag_kernel writes (the 64
// lanes' fragments of one (column block, k-step) are 1 KB contiguous, so a wave-instruction reads 8 whole cache
// lines; row-major it read 16 half lines, and the per-window weight stream L2 -> CU bounds the GEMM stages)
template <int K, int NJ>
struct BFrag {
  bf16x8_t v[NJ][K / 32];
};

template <int K, int NJ>
__device__ __forceinline__ void load_bfrag(const bf16_t* __restrict__ Wg, BFrag<K, NJ>& f, int wid, int lane) {
#pragma unroll
  for (int s = 0; s < K / 32; ++s)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      f.v[j][s] = *reinterpret_cast<const bf16x8_t*>(Wg + ((long)((wid + 4 * j) * (K / 32) + s) * 64 + lane) * 8);
}

// acc[rb][j] += A[rows rb*16 .. +15][0..K) . W^T for the wave's column blocks (A: LDS bf16, row stride lda; the
// caller initialises acc, e.g. with the bias). Blocks j < NTR are transposed tiles - the weight fragment is the MFMA
// A operand, so lane (g, l15) holds out[token rb*16 + l15][n = cb*16 + 4g .. +3]: four consecutive columns of one
// row, one 8-byte LDS store; blocks j >= NTR hold out[token rb*16 + 4g + r][n = cb*16 + l15] (four tokens of one
// column: the layout of V^T).
template <int K, int NJ, int NTR>
__device__ __forceinline__ void gemm_rows(const bf16_t* As, int lda, const BFrag<K, NJ>& f, f32x4 (&acc)[4][NJ],
                                          int lane) {
  const int l15 = lane & 15, g = lane >> 4;
#pragma unroll
  for (int s = 0; s < K / 32; ++s) {
    bf16x8_t a[4];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
      a[rb] = *reinterpret_cast<const bf16x8_t*>(As + (rb * 16 + l15) * lda + 32 * s + 8 * g);
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        acc[rb][j] = j < NTR ? mfma_b(f.v[j][s], a[rb], acc[rb][j]) : mfma_b(a[rb], f.v[j][s], acc[rb][j]);
  }
}

// 4 consecutive bf16 <-> fp32 (8 bytes)
__device__ __forceinline__ uint2 pack4(f32x4 v) { return make_uint2(pack_bf16x2(v.x, v.y), pack_bf16x2(v.z, v.w)); }
__device__ __forceinline__ f32x4 unpack4(uint2 u) {
  return f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
               __uint_as_float(u.y & 0xffff0000u)};
}

// LayerNorm of rows [0, 49) of S (bf16, stride ST) into U (bf16, stride ST): 4 lanes per row (a DPP quad), each
// holding C/4 values widened to fp32 from 16-byte reads; two-pass statistics; LN parameters from LDS
template <int C, int ST>
__device__ __forceinline__ void row_layernorm_b(const bf16_t* S, bf16_t* U, const float* __restrict__ lnw,
                                                const float* __restrict__ lnb, float eps, int tid) {
  constexpr int CP = C / 4;  // elements per lane (16 or 32)
  const int r = tid >> 2, qd = tid & 3;
  const bool valid = r < SB_NR;
  float v[CP];
#pragma unroll
  for (int i = 0; i < CP / 8; ++i) {
    uint4 u = make_uint4(0u, 0u, 0u, 0u);
    if (valid) u = *reinterpret_cast<const uint4*>(S + r * ST + qd * CP + 8 * i);
    float f[8];
    unpack8(u, f);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[8 * i + k] = f[k];
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < CP; ++i) s += v[i];
  const float mean = quad_sum(s) * (1.0f / (float)C);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < CP; ++i) {
    v[i] -= mean;
    q += v[i] * v[i];
  }
  const float rs = __builtin_amdgcn_rsqf(quad_sum(q) * (1.0f / (float)C) + eps);
  if (!valid) return;
#pragma unroll
  for (int i = 0; i < CP / 8; ++i) {
    float f[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = qd * CP + 8 * i + k;
      f[k] = v[8 * i + k] * rs * lnw[c] + lnb[c];
    }
    *reinterpret_cast<uint4*>(U + r * ST + qd * CP + 8 * i) = pack8(f);
  }
}

template <int C, int NH>
__global__ __launch_bounds__(256, 2) void swin_fused_bf16_kernel(SwinBArgs p) {
  constexpr int HD = C / NH;
  constexpr int HID = 2 * C;
  constexpr int ST = C + 8;        // T / U / O row stride (elements)
  constexpr int SQK = 2 * C + 8;   // [Q | K] row stride; the MLP hidden reuses the region (HID == 2C)
  constexpr int SVT = 72;          // V^T row stride: keys 0..63 (+8)
  static_assert(HD == 32 || HD == 64, "head dim");
  static_assert(C == 64 || C == 128, "channels");
  constexpr int T_OFF = 0;
  constexpr int U_OFF = T_OFF + SB_NR * ST;
  constexpr int QK_OFF = U_OFF + SB_NR * ST;
  constexpr int VT_OFF = QK_OFF + SB_NR * SQK;
  constexpr int END = VT_OFF + C * SVT;
  static_assert(2 * C * 81 <= END - QK_OFF, "fp32 halo patch must fit the QKV region");
  static_assert(15 * SQK <= C * SVT, "padding-row reads of the QKV region stay inside V^T");
  // fp32 parameters staged once per workgroup: every epilogue reads LDS, so no global load sits behind a weight
  // prefetch in the in-order vmcnt queue (a bias load after a prefetch made each stage wait for the next stage's
  // weights)
  constexpr int P_BIN = 0, P_BO = 3 * C, P_B1 = 4 * C, P_B2 = 6 * C, P_SC = 7 * C, P_SH = 8 * C, P_L1W = 9 * C,
                P_L1B = 10 * C, P_L2W = 11 * C, P_L2B = 12 * C, NPAR = 13 * C;
  __shared__ __attribute__((aligned(16))) bf16_t sm[END];
  __shared__ __attribute__((aligned(16))) float par[NPAR];
  bf16_t* T = sm + T_OFF;
  bf16_t* U = sm + U_OFF;
  bf16_t* QK = sm + QK_OFF;
  bf16_t* Vt = sm + VT_OFF;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l15 = lane & 15, g = lane >> 4;
  const int H = p.H, W = p.W;
  const long HW = (long)H * W;
  // XCD-aware window order: workgroup i runs on XCD i % 8 and takes windows from that XCD's contiguous range, so
  // horizontally adjacent windows (whose 7-pixel rows share 128-byte lines of x and y) meet in one L2
  const long nwin_total = (long)p.B * p.nWin;
  const long per_xcd = (nwin_total + 7) >> 3;
  const long gw = (long)(blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  if (gw >= nwin_total || (blockIdx.x >> 3) >= per_xcd) return;
  const int img = (int)(gw / p.nWin), win = (int)(gw - (long)img * p.nWin);
  const int wy = win / p.nWx, wx = win - (win / p.nWx) * p.nWx;
  const bf16_t* xb = p.x + (long)img * C * HW;

  // halo -> registers first, then the parameters (their LDS stores wait for the halo too: one latency, not two),
  // the depthwise taps and the QKV weight prefetch (last in the vmcnt queue, so the halo wait does not wait for it).
  // halo [C][9][9] -> LDS fp32 [c][py][px] (stride 81 per channel). Two load layouts (uniform branch on W):
  //  * W % 8 == 0: 16-byte loads of 8-pixel-aligned chunks - two per (channel, patch row) cover the 9 columns at the
  //    window's offset within the first chunk (9C/128 loads per lane instead of C/3 two-byte loads); chunks outside
  //    the image (rows, or the chunk left of column 0 / right of W) get an out-of-range offset and load zeros;
  //  * otherwise: row slot s = 7*wid + lane/9 < 27 covers (channel 3i + s/9, patch row s%9) at step i, lane%9 the
  //    column, so a lane's byte offset is fixed across the C/3 steps (the step advances the scalar offset by 3
  //    planes) and out-of-image lanes get an out-of-range offset that the buffer load returns as 0.
  float* halo = reinterpret_cast<float*>(sm + QK_OFF);
  const unsigned long long xa = (unsigned long long)xb;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(xa >> 32)) << 32) |
              (unsigned)__builtin_amdgcn_readfirstlane((unsigned)xa)),
      (short)0, __builtin_amdgcn_readfirstlane((int)(C * HW * 2)), 0x00020000);
  const bool chunked = (W & 7) == 0;
  constexpr int NPAIR = 9 * C;                 // (channel, patch row) pairs
  constexpr int NST = (NPAIR + 127) / 128;      // 128 pairs (256 lanes, 2 chunks each) per step
  constexpr int NHS = (C + 2) / 3;
  const int hq = tid >> 1, hch = tid & 1;
  const int s0 = wx * 7 - 1, a0 = s0 & ~7, hoff = s0 - a0;  // first halo column, its 8-px chunk, offset in it
  uint4 hc[NST];
  float hv[NHS];
  const int hl_r = lane / 9, hl_px = lane - (lane / 9) * 9;
  const int hslot = 7 * wid + hl_r;  // valid < 27 (lane 63 and slot 27 idle)
  const int hcs = hslot / 9, hpy = hslot - (hslot / 9) * 9;
  if (chunked) {
    const int col = a0 + 8 * hch;
    const bool colok = col >= 0 && col + 8 <= W;
#pragma unroll
    for (int st = 0; st < NST; ++st) {
      const int pr = st * 128 + hq;
      const int c = pr / 9, py = pr - (pr / 9) * 9;
      const int hh = wy * 7 - 1 + py;
      const bool ok = pr < NPAIR && colok && (unsigned)hh < (unsigned)H;
      const unsigned v = ok ? (unsigned)(((long)c * HW + (long)hh * W + col) * 2) : 0x80000000u;
      const auto r = __builtin_amdgcn_raw_buffer_load_b128(rx, v, 0, 0);
      hc[st] = make_uint4(r[0], r[1], r[2], r[3]);
    }
  } else {
    const int hh = wy * 7 - 1 + hpy, wc = wx * 7 - 1 + hl_px;
    const bool ok = hl_r < 7 && hslot < 27 && (unsigned)hh < (unsigned)H && (unsigned)wc < (unsigned)W;
    const unsigned voff = ok ? (unsigned)((hcs * HW + (long)hh * W + wc) * 2) : 0x80000000u;
#pragma unroll
    for (int i = 0; i < NHS; ++i) {
      const unsigned v = (3 * i + hcs < C) ? voff : 0x80000000u;
      hv[i] = bf2f(__builtin_amdgcn_raw_buffer_load_b16(rx, v, (int)(i * 3 * HW * 2), 0));
    }
  }
  // parameters -> LDS (every load first, then the stores), depthwise taps -> registers
  {
    constexpr int NPT = (NPAR + 255) / 256;
    float pv[NPT];
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int e = tid + 256 * i;
      const int w = e / C, c = e - w * C;
      const float* src = w < 3 ? p.bin + w * C : w == 3 ? p.bo : w < 6 ? p.b1 + (w - 4) * C : w == 6 ? p.b2
                       : w == 7 ? p.bn_scale : w == 8 ? p.bn_shift : w == 9 ? p.ln1_w : w == 10 ? p.ln1_b
                       : w == 11 ? p.ln2_w : p.ln2_b;
      pv[i] = e < NPAR ? src[c] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < NPT; ++i)
      if (tid + 256 * i < NPAR) par[tid + 256 * i] = pv[i];
  }
  const int dc = tid % C;
  float k[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) k[i] = p.dw[dc * 9 + i];
  constexpr int NJ_QKV = 3 * C / 64;
  BFrag<C, NJ_QKV> f_qkv;
  load_bfrag(p.win, f_qkv, wid, lane);

  // ---- stage 0: halo -> LDS (fp32: conflict-free stride-81 reads below), depthwise conv -> T ----
  if (chunked) {
    // lane (pair, chunk) holds columns 8*chunk .. +7 of the 16 from a0: halo column j = 8*chunk + e - hoff
#pragma unroll
    for (int st = 0; st < NST; ++st) {
      const int pr = st * 128 + hq;
      float f[8];
      unpack8(hc[st], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int j = 8 * hch + e - hoff;
        if (pr < NPAIR && j >= 0 && j < 9) halo[pr * 9 + j] = f[e];
      }
    }
  } else if (hl_r < 7 && hslot < 27) {
#pragma unroll
    for (int i = 0; i < NHS; ++i)
      if (3 * i + hcs < C) halo[(3 * i + hcs) * 81 + hpy * 9 + hl_px] = hv[i];
  }
  __syncthreads();
  {
    const int c = dc;
    for (int iy = tid / C; iy < 7; iy += 256 / C) {
      const float* hp = halo + c * 81 + iy * 9;
      float r[3][9];
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 9; ++kx) r[ky][kx] = hp[ky * 9 + kx];
      const bool rowok = wy * 7 + iy < H;
#pragma unroll
      for (int ix = 0; ix < 7; ++ix) {
        float v = 0.f;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) v = fmaf(k[ky * 3 + kx], r[ky][ix + kx], v);
        T[(iy * 7 + ix) * ST + c] = (rowok && wx * 7 + ix < W) ? f2bf(v) : (bf16_t)0;
      }
    }
  }
  __syncthreads();

  // ---- stage 1: U = LN1(T) ----
  row_layernorm_b<C, ST>(T, U, par + P_L1W, par + P_L1B, p.ln1_eps, tid);
  __syncthreads();

  // ---- stage 2: [Q | K] = U Win^T + b (rows < 49), V^T[d][key] (keys >= 49 zero) ----
  constexpr int NJ_O = C / 64;
  BFrag<C, NJ_O> f_o;  // out-proj weights: in flight during the QKV epilogue and attention
  {
    constexpr int NTR = 2 * C / 64;  // Q | K column blocks: transposed tiles; V blocks: V^T layout
    f32x4 acc[4][NJ_QKV];
#pragma unroll
    for (int j = 0; j < NJ_QKV; ++j) {
      const f32x4 b = j < NTR ? *reinterpret_cast<const f32x4*>(par + P_BIN + (wid + 4 * j) * 16 + 4 * g)
                              : f32x4{1.f, 1.f, 1.f, 1.f} * par[P_BIN + (wid + 4 * j) * 16 + l15];
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) acc[rb][j] = b;
    }
    gemm_rows<C, NJ_QKV, NTR>(U, ST, f_qkv, acc, lane);
    load_bfrag(p.wo, f_o, wid, lane);
#pragma unroll
    for (int j = 0; j < NJ_QKV; ++j) {
      if (j < NTR) {
        const int n4 = (wid + 4 * j) * 16 + 4 * g;
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          const int row = rb * 16 + l15;
          if (row < SB_NR) *reinterpret_cast<uint2*>(QK + row * SQK + n4) = pack4(acc[rb][j]);
        }
      } else {
        const int d = (wid + 4 * j) * 16 + l15 - 2 * C;
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          const int row0 = rb * 16 + 4 * g;
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (row0 + r < SB_NR) ? acc[rb][j][r] : 0.f;
          *reinterpret_cast<uint2*>(Vt + d * SVT + row0) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
        }
      }
    }
  }
  __syncthreads();

  // ---- stage 3: attention; wave = 16 queries (rows wid*16 + l15), all heads; O -> U region ----
  {
    const int q0 = wid * 16;
    const int qr = (q0 + l15 < SB_NR) ? q0 + l15 : SB_NR - 1;  // padding queries read a real row (dropped)
    const float c2 = p.scale * 1.44269504088896341f;
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      // S^T[key][q] = sum_d K[key][d] Q[q][d]; key blocks of 16
      bf16x8_t qf[HD / 32];
#pragma unroll
      for (int s = 0; s < HD / 32; ++s)
        qf[s] = *reinterpret_cast<const bf16x8_t*>(QK + qr * SQK + h * HD + 32 * s + 8 * g);
      f32x4 st[4];
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        st[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int key = (kb * 16 + l15 < SB_NR) ? kb * 16 + l15 : SB_NR - 1;
#pragma unroll
        for (int s = 0; s < HD / 32; ++s)
          st[kb] = mfma_b(*reinterpret_cast<const bf16x8_t*>(QK + key * SQK + C + h * HD + 32 * s + 8 * g), qf[s],
                          st[kb]);
      }
      // lane holds S^T[key = kb*16 + 4g + r][q = l15]: softmax over keys (in lane, then over the 4 lane groups)
      float mx = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (kb * 16 + 4 * g + r >= SB_NR) st[kb][r] = -INFINITY;
          mx = fmaxf(mx, st[kb][r]);
        }
      mx = xor32_max(xor16_max(mx));
      const float mc = -mx * c2;
      float sum = 0.f;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __builtin_amdgcn_exp2f(fmaf(st[kb][r], c2, mc));
          st[kb][r] = e;
          sum += e;
        }
      const float inv = __builtin_amdgcn_rcpf(xor32_sum(xor16_sum(sum)));
      // P^T fragments: k-step s (keys 32s..32s+31): element j = key 32s + 4g + j (j < 4), 32s + 16 + 4g + j - 4
      bf16x8_t pf[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const uint32_t w0 = pack_bf16x2(st[2 * s][0] * inv, st[2 * s][1] * inv);
        const uint32_t w1 = pack_bf16x2(st[2 * s][2] * inv, st[2 * s][3] * inv);
        const uint32_t w2 = pack_bf16x2(st[2 * s + 1][0] * inv, st[2 * s + 1][1] * inv);
        const uint32_t w3 = pack_bf16x2(st[2 * s + 1][2] * inv, st[2 * s + 1][3] * inv);
        pf[s] = __builtin_bit_cast(bf16x8_t, make_uint4(w0, w1, w2, w3));
      }
      // O^T[d][q] = sum_key V^T[d][key] P^T[key][q]
#pragma unroll
      for (int db = 0; db < HD / 16; ++db) {
        f32x4 o = {0.f, 0.f, 0.f, 0.f};
        const bf16_t* vr = Vt + (h * HD + db * 16 + l15) * SVT + 4 * g;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const uint2 lo = *reinterpret_cast<const uint2*>(vr + 32 * s);
          const uint2 hi = *reinterpret_cast<const uint2*>(vr + 32 * s + 16);
          o = mfma_b(__builtin_bit_cast(bf16x8_t, make_uint4(lo.x, lo.y, hi.x, hi.y)), pf[s], o);
        }
        // lane holds O^T[d = db*16 + 4g + r][q = l15] -> O[q][h*HD + d .. +3]
        if (q0 + l15 < SB_NR)
          *reinterpret_cast<uint2*>(U + (q0 + l15) * ST + h * HD + db * 16 + 4 * g) =
              make_uint2(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]));
      }
    }
  }
  __syncthreads();

  // ---- stage 4: T += O Wo^T + bo ----
  constexpr int NJ_1 = HID / 64;
  BFrag<C, NJ_1> f_1;  // MLP1 weights: in flight during out-proj and LN2
  load_bfrag(p.w1, f_1, wid, lane);
  {
    f32x4 acc[4][NJ_O];
#pragma unroll
    for (int j = 0; j < NJ_O; ++j) {
      const f32x4 b = *reinterpret_cast<const f32x4*>(par + P_BO + (wid + 4 * j) * 16 + 4 * g);
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) acc[rb][j] = b;
    }
    gemm_rows<C, NJ_O, NJ_O>(U, ST, f_o, acc, lane);
#pragma unroll
    for (int j = 0; j < NJ_O; ++j) {
      const int n4 = (wid + 4 * j) * 16 + 4 * g;
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        const int row = rb * 16 + l15;
        if (row < SB_NR) {
          uint2* tp = reinterpret_cast<uint2*>(T + row * ST + n4);
          *tp = pack4(unpack4(*tp) + acc[rb][j]);
        }
      }
    }
  }
  __syncthreads();

  // ---- stage 5: U = LN2(T) ----
  row_layernorm_b<C, ST>(T, U, par + P_L2W, par + P_L2B, p.ln2_eps, tid);
  __syncthreads();

  // ---- stage 6: H = GELU(U W1^T + b1) -> QK region ----
  bf16_t* Hd = QK;
  constexpr int NJ_2 = C / 64;
  BFrag<HID, NJ_2> f_2;  // MLP2 weights
  load_bfrag(p.w2, f_2, wid, lane);
  {
    f32x4 acc[4][NJ_1];
#pragma unroll
    for (int j = 0; j < NJ_1; ++j) {
      const f32x4 b = *reinterpret_cast<const f32x4*>(par + P_B1 + (wid + 4 * j) * 16 + 4 * g);
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) acc[rb][j] = b;
    }
    gemm_rows<C, NJ_1, NJ_1>(U, ST, f_1, acc, lane);
#pragma unroll
    for (int j = 0; j < NJ_1; ++j) {
      const int n4 = (wid + 4 * j) * 16 + 4 * g;
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        const int row = rb * 16 + l15;
        const f32x2 lo = gelu2_bf16_(f32x2{acc[rb][j][0], acc[rb][j][1]});
        const f32x2 hi = gelu2_bf16_(f32x2{acc[rb][j][2], acc[rb][j][3]});
        if (row < SB_NR)
          *reinterpret_cast<uint2*>(Hd + row * SQK + n4) = make_uint2(pack_bf16x2(lo.x, lo.y), pack_bf16x2(hi.x, hi.y));
      }
    }
  }
  __syncthreads();

  // ---- stage 7: T += H W2^T + b2; the pw weights and this lane's residual pixels are loaded first (in flight
  // during MLP2) ----
  constexpr int NCB_PW = C / 64;  // output-channel blocks per wave
  bf16x8_t wa[NCB_PW][C / 32];
#pragma unroll
  for (int j = 0; j < NCB_PW; ++j)
#pragma unroll
    for (int s = 0; s < C / 32; ++s)
      wa[j][s] = *reinterpret_cast<const bf16x8_t*>(p.wpw + ((long)((wid + 4 * j) * (C / 32) + s) * 64 + lane) * 8);
  // residual x and the y stores: buffer ops on per-image descriptors; a lane's voffset is fixed (channel row 4g of
  // block wid, its token) and out-of-window / cropped tokens get an out-of-range voffset (loads return 0, stores are
  // dropped), so there is no per-element branch (a branch per load serialised them behind s_waitcnt vmcnt(0))
  constexpr unsigned OOB = 0x80000000u;
  const int HWi = (int)HW;
  auto rsrc_of = [&](const bf16_t* base) {
    const unsigned long long a = (unsigned long long)base;
    return __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(a >> 32)) << 32) |
                (unsigned)__builtin_amdgcn_readfirstlane((unsigned)a)),
        (short)0, __builtin_amdgcn_readfirstlane(C * HWi * 2), 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rxr = rsrc_of(xb);
  unsigned vtok[4];
#pragma unroll
  for (int tb = 0; tb < 4; ++tb) {
    const int tok = tb * 16 + l15;
    const int iy = tok / 7, ix = tok - (tok / 7) * 7;
    const int hh = wy * 7 + iy, ww = wx * 7 + ix;
    vtok[tb] = (tok < SB_NR && hh < H && ww < W) ? (unsigned)(((wid * 16 + 4 * g) * HWi + hh * W + ww) * 2) : OOB;
  }
  bf16_t xres[NCB_PW][4][4];
#pragma unroll
  for (int j = 0; j < NCB_PW; ++j)
#pragma unroll
    for (int tb = 0; tb < 4; ++tb)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        xres[j][tb][r] = __builtin_amdgcn_raw_buffer_load_b16(rxr, vtok[tb], (64 * j + r) * HWi * 2, 0);
  {
    f32x4 acc[4][NJ_2];
#pragma unroll
    for (int j = 0; j < NJ_2; ++j) {
      const f32x4 b = *reinterpret_cast<const f32x4*>(par + P_B2 + (wid + 4 * j) * 16 + 4 * g);
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) acc[rb][j] = b;
    }
    gemm_rows<HID, NJ_2, NJ_2>(Hd, SQK, f_2, acc, lane);
#pragma unroll
    for (int j = 0; j < NJ_2; ++j) {
      const int n4 = (wid + 4 * j) * 16 + 4 * g;
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        const int row = rb * 16 + l15;
        if (row < SB_NR) {
          uint2* tp = reinterpret_cast<uint2*>(T + row * ST + n4);
          *tp = pack4(unpack4(*tp) + acc[rb][j]);
        }
      }
    }
  }
  __syncthreads();

  // ---- stage 8: Y^T[c][tok] = Wpw . T^T; y = x + SiLU(BN(Y)) at the window's valid pixels ----
  {
    const __amdgpu_buffer_rsrc_t ryr = rsrc_of(p.y + (long)img * C * HW);
#pragma unroll
    for (int j = 0; j < NCB_PW; ++j) {
      const int cb = wid + 4 * j;
      f32x4 acc[4];
#pragma unroll
      for (int tb = 0; tb < 4; ++tb) acc[tb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < C / 32; ++s)
#pragma unroll
        for (int tb = 0; tb < 4; ++tb)
          acc[tb] = mfma_b(wa[j][s], *reinterpret_cast<const bf16x8_t*>(T + (tb * 16 + l15) * ST + 32 * s + 8 * g),
                           acc[tb]);
      // lane holds Y^T[c = cb*16 + 4g + r][tok = tb*16 + l15]
#pragma unroll
      for (int tb = 0; tb < 4; ++tb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = cb * 16 + 4 * g + r;
          __builtin_amdgcn_raw_buffer_store_b16(
              f2bf(bf2f(xres[j][tb][r]) + silu_fast_(acc[tb][r] * par[P_SC + c] + par[P_SH + c])), ryr, vtok[tb],
              (64 * j + r) * HWi * 2, 0);
        }
    }
  }
}

// fragment-major copies of the five weight matrices: thread = one 8-element run W[n][k..k+7] (16 B in, 16 B out);
// element (n, k) of W [N][K] lands at ((n/16 * K/32 + k/32) * 64 + (k%32)/8 * 16 + n%16) * 8 + k%8
struct WFragArgs {
  const bf16_t* src[5];
  bf16_t* dst[5];
  int N[5], K[5];
  long end[5];  // cumulative 8-element run counts
};

__global__ void __launch_bounds__(256) swin_wfrag_kernel(WFragArgs a) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.end[4]) return;
  int m = 0;
#pragma unroll
  for (int t = 0; t < 4; ++t) m += (i >= a.end[t]) ? 1 : 0;
  const long r = i - (m ? a.end[m - 1] : 0);
  const int K = a.K[m], k8 = K / 8;
  const int n = (int)(r / k8), k = (int)(r % k8) * 8;
  const bf16x8_t v = *reinterpret_cast<const bf16x8_t*>(a.src[m] + (long)n * K + k);
  const long o = ((long)((n >> 4) * (K / 32) + (k >> 5)) * 64 + ((k & 31) >> 3) * 16 + (n & 15)) * 8;
  *reinterpret_cast<bf16x8_t*>(a.dst[m] + o) = v;
}

}  // namespace ys

using namespace ys;

size_t yolosod_swin_fused_bf16_wfrag_elems(int C, int mlp_hidden) {
  return (size_t)5 * C * C + (size_t)2 * C * mlp_hidden;
}

// shapes the fused bf16 kernel takes: 7x7 windows, C 64 (2 heads) / 128 (2 or 4 heads), MLP hidden 2C
bool yolosod_swin_fused_bf16_ok(int C, int num_heads, int wh, int ww, int mlp_hidden) {
  return wh == 7 && ww == 7 && mlp_hidden == 2 * C &&
         ((C == 128 && (num_heads == 2 || num_heads == 4)) || (C == 64 && num_heads == 2));
}

// returns 1 if launched, 0 if the shape is not handled (decomposed path), < 0 on error
int yolosod_swin_fused_bf16_launch(const bf16_t* x, bf16_t* y, int B, int C, int H, int W, int num_heads, int wh,
                                   int ww, int nWx, int nWin, const float* dw_w, const float* ln1_w, const float* ln1_b,
                                   float ln1_eps, const bf16_t* in_proj_w, const float* in_proj_b,
                                   const bf16_t* out_proj_w, const float* out_proj_b, const float* ln2_w,
                                   const float* ln2_b, float ln2_eps, const bf16_t* mlp1_w, const float* mlp1_b,
                                   int mlp_hidden, const bf16_t* mlp2_w, const float* mlp2_b, const bf16_t* pw_w,
                                   const float* bn_scale, const float* bn_shift, bf16_t* wfrag, hipStream_t st) {
  if (!yolosod_swin_fused_bf16_ok(C, num_heads, wh, ww, mlp_hidden) || (long)B * nWin >= (1L << 31)) return 0;
  // weight planes in fragment-major order (wfrag: yolosod_swin_fused_bf16_wfrag_elems(C, hid) bf16)
  const int hid = mlp_hidden;
  WFragArgs fa{};
  const bf16_t* srcs[5] = {in_proj_w, out_proj_w, mlp1_w, mlp2_w, pw_w};
  const int Ns[5] = {3 * C, C, hid, C, C}, Ks[5] = {C, C, C, hid, C};
  long run = 0, off = 0;
  for (int t = 0; t < 5; ++t) {
    fa.src[t] = srcs[t];
    fa.dst[t] = wfrag + off;
    fa.N[t] = Ns[t];
    fa.K[t] = Ks[t];
    run += (long)Ns[t] * Ks[t] / 8;
    fa.end[t] = run;
    off += (long)Ns[t] * Ks[t];
  }
  hipLaunchKernelGGL(swin_wfrag_kernel, dim3((unsigned)((run + 255) / 256)), dim3(256), 0, st, fa);
  SwinBArgs a{x, y, B, H, W, nWx, nWin, dw_w, ln1_w, ln1_b, ln1_eps, fa.dst[0], in_proj_b, fa.dst[1], out_proj_b,
              ln2_w, ln2_b, ln2_eps, fa.dst[2], mlp1_b, fa.dst[3], mlp2_b, fa.dst[4], bn_scale, bn_shift,
              1.0f / sqrtf((float)(C / num_heads))};
  const long nwin = (long)B * nWin;
  const dim3 grid((unsigned)(8 * ((nwin + 7) / 8)));
  if (C == 128 && num_heads == 2) hipLaunchKernelGGL((swin_fused_bf16_kernel<128, 2>), grid, dim3(256), 0, st, a);
  else if (C == 128 && num_heads == 4) hipLaunchKernelGGL((swin_fused_bf16_kernel<128, 4>), grid, dim3(256), 0, st, a);
  else if (C == 64 && num_heads == 2) hipLaunchKernelGGL((swin_fused_bf16_kernel<64, 2>), grid, dim3(256), 0, st, a);
  else return 0;
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("swin_fused_bf16: launch failed: %s", hipGetErrorString(e));
    return -1;
  }
  return 1;
}
