// Fused SwinBlock for C = 64 (the P2 instance L28 of the paper model) with the projection / MLP / pw GEMMs on the
// bf16 matrix cores at fp32 accuracy.
//
// Why: on gfx950 the fp32 MFMA (v_mfma_f32_16x16x4_f32, 157 TF/s) shares the SIMD with the VALU - they never
// co-execute - and the fused fp32 kernel (swin_fused.hip) spends ~58 % of its cycles in it. The bf16 MFMA runs 16x
// faster per instruction-cycle and beside other waves' VALU. An fp32 operand splits exactly enough into three bf16
// terms, v = h + m + l (h = bf16(v), m = bf16(v - h), l = bf16(v - h - m), round-to-nearest-even: |v - h - m - l| <=
// 2^-27 |v|, below fp32's own 2^-24), and a product into the six terms of order >= 2^-16,
//   a.b ~ ah.bh + ah.bm + am.bh + ah.bl + am.bm + al.bh     (dropped: am.bl, al.bm, al.bl <= ~2^-26 |a.b|),
// each an exact bf16 x bf16 product accumulated in fp32 by the MFMA - the same accumulation as the fp32 MFMA, with a
// representation error below fp32 rounding. Six v_mfma_f32_16x16x32_bf16 (16 cycles each) replace eight
// v_mfma_f32_16x16x4_f32 (32 cycles each) per 16x16x32 block: 2.7x fewer matrix cycles. Weights are split once per
// call by a prep kernel (with the LayerNorm affine terms folded in: W' = W diag(gamma), b' = b + W beta, so the
// kernel's LayerNorms only normalise); activations are split by their producer (LayerNorm, attention, GELU, the
// last residual add) when they are written to LDS, three bf16 planes per operand.
// The attention (S = QK^T, O = PV: ~18 % of the block's FLOPs) stays on exact fp32 MFMA with the S^T-accumulator
// trick of swin_fused.hip.
//
// One 256-thread workgroup per 7x7 window, three per CU (LDS 54 KB): T (fp32 residual stream [49][68]) | X (halo
// patch -> three bf16 planes [64][72] of U1 -> QKV fp32 [49][196] -> O planes -> U2 planes -> MLP hidden half planes
// -> final T planes for the pw GEMM) | parameters. Each producer keeps its result in registers until every wave has
// read X's previous content. GEMM tiles cover token rows 0..63 (four 16-row blocks; rows 49..63 are finite padding
// whose outputs are dropped) and are transposed (the weight planes are the MFMA A operand): lane (g, l15) holds
// out[token rb*16 + l15][n = cb*16 + 4g .. +3].
//
// Status: OFF by default. Numerically it matches the fp32 kernel (the model tests' errors are unchanged), but on
// MI355X it is slower at the L28 shape (bench_ops, same box): swin_fused.hip 0.91-0.93 ms; this design at two
// workgroups per CU (81 KB LDS, one region per operand) 0.99 ms, persistent with the next halo prefetched 1.02 ms,
// three per CU (this layout, 15 barriers, 168 VGPRs with spills) 1.10 ms. The matrix cycles per window drop from
// 16.9k to 10k, but the six-product chains, the operand splits (~500 VALU per wave) and the extra barriers leave
// the window's latency higher, and the HIP compiler's schedule does not hide it at these occupancies.
//
// Reference semantics as swin_fused.hip (ultralytics/nn/modules/blocks_transformer.py:8-171).
#include "common.h"
#include <math.h>
#include <stdlib.h>

namespace ys {
namespace x3 {

constexpr int NR = 49;   // tokens per 7x7 window
constexpr int XR = 48;   // attention: token row 48 on the VALU (rows 0..47 = three 16-row fp32 MFMA blocks)
constexpr int HPW = 12;  // halo patch row stride (9 used)

struct Args {
  const float* x;
  float* y;
  int B, H, W, nWx, nWin;
  const float* dw;     // [C][9]
  float ln1_eps, ln2_eps;
  const bf16_t* win;   // planes [3][3C][C], LN1 affine folded
  const float* bin;    // [3C] folded
  const bf16_t* wo;    // [3][C][C]
  const float* bo;
  const bf16_t* w1;    // [3][HID][C], LN2 affine folded
  const float* b1;     // [HID] folded
  const bf16_t* w2;    // [3][C][HID]
  const float* b2;
  const bf16_t* wpw;   // [3][C][C]
  const float* bn_scale;
  const float* bn_shift;
  float scale;
};

__device__ __forceinline__ f32x4 mfma16(bf16x8_t a, bf16x8_t b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float dot4_acc(float4 a, float4 b, float acc) {
  acc = fmaf(a.x, b.x, acc);
  acc = fmaf(a.y, b.y, acc);
  acc = fmaf(a.z, b.z, acc);
  return fmaf(a.w, b.w, acc);
}
__device__ __forceinline__ float group4_sum(float v) { return xor32_sum(xor16_sum(v)); }

// one split level of a pair: the bf16 pair nearest to r (round to nearest even); r becomes the (exact) remainder
__device__ __forceinline__ uint32_t split_level(f32x2& r) {
  const uint32_t h = pack_bf16x2(r.x, r.y);
  r = r - f32x2{__uint_as_float(h << 16), __uint_as_float(h & 0xffff0000u)};  // v_pk_add_f32 (neg)
  return h;
}
// v = h + m + l (bf16, round to nearest even at each step)
__device__ __forceinline__ void split4(f32x4 v, uint2& h, uint2& m, uint2& l) {
  f32x2 a = {v.x, v.y}, b = {v.z, v.w};
  h.x = split_level(a);
  h.y = split_level(b);
  m.x = split_level(a);
  m.y = split_level(b);
  l.x = pack_bf16x2(a.x, a.y);
  l.y = pack_bf16x2(b.x, b.y);
}
// the three planes of 4 consecutive elements of row `row`, column `col` (a multiple of 4)
template <int PS, int PL>
__device__ __forceinline__ void store_planes4(bf16_t* P, int row, int col, f32x4 v) {
  uint2 h, m, l;
  split4(v, h, m, l);
  bf16_t* d = P + row * PS + col;
  *reinterpret_cast<uint2*>(d) = h;
  *reinterpret_cast<uint2*>(d + PL) = m;
  *reinterpret_cast<uint2*>(d + 2 * PL) = l;
}

// Weight-plane fragments of one GEMM for this wave's column blocks cb = cb0 + 4j: lane (g, l15) holds
// W_p[cb*16 + l15][koff + 32s + 8g .. +7] (16-byte global loads, L2-resident).
template <int K, int NJ>
struct WP {
  bf16x8_t v[NJ][K / 32][3];
};
template <int K, int NJ>
__device__ __forceinline__ void load_wp(const bf16_t* __restrict__ Wp, int N, int KT, int koff, int cb0, WP<K, NJ>& f,
                                        int lane) {
  const int l15 = lane & 15, g = lane >> 4;
#pragma unroll
  for (int p = 0; p < 3; ++p)
#pragma unroll
    for (int s = 0; s < K / 32; ++s)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        f.v[j][s][p] = *reinterpret_cast<const bf16x8_t*>(
            Wp + ((long)p * N + (cb0 + 4 * j) * 16 + l15) * KT + koff + 32 * s + 8 * g);
}

// acc[rb][j] += (A[rows rb*16 .. +15][0, K) . W^T)^T: A = three LDS planes (row stride PS, plane stride PL), the
// weight planes as the MFMA A operand, so the lane holds out[token rb*16 + l15][n = cb*16 + 4g .. +3]. Six products
// per (k-step, row block, column block), smallest terms first. The LDS operand reads run two (k-step, row block)
// steps ahead of the MFMAs (at two waves per SIMD a read waited for right before its MFMAs exposes its latency).
template <int K, int NJ, int PS, int PL>
__device__ __forceinline__ void gemm_x3(const bf16_t* A, const WP<K, NJ>& w, f32x4 (&acc)[4][NJ], int lane) {
  const int l15 = lane & 15, g = lane >> 4;
  constexpr int NS = (K / 32) * 4;  // steps (s, rb), rb fastest
  const bf16_t* a0 = A + l15 * PS + 8 * g;
  bf16x8_t u[3][3];
  auto ld = [&](int i, bf16x8_t (&v)[3]) {
    const bf16_t* ar = a0 + (i & 3) * 16 * PS + 32 * (i >> 2);
    v[0] = *reinterpret_cast<const bf16x8_t*>(ar);
    v[1] = *reinterpret_cast<const bf16x8_t*>(ar + PL);
    v[2] = *reinterpret_cast<const bf16x8_t*>(ar + 2 * PL);
  };
  ld(0, u[0]);
  ld(1, u[1]);
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    if (i + 2 < NS) ld(i + 2, u[(i + 2) % 3]);
    const int s = i >> 2, rb = i & 3;
    const bf16x8_t* v = u[i % 3];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      f32x4 c = acc[rb][j];
      c = mfma16(w.v[j][s][2], v[0], c);
      c = mfma16(w.v[j][s][1], v[1], c);
      c = mfma16(w.v[j][s][0], v[2], c);
      c = mfma16(w.v[j][s][1], v[0], c);
      c = mfma16(w.v[j][s][0], v[1], c);
      acc[rb][j] = mfma16(w.v[j][s][0], v[0], c);
    }
  }
}

// LayerNorm statistics of token rows [0, 49) of T (fp32, stride LT) and the normalised rows (affine folded into the
// next GEMM) as three bf16 planes; rows 49..63 get zeros. 4 lanes per row (a DPP quad), C/4 values each.
template <int C, int LT, int PS, int PL>
__device__ __forceinline__ void ln_planes(const float* T, bf16_t* P, float eps, int tid) {
  constexpr int CP = C / 4;
  const int r = tid >> 2, qd = tid & 3;
  const bool valid = r < NR;
  f32x4 v[CP / 4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < CP / 4; ++i) {
    v[i] = valid ? *reinterpret_cast<const f32x4*>(T + r * LT + qd * CP + 4 * i) : f32x4{0.f, 0.f, 0.f, 0.f};
    s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  }
  const float mean = quad_sum(s) * (1.0f / (float)C);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < CP / 4; ++i) {
    v[i] -= mean;
    q += (v[i].x * v[i].x + v[i].y * v[i].y) + (v[i].z * v[i].z + v[i].w * v[i].w);
  }
  const float rs = valid ? __builtin_amdgcn_rsqf(quad_sum(q) * (1.0f / (float)C) + eps) : 0.f;
#pragma unroll
  for (int i = 0; i < CP / 4; i += 2) {
    uint2 h0, m0, l0, h1, m1, l1;
    split4(v[i] * rs, h0, m0, l0);
    split4(v[i + 1] * rs, h1, m1, l1);
    bf16_t* d = P + r * PS + qd * CP + 4 * i;
    *reinterpret_cast<uint4*>(d) = make_uint4(h0.x, h0.y, h1.x, h1.y);
    *reinterpret_cast<uint4*>(d + PL) = make_uint4(m0.x, m0.y, m1.x, m1.y);
    *reinterpret_cast<uint4*>(d + 2 * PL) = make_uint4(l0.x, l0.y, l1.x, l1.y);
  }
}

template <int C, int NH>
__global__ __launch_bounds__(256, 3) void swin_x3_kernel(Args p) {
  constexpr int HD = C / NH;
  constexpr int HID = 2 * C;
  constexpr int LT = C + 4;      // T row stride (floats)
  constexpr int LQ = 3 * C + 4;  // QKV row stride (floats)
  constexpr int PS = C + 8;      // plane row stride (bf16)
  constexpr int PL = 64 * PS;    // plane stride
  constexpr int NHS = (C + 2) / 3;
  static_assert(C == 64 && HID / 2 == C, "the plane regions are sized for C = 64 (hidden halves of 64)");
  static_assert(HD % 16 == 0 && HD <= 64, "head dim");
  constexpr int T_B = NR * LT * 4;
  constexpr int QKV_B = NR * LQ * 4;
  constexpr int PLN_B = 3 * PL * 2;
  constexpr int HALO_B = 3 * NHS * 9 * HPW * 4;
  constexpr int X_B = QKV_B > HALO_B ? (QKV_B > PLN_B ? QKV_B : PLN_B) : (HALO_B > PLN_B ? HALO_B : PLN_B);
  constexpr int NPAR = 3 * C + C + HID + C + 2 * C;
  static_assert(T_B % 16 == 0 && X_B % 16 == 0, "16-byte aligned regions");
  static_assert(T_B + X_B + NPAR * 4 <= 160 * 1024 / 3, "three workgroups per CU");
  __shared__ __attribute__((aligned(16))) char smem[T_B + X_B + NPAR * 4];
  float* T = reinterpret_cast<float*>(smem);
  char* X = smem + T_B;
  float* Q = reinterpret_cast<float*>(X);
  bf16_t* P = reinterpret_cast<bf16_t*>(X);
  float* par = reinterpret_cast<float*>(smem + T_B + X_B);
  constexpr int P_BIN = 0, P_BO = 3 * C, P_B1 = 4 * C, P_B2 = 4 * C + HID, P_SC = 5 * C + HID, P_SH = 6 * C + HID;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l15 = lane & 15, g = lane >> 4;
  const int H = p.H, W = p.W;
  const int HWi = H * W;  // per-image offsets are 32-bit (the launcher checks C*H*W < 2^30)

  // XCD-aware window order: workgroup i runs on XCD i % 8 and takes windows from that XCD's contiguous range, so
  // horizontally adjacent windows (whose 7-pixel rows share 128-byte lines of x and y) meet in one L2
  const long nwin_total = (long)p.B * p.nWin;
  const long per_xcd = (nwin_total + 7) >> 3;
  const long gwl = (long)(blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  if (gwl >= nwin_total || (blockIdx.x >> 3) >= per_xcd) return;
  const int gw = __builtin_amdgcn_readfirstlane((int)gwl);
  const int img = gw / p.nWin, win = gw - (gw / p.nWin) * p.nWin;
  const int wy = win / p.nWx, wx = win - (win / p.nWx) * p.nWx;
  auto rsrc_of = [&](const float* base) {
    const unsigned long long a = (unsigned long long)base;
    return __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(a >> 32)) << 32) |
                (unsigned)__builtin_amdgcn_readfirstlane((unsigned)a)),
        (short)0, __builtin_amdgcn_readfirstlane(C * HWi * 4), 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rx = rsrc_of(p.x + (long)img * C * HWi);
  constexpr unsigned OOB = 0x80000000u;

  // halo patch [C][9][9] -> registers: row slot s = 7*wid + lane/9 < 27 is (channel 3i + s/9, patch row s%9) at
  // step i, lane%9 the column; out-of-image lanes get an out-of-range voffset (the buffer load returns 0)
  const int hl_r = lane / 9, hl_px = lane - (lane / 9) * 9;
  const int hslot = 7 * wid + hl_r;
  float hv[NHS];
  {
    const int hcs = hslot / 9, hpy = hslot - (hslot / 9) * 9;
    const int hh = wy * 7 - 1 + hpy, wc = wx * 7 - 1 + hl_px;
    const bool ok = hl_r < 7 && hslot < 27 && (unsigned)hh < (unsigned)H && (unsigned)wc < (unsigned)W;
    const unsigned voff = ok ? (unsigned)((hcs * HWi + hh * W + wc) * 4) : OOB;
    const unsigned vlast = (3 * (NHS - 1) + hcs < C) ? voff : OOB;
#pragma unroll
    for (int i = 0; i < NHS; ++i)
      hv[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, i == NHS - 1 ? vlast : voff,
                                                                            i * 3 * HWi * 4, 0));
  }
  for (int e = tid; e < NPAR; e += 256) {
    float v;
    if (e < P_BO) v = p.bin[e];
    else if (e < P_B1) v = p.bo[e - P_BO];
    else if (e < P_B2) v = p.b1[e - P_B1];
    else if (e < P_SC) v = p.b2[e - P_B2];
    else if (e < P_SH) v = p.bn_scale[e - P_SC];
    else v = p.bn_shift[e - P_SH];
    par[e] = v;
  }
  const int dw_c = tid % C;
  float dwk[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) dwk[i] = p.dw[dw_c * 9 + i];
  // QKV weight planes of column block wid (the Q block): in flight during the halo store, dw conv and LN1
  WP<C, 1> f_q;
  load_wp(p.win, 3 * C, C, 0, wid, f_q, lane);

  // ---- halo -> X (fp32 [27i + slot][HPW]) -> dw3x3 -> T (cropped / padded tokens = 0) ----
  float* halo = Q;
  if (hl_r < 7 && hslot < 27) {
#pragma unroll
    for (int i = 0; i < NHS; ++i) halo[(27 * i + hslot) * HPW + hl_px] = hv[i];
  }
  __syncthreads();
  for (int item = tid; item < C * 7; item += 256) {
    const int iy = item / C;
    const float* hp = halo + (dw_c * 9 + iy) * HPW;
    float r[3][12];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int q4 = 0; q4 < 3; ++q4) {
        const float4 v = *reinterpret_cast<const float4*>(hp + ky * HPW + 4 * q4);
        r[ky][4 * q4] = v.x; r[ky][4 * q4 + 1] = v.y; r[ky][4 * q4 + 2] = v.z; r[ky][4 * q4 + 3] = v.w;
      }
    const bool rowok = wy * 7 + iy < H;
#pragma unroll
    for (int ix = 0; ix < 7; ++ix) {
      const float v = dwk[0] * r[0][ix] + dwk[1] * r[0][ix + 1] + dwk[2] * r[0][ix + 2] + dwk[3] * r[1][ix] +
                      dwk[4] * r[1][ix + 1] + dwk[5] * r[1][ix + 2] + dwk[6] * r[2][ix] + dwk[7] * r[2][ix + 1] +
                      dwk[8] * r[2][ix + 2];
      T[(iy * 7 + ix) * LT + dw_c] = (rowok && wx * 7 + ix < W) ? v : 0.f;
    }
  }
  __syncthreads();

  // ---- LN1 -> X planes ----
  ln_planes<C, LT, PS, PL>(T, P, p.ln1_eps, tid);
  __syncthreads();

  // ---- QKV = U1 Win'^T + b_in': three column-block passes (one weight-plane set in flight ahead); the results stay
  // in registers until every wave has read U1, then replace it in X as fp32 [49][LQ] ----
  constexpr int NJ_QKV = 3 * C / 64;
  f32x4 aq[NJ_QKV][4][1];
  {
    WP<C, 1> f_n;
#pragma unroll
    for (int j = 0; j < NJ_QKV; ++j) {
      if (j + 1 < NJ_QKV) load_wp(p.win, 3 * C, C, 0, wid + 4 * (j + 1), f_n, lane);
      const f32x4 b = *reinterpret_cast<const f32x4*>(par + P_BIN + (wid + 4 * j) * 16 + 4 * g);
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) aq[j][rb][0] = b;
      gemm_x3<C, 1, PS, PL>(P, f_q, aq[j], lane);
      if (j + 1 < NJ_QKV) f_q = f_n;
    }
  }
  WP<C, 1> f_o;
  load_wp(p.wo, C, C, 0, wid, f_o, lane);  // out-proj planes: in flight during attention
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NJ_QKV; ++j)
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
      if (rb < 3 || l15 == 0)
        *reinterpret_cast<f32x4*>(Q + (rb * 16 + l15) * LQ + (wid + 4 * j) * 16 + 4 * g) = aq[j][rb][0];
  __syncthreads();

  // ---- attention (fp32 MFMA), wave = 16 queries, all heads; O stays in registers until every wave has read K / V,
  // then replaces QKV in X as planes (rows 0..63: padding queries are copies of query 48, finite) ----
  WP<C, 1> f_1a;
  load_wp(p.w1, HID, C, 0, wid, f_1a, lane);  // MLP1 (hidden half 0) planes
  f32x4 ov[NH][HD / 16];
  {
    const int q = wid * 16 + l15;
    const int qrow = q < XR ? q : XR;
    constexpr int DQ = HD / 4;
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
    // lane holds S^T[key = kb*16 + 4g + r][q = l15] per head (+ key 48 after the group sum): softmax over the keys
    // on the raw scores with exp2 (scale*log2 e folded into one FMA), 1/sum applied to O
    const float c2 = p.scale * 1.44269504088896341f;
    float p48[NH], inv[NH];
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const float sv48 = group4_sum(s48[h]);
      float mx = sv48;
#pragma unroll
      for (int kb = 0; kb < 3; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, st[h][kb][r]);
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
    // O^T[d][q] = sum_key V[key][d] P[q][key] (MFMA (kb, r) consumes keys kb*16 + 4g' + r), key 48 rank-1 update
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
      for (int db = 0; db < HD / 16; ++db) ov[h][db] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < 3; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float* vrow = Q + (kb * 16 + 4 * g + r) * LQ + 2 * C + l15;
#pragma unroll
        for (int h = 0; h < NH; ++h)
#pragma unroll
          for (int db = 0; db < HD / 16; ++db) ov[h][db] = mfma4(vrow[h * HD + db * 16], st[h][kb][r], ov[h][db]);
      }
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
      for (int db = 0; db < HD / 16; ++db) {
        const float4 v48 = *reinterpret_cast<const float4*>(Q + XR * LQ + 2 * C + h * HD + db * 16 + 4 * g);
        ov[h][db][0] = fmaf(v48.x, p48[h], ov[h][db][0]) * inv[h];
        ov[h][db][1] = fmaf(v48.y, p48[h], ov[h][db][1]) * inv[h];
        ov[h][db][2] = fmaf(v48.z, p48[h], ov[h][db][2]) * inv[h];
        ov[h][db][3] = fmaf(v48.w, p48[h], ov[h][db][3]) * inv[h];
      }
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < NH; ++h)
#pragma unroll
    for (int db = 0; db < HD / 16; ++db)
      store_planes4<PS, PL>(P, wid * 16 + l15, h * HD + db * 16 + 4 * g, ov[h][db]);
  __syncthreads();

  // ---- T += O Wo^T + bo ----
  WP<C, 1> f_1b;
  load_wp(p.w1, HID, C, 0, wid + 4, f_1b, lane);  // MLP1 (hidden half 1) planes
  {
    f32x4 acc[4][1];
    const f32x4 b = *reinterpret_cast<const f32x4*>(par + P_BO + wid * 16 + 4 * g);
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) acc[rb][0] = b;
    gemm_x3<C, 1, PS, PL>(P, f_o, acc, lane);
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      const int tok = rb * 16 + l15;
      if (rb < 3 || l15 == 0) {
        f32x4* tp = reinterpret_cast<f32x4*>(T + tok * LT + wid * 16 + 4 * g);
        *tp = *tp + acc[rb][0];
      }
    }
  }
  __syncthreads();

  // ---- LN2 -> X planes ----
  ln_planes<C, LT, PS, PL>(T, P, p.ln2_eps, tid);
  WP<C, 1> f_2a;
  load_wp(p.w2, C, HID, 0, wid, f_2a, lane);  // MLP2 planes, k in [0, 64)
  __syncthreads();

  // ---- MLP: both hidden halves Hh = GELU(U2 W1h'^T + b1h') into registers; then half by half as planes into X,
  // each followed by its MLP2 partial acc2 += Hh W2[:, half]^T ----
  f32x4 hid[2][4];
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    f32x4 acc[4][1];
    const f32x4 b = *reinterpret_cast<const f32x4*>(par + P_B1 + (wid + 4 * half) * 16 + 4 * g);
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) acc[rb][0] = b;
    gemm_x3<C, 1, PS, PL>(P, half == 0 ? f_1a : f_1b, acc, lane);
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      const f32x2 lo = gelu2_fast_(f32x2{acc[rb][0][0], acc[rb][0][1]});
      const f32x2 hi = gelu2_fast_(f32x2{acc[rb][0][2], acc[rb][0][3]});
      hid[half][rb] = f32x4{lo.x, lo.y, hi.x, hi.y};
    }
  }
  WP<C, 1> f_2b;
  load_wp(p.w2, C, HID, C, wid, f_2b, lane);  // MLP2 planes, k in [64, 128)
  f32x4 acc2[4][1];
  {
    const f32x4 b = *reinterpret_cast<const f32x4*>(par + P_B2 + wid * 16 + 4 * g);
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) acc2[rb][0] = b;
  }
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    __syncthreads();  // every wave has read X (U2, then hidden half 0)
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) store_planes4<PS, PL>(P, rb * 16 + l15, wid * 16 + 4 * g, hid[half][rb]);
    __syncthreads();
    gemm_x3<C, 1, PS, PL>(P, half == 0 ? f_2a : f_2b, acc2, lane);
  }

  // pw planes and this lane's residual x / BN terms: in flight during the final T update
  WP<C, 1> f_pw;
  load_wp(p.wpw, C, C, 0, wid, f_pw, lane);
  const __amdgpu_buffer_rsrc_t ry = rsrc_of(p.y + (long)img * C * HWi);
  unsigned vtok[4];  // byte offset of (channel wid*16 + 4g, token tb*16 + l15), or out of range
#pragma unroll
  for (int tb = 0; tb < 4; ++tb) {
    const int tok = tb * 16 + l15;
    const int iy = tok / 7, ix = tok - (tok / 7) * 7;
    const int hh = wy * 7 + iy, wc = wx * 7 + ix;
    vtok[tb] = (tok < NR && hh < H && wc < W) ? (unsigned)(((wid * 16 + 4 * g) * HWi + hh * W + wc) * 4) : OOB;
  }
  float xr[4][4];
#pragma unroll
  for (int tb = 0; tb < 4; ++tb)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      xr[tb][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, vtok[tb], r * HWi * 4, 0));

  // ---- final T = T + MLP -> X planes (rows >= 49 zero): the pw GEMM's operand ----
  __syncthreads();  // every wave has read hidden half 1
#pragma unroll
  for (int rb = 0; rb < 4; ++rb) {
    const int tok = rb * 16 + l15;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (tok < NR) v = *reinterpret_cast<const f32x4*>(T + tok * LT + wid * 16 + 4 * g) + acc2[rb][0];
    store_planes4<PS, PL>(P, tok, wid * 16 + 4 * g, v);
  }
  __syncthreads();

  // ---- y = x + SiLU(BN(Wpw T^T)): tile Y^T[c][tok], lane holds c = wid*16 + 4g + r, token tb*16 + l15 ----
  {
    f32x4 acc[4][1];
#pragma unroll
    for (int tb = 0; tb < 4; ++tb) acc[tb][0] = f32x4{0.f, 0.f, 0.f, 0.f};
    gemm_x3<C, 1, PS, PL>(P, f_pw, acc, lane);
    const f32x4 sc = *reinterpret_cast<const f32x4*>(par + P_SC + wid * 16 + 4 * g);
    const f32x4 sh = *reinterpret_cast<const f32x4*>(par + P_SH + wid * 16 + 4 * g);
#pragma unroll
    for (int tb = 0; tb < 4; ++tb)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        __builtin_amdgcn_raw_buffer_store_b32(
            __builtin_bit_cast(unsigned, xr[tb][r] + silu_fast_(acc[tb][0][r] * sc[r] + sh[r])), ry, vtok[tb],
            r * HWi * 4, 0);
  }
}

// Weight preparation: LN affine folds and the three-plane split, one wave per output row (lanes along k,
// coalesced); also the BN fold of the pw conv. Rows: [0,3C) in_proj (LN1 folded) | [3C,4C) out_proj | [4C,4C+HID)
// mlp1 (LN2 folded) | mlp2 (K = HID) | pw | C BN entries.
struct PrepArgs {
  const float *win, *bin, *ln1_w, *ln1_b, *wo, *w1, *b1, *ln2_w, *ln2_b, *w2, *wpw;
  const float *bn_w, *bn_b, *bn_m, *bn_v;
  float bn_eps;
  int C, HID;
  bf16_t *pin, *po, *p1, *p2, *ppw;
  float *bin_f, *b1_f, *bn_sc, *bn_sh;
};

__global__ __launch_bounds__(256) void swin_x3_prep_kernel(PrepArgs a) {
  const int C = a.C, HID = a.HID;
  const int lane = threadIdx.x & 63;
  int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  const float* src;
  const float* gam = nullptr;
  const float* bet = nullptr;
  const float* bsrc = nullptr;
  float* bdst = nullptr;
  bf16_t* dst;
  int N, K;
  if (n < 3 * C) {
    src = a.win; gam = a.ln1_w; bet = a.ln1_b; bsrc = a.bin; bdst = a.bin_f; dst = a.pin; N = 3 * C; K = C;
  } else if ((n -= 3 * C) < C) {
    src = a.wo; dst = a.po; N = C; K = C;
  } else if ((n -= C) < HID) {
    src = a.w1; gam = a.ln2_w; bet = a.ln2_b; bsrc = a.b1; bdst = a.b1_f; dst = a.p1; N = HID; K = C;
  } else if ((n -= HID) < C) {
    src = a.w2; dst = a.p2; N = C; K = HID;
  } else if ((n -= C) < C) {
    src = a.wpw; dst = a.ppw; N = C; K = C;
  } else if ((n -= C) < C) {
    if (lane == 0) {
      const float inv = 1.0f / sqrtf(a.bn_v[n] + a.bn_eps);
      const float sc = a.bn_w[n] * inv;
      a.bn_sc[n] = sc;
      a.bn_sh[n] = a.bn_b[n] - a.bn_m[n] * sc;
    }
    return;
  } else {
    return;
  }
  const float* row = src + (long)n * K;
  float bacc = 0.f;
  for (int k = lane; k < K; k += 64) {
    const float w = row[k];
    if (bet) bacc = fmaf(w, bet[k], bacc);
    const float v = gam ? w * gam[k] : w;
    const bf16_t h = f2bf(v);
    const float r1 = v - bf2f(h);
    const bf16_t m = f2bf(r1);
    const bf16_t l = f2bf(r1 - bf2f(m));
    dst[(long)n * K + k] = h;
    dst[((long)N + n) * K + k] = m;
    dst[(2L * N + n) * K + k] = l;
  }
  if (bdst) {
    bacc = wave_sum(bacc);
    if (lane == 0) bdst[n] = bsrc[n] + bacc;
  }
}

}  // namespace x3
}  // namespace ys

using namespace ys;

// Opt-in (YOLOSOD_SWIN_X3=1, or the test hook below): measured slower than swin_fused.hip on MI355X - see the header.
static int g_swin_x3 = -1;
static bool swin_x3_env() {
  if (g_swin_x3 < 0) {
    const char* e = getenv("YOLOSOD_SWIN_X3");
    g_swin_x3 = (e && atoi(e) != 0) ? 1 : 0;
  }
  return g_swin_x3 != 0;
}

// Test hook: route C = 64 SwinBlocks through this kernel (1) or swin_fused.hip (0).
YS_EXPORT void yolosod_debug_set_swin_x3(int on) { g_swin_x3 = on ? 1 : 0; }

bool yolosod_swin_x3_ok(int C, int num_heads, int wh, int ww, int mlp_hidden) {
  return swin_x3_env() && C == 64 && num_heads == 2 && wh == 7 && ww == 7 && mlp_hidden == 2 * C;
}

size_t yolosod_swin_x3_workspace(int C, int mlp_hidden) {
  Sizer s;
  s.take<bf16_t>((size_t)3 * 3 * C * C);           // in_proj planes
  s.take<bf16_t>((size_t)3 * C * C);               // out_proj
  s.take<bf16_t>((size_t)3 * mlp_hidden * C);      // mlp1
  s.take<bf16_t>((size_t)3 * C * mlp_hidden);      // mlp2
  s.take<bf16_t>((size_t)3 * C * C);               // pw
  s.take<float>((size_t)3 * C + mlp_hidden + 2 * C);  // folded biases, BN scale / shift
  return s.off;
}

// returns 1 if launched, 0 if the shape is not handled, < 0 on error
int yolosod_swin_x3_launch(const float* x, float* y, int B, int C, int H, int W, int num_heads, int wh, int ww,
                           int nWx, int nWin,
                           const float* dw_w, const float* ln1_w, const float* ln1_b, float ln1_eps,
                           const float* in_proj_w, const float* in_proj_b, const float* out_proj_w,
                           const float* out_proj_b, const float* ln2_w, const float* ln2_b, float ln2_eps,
                           const float* mlp1_w, const float* mlp1_b, int mlp_hidden, const float* mlp2_w,
                           const float* mlp2_b, const float* pw_w, const float* bn_w, const float* bn_b,
                           const float* bn_mean, const float* bn_var, float bn_eps, void* workspace,
                           size_t workspace_bytes, hipStream_t st) {
  if (!yolosod_swin_x3_ok(C, num_heads, wh, ww, mlp_hidden)) return 0;
  if ((long)C * H * W >= (1L << 30) || (long)B * nWin >= (1L << 31)) return 0;
  Carver cv(workspace, workspace_bytes);
  bf16_t* pin = cv.take<bf16_t>((size_t)3 * 3 * C * C);
  bf16_t* po = cv.take<bf16_t>((size_t)3 * C * C);
  bf16_t* p1 = cv.take<bf16_t>((size_t)3 * mlp_hidden * C);
  bf16_t* p2 = cv.take<bf16_t>((size_t)3 * C * mlp_hidden);
  bf16_t* ppw = cv.take<bf16_t>((size_t)3 * C * C);
  float* fb = cv.take<float>((size_t)3 * C + mlp_hidden + 2 * C);
  if (!fb) {
    set_error("swin_x3: workspace too small (%zu)", workspace_bytes);
    return -1;
  }
  x3::PrepArgs pa{in_proj_w, in_proj_b, ln1_w, ln1_b, out_proj_w, mlp1_w, mlp1_b, ln2_w, ln2_b, mlp2_w, pw_w,
                  bn_w, bn_b, bn_mean, bn_var, bn_eps, C, mlp_hidden, pin, po, p1, p2, ppw,
                  fb, fb + 3 * C, fb + 3 * C + mlp_hidden, fb + 4 * C + mlp_hidden};
  const int rows = 3 * C + C + mlp_hidden + C + C + C;
  hipLaunchKernelGGL(x3::swin_x3_prep_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, pa);
  x3::Args a{x, y, B, H, W, nWx, nWin, dw_w, ln1_eps, ln2_eps, pin, fb, po, out_proj_b, p1, fb + 3 * C, p2, mlp2_b,
             ppw, fb + 3 * C + mlp_hidden, fb + 4 * C + mlp_hidden, 1.0f / sqrtf((float)(C / num_heads))};
  const long nwin = (long)B * nWin;
  hipLaunchKernelGGL((x3::swin_x3_kernel<64, 2>), dim3((unsigned)(8 * ((nwin + 7) / 8))), dim3(256), 0, st, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("swin_x3: launch failed: %s", hipGetErrorString(e));
    return -1;
  }
  return 1;
}
