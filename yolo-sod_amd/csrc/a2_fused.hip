// A2_Attn's LayerNorm -> QKV projection -> multi-head attention in one kernel per (image, head), on the fp16 matrix
// cores at fp32 accuracy (the two-term split of swin_x3.hip: v = h + l, a.b ~ ah.bh + ah.bl + al.bh).
//
// Reference: ultralytics/nn/modules/a2_attn.py:50-53 - seq_norm = layer_norm(seq); attention(seq_norm, seq_norm,
// seq_norm) with nn.MultiheadAttention (batch_first): q, k, v = seq_norm @ W_in^T + b_in split in three; per head
// softmax(q k^T / sqrt(64)) v. The out-projection of the MHA is folded with the output 1x1 conv (A2_Attn._fused_out)
// and runs as the following token GEMM; the pooling before it is a2_pool_tokens_kernel.
//
// Why one kernel: the decomposed path wrote the normalised tokens, then Q/K/V [tokens][3C] (31 MB at bs 32) to HBM
// and read them back in the attention kernel, over three launches. Here one 512-thread workgroup per (image, head)
// keeps everything of its head on chip:
//   1. K loop over the C input channels in 64-wide stages: the stage's slice of the pooled tokens [L][64] is read
//      from HBM / L2 one stage ahead, normalised with the per-token (mean, rstd) of row_stats_kernel (the LN affine
//      is folded into the prepared weights: W' = W diag(gamma), b' = b + W beta) and stored as two fp16 planes in
//      LDS (double-buffered); wave w owns head-local column block w & 3 of Q, K and V (16 output dims each) for half
//      of the tokens (w >> 2) - its weight fragments stream from L2 in the fragment-major layout of the prep kernel,
//      one stage ahead.
//   2. Q and K go to LDS as [token][d] planes, V as V^T [d][token] planes (computed with the operands swapped, so a
//      lane holds 4 consecutive tokens of one dim).
//   3. Attention: wave w takes query blocks w, w+8: S^T = K Q^T per 16-key block (the Q fragments read with the
//      k permutation that makes the S^T accumulators the P^T operand of O^T = V^T P^T), softmax over keys in
//      registers (exp2, 1/sum applied to O), O written token-major [B*L][C] at the head's 64 columns.
// Weights are scaled by 64 (exact) at the split so their low terms stay normal fp16; Q, K, V keep the factor: it is
// folded into the softmax's exp2 scale and into 1/sum.
#include "common.h"
#include <math.h>

namespace ys {
namespace a2f {

constexpr float WSC = 64.0f;
constexpr int HD = 64;          // head dim (the kernel's shape)
constexpr int KS = 64;          // k stage (two 32-k MFMA steps)
constexpr int PSA = KS + 8;     // activation plane row stride (halves): 9 16-byte quads, conflict-free b128 reads
constexpr int PSQ = HD + 4;     // Q / K plane row stride (34 dwords: the 8-byte fragment reads of 16 rows hit distinct bank pairs)
constexpr int MAXTB = 10;       // token blocks of 16: L <= 160

__device__ __forceinline__ f32x4 mfma16(f16x8_t a, f16x8_t b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

struct Args {
  const float* S;      // [B*L][C] pooled tokens
  const float* stats;  // [B*L][2] (mean, rstd)
  const h16_t* w;      // prepared in_proj planes [2][3C][C] (x64, LN affine folded, fragment-major)
  const float* b;      // [3C] folded bias
  float* O;            // [B*L][C] attention output (heads concatenated)
  int L, C;
  float scale;         // 1 / sqrt(HD)
  unsigned* range_flag;
  const unsigned* prep_flag;
};

template <int NTB>
__global__ __launch_bounds__(512, 1) void a2_qkv_attn_kernel(Args p) {
  constexpr int NW = 8;                 // waves: (column block 0..3 of Q / K / V) x (token half 0..1)
  constexpr int NT = 64 * NW;
  constexpr int TBH = (NTB + 1) / 2;    // token blocks per half
  constexpr int NL = NTB * 16;          // padded tokens
  constexpr int APL = NL * PSA;         // activation plane (halves)
  constexpr int QPL = NL * PSQ;         // Q / K plane
  constexpr int PSV = NL + 4;           // V^T row stride (an odd multiple of 2 dwords mod 32: conflict-free 8-byte reads)
  constexpr int VPL = HD * PSV;         // V^T plane
  constexpr int A_B = 2 * 2 * APL * 2;  // two buffers x two planes
  constexpr int QKV_B = (2 * QPL * 2 + 2 * VPL) * 2;
  constexpr int R_B = A_B > QKV_B ? A_B : QKV_B;
  static_assert(R_B + NL * 8 <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[R_B + NL * 8];
  h16_t* Ab = reinterpret_cast<h16_t*>(smem);               // [2 buf][2 plane][NL][PSA]
  h16_t* Qp = reinterpret_cast<h16_t*>(smem);               // [2][NL][PSQ]   (after the K loop)
  h16_t* Kp = Qp + 2 * QPL;                                 // [2][NL][PSQ]
  h16_t* Vt = Kp + 2 * QPL;                                 // [2][HD][PSV]
  float2* st = reinterpret_cast<float2*>(smem + R_B);       // (mean, rstd) per token

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, g = lane >> 4;
  const int cblk = wid & 3, tb0 = (wid >> 2) * TBH;
  const int C = p.C, L = p.L;
  const int heads = C / HD;
  // XCD-aware: the heads of one image run on one XCD (they read the same pooled tokens from its L2)
  const int nblk = gridDim.x;
  const int wg = (nblk & 7) ? (int)blockIdx.x : (int)(blockIdx.x & 7) * (nblk >> 3) + (int)(blockIdx.x >> 3);
  const int img = wg / heads, h = wg - img * heads;
  float rng = 0.f;

  const float* Sb = p.S + (long)img * L * C;
  for (int t = tid; t < NL; t += NT) {
    const float2 v = t < L ? *reinterpret_cast<const float2*>(p.stats + 2 * ((long)img * L + t)) : make_float2(0.f, 0.f);
    st[t] = v;
  }
  // staging items of one 64-wide k stage: token rows as float4 (NL * 16 per stage)
  constexpr int NIT = (NL * 16 + NT - 1) / NT;
  float4 sA[NIT], sB[NIT];  // stage s + 1 and s + 2 in flight (two register sets)
  auto load_stage = [&](float4 (&stg)[NIT], int s) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int e = tid + NT * i;
      const int t = e >> 4, q = e & 15;
      stg[i] = (e < NL * 16 && t < L) ? *reinterpret_cast<const float4*>(Sb + (long)t * C + KS * s + 4 * q)
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_stage = [&](const float4 (&stg)[NIT], int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int e = tid + NT * i;
      if (e < NL * 16) {
        const int t = e >> 4, q = e & 15;
        const float2 ms = st[t];
        const float4 v = stg[i];
        const f32x4 u = f32x4{(v.x - ms.x) * ms.y, (v.y - ms.x) * ms.y, (v.z - ms.x) * ms.y, (v.w - ms.x) * ms.y};
        uint2 hh, ll;
        split4(u, hh, ll);
        h16_t* d = Ab + (buf * 2) * APL + t * PSA + 4 * q;
        *reinterpret_cast<uint2*>(d) = hh;
        *reinterpret_cast<uint2*>(d + APL) = ll;
      }
    }
  };
  // weight fragments of column block cblk of Q, K, V (rows h*64 + 16 cblk + [0,16) of each third); 32-k steps
  const int nk32 = C / 32;
  const int nstage = C / KS;
  const long pst = (long)3 * C * C;  // plane stride
  int nbr[3];
#pragma unroll
  for (int m = 0; m < 3; ++m) nbr[m] = (m * C + h * HD) / 16 + cblk;
  auto wfrag = [&](int m, int s32, int pl) {
    return *reinterpret_cast<const f16x8_t*>(p.w + pl * pst + ((long)(nbr[m] * nk32 + s32) * 64 + lane) * 8);
  };
  f16x8_t wa[3][2], wb[3][2];  // [m][plane] of two consecutive 32-k sub-steps (a rolling prefetch)
  auto load_w = [&](f16x8_t (&w)[3][2], int s32) {
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      w[m][0] = wfrag(m, s32, 0);
      w[m][1] = wfrag(m, s32, 1);
    }
  };
  load_w(wa, 0);
  // accumulators: Q, K (lane: token tb*16 + l15, dims 16 cblk + 4g + r) and V swapped (lane: dim 16 cblk + l15,
  // tokens tb*16 + 4g + r); start from 64 b'
  f32x4 acc[3][TBH];
  {
    const f32x4 bq = *reinterpret_cast<const f32x4*>(p.b + h * HD + 16 * cblk + 4 * g) * WSC;
    const f32x4 bk = *reinterpret_cast<const f32x4*>(p.b + C + h * HD + 16 * cblk + 4 * g) * WSC;
    const float bv = p.b[2 * C + h * HD + 16 * cblk + l15] * WSC;
#pragma unroll
    for (int i = 0; i < TBH; ++i) {
      acc[0][i] = bq;
      acc[1][i] = bk;
      acc[2][i] = f32x4{bv, bv, bv, bv};
    }
  }
  load_stage(sA, 0);
  load_stage(sB, nstage > 1 ? 1 : 0);
  __syncthreads();  // stats in LDS
  store_stage(sA, 0);
  auto mma = [&](const f16x8_t (&w)[3][2], int buf, int u) __attribute__((always_inline)) {
    const h16_t* a0 = Ab + (buf * 2) * APL + l15 * PSA + 32 * u + 8 * g;
#pragma unroll
    for (int i = 0; i < TBH; ++i) {
      const int tb = tb0 + i;
      if (tb < NTB) {
        const f16x8_t xh = *reinterpret_cast<const f16x8_t*>(a0 + tb * 16 * PSA);
        const f16x8_t xl = *reinterpret_cast<const f16x8_t*>(a0 + tb * 16 * PSA + APL);
#pragma unroll
        for (int m = 0; m < 2; ++m) {  // Q, K: weights as the A operand (rows = dims), tokens as B
          f32x4 c = mfma16(w[m][1], xh, acc[m][i]);
          c = mfma16(w[m][0], xl, c);
          acc[m][i] = mfma16(w[m][0], xh, c);
        }
        {  // V: tokens as the A operand, weights as B (lane: 4 consecutive tokens of one dim)
          f32x4 c = mfma16(xh, w[2][1], acc[2][i]);
          c = mfma16(xl, w[2][0], c);
          acc[2][i] = mfma16(xh, w[2][0], c);
        }
      }
    }
  };
  auto stage = [&](int s, float4 (&stored)[NIT], float4 (&next)[NIT]) __attribute__((always_inline)) {
    // entry: stage s is in buffer s & 1, `next` holds stage s + 1's loads in flight, `stored` is free
    const int buf = s & 1;
    // unconditional (clamped) loads: a register set written on some trips only becomes a phi whose copies wait
    // for the loads in flight
    load_stage(stored, s + 2 < nstage ? s + 2 : nstage - 1);
    __syncthreads();  // stage s's planes stored; every wave is done with stage s - 1's buffer
    load_w(wb, 2 * s + 1);
    mma(wa, buf, 0);
    load_w(wa, s + 1 < nstage ? 2 * s + 2 : 2 * s + 1);
    mma(wb, buf, 1);
    if (s + 1 < nstage) store_stage(next, buf ^ 1);
  };
  for (int s = 0; s < nstage; s += 2) {
    stage(s, sA, sB);
    if (s + 1 < nstage) stage(s + 1, sB, sA);
  }
  __syncthreads();  // every wave is done with the activation planes (Q / K / V^T reuse the region)
  // Q, K -> [token][d] planes, V -> V^T [d][token] planes (all x64); padded tokens hold finite values
#pragma unroll
  for (int i = 0; i < TBH; ++i) {
    const int tb = tb0 + i;
    if (tb < NTB) {
      const int tok = tb * 16 + l15;
      uint2 hh, ll;
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const f32x4 v = acc[m][i];
        rng = range_acc(rng, v);
        split4(v, hh, ll);
        h16_t* d = (m == 0 ? Qp : Kp) + tok * PSQ + 16 * cblk + 4 * g;
        *reinterpret_cast<uint2*>(d) = hh;
        *reinterpret_cast<uint2*>(d + QPL) = ll;
      }
      rng = range_acc(rng, acc[2][i]);
      split4(acc[2][i], hh, ll);
      h16_t* d = Vt + (16 * cblk + l15) * PSV + tb * 16 + 4 * g;
      *reinterpret_cast<uint2*>(d) = hh;
      *reinterpret_cast<uint2*>(d + VPL) = ll;
    }
  }
  __syncthreads();

  // attention: S^T[key][q] per 16-key block; slot j of lane group g in 32-d step s is head dim 32s + 4g + j (j < 4)
  // or 32s + 16 + 4g + j - 4 for both the Q (B) and K (A) fragments
  const float c2 = p.scale * 1.44269504088896341f * (1.0f / (WSC * WSC));
  for (int qb = wid; qb < NTB; qb += NW) {
    f16x8_t qh[2], ql[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const h16_t* qr = Qp + (qb * 16 + l15) * PSQ + 32 * s + 4 * g;
      const uint2 a0 = *reinterpret_cast<const uint2*>(qr), a1 = *reinterpret_cast<const uint2*>(qr + 16);
      const uint2 b0 = *reinterpret_cast<const uint2*>(qr + QPL), b1 = *reinterpret_cast<const uint2*>(qr + QPL + 16);
      qh[s] = __builtin_bit_cast(f16x8_t, make_uint4(a0.x, a0.y, a1.x, a1.y));
      ql[s] = __builtin_bit_cast(f16x8_t, make_uint4(b0.x, b0.y, b1.x, b1.y));
    }
    f32x4 sc[NTB];
#pragma unroll
    for (int kb = 0; kb < NTB; ++kb) {
      f32x4 c = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const h16_t* kr = Kp + (kb * 16 + l15) * PSQ + 32 * s + 4 * g;
        const uint2 a0 = *reinterpret_cast<const uint2*>(kr), a1 = *reinterpret_cast<const uint2*>(kr + 16);
        const uint2 b0 = *reinterpret_cast<const uint2*>(kr + QPL), b1 = *reinterpret_cast<const uint2*>(kr + QPL + 16);
        const f16x8_t kh = __builtin_bit_cast(f16x8_t, make_uint4(a0.x, a0.y, a1.x, a1.y));
        const f16x8_t kl = __builtin_bit_cast(f16x8_t, make_uint4(b0.x, b0.y, b1.x, b1.y));
        c = mfma16(kl, qh[s], c);
        c = mfma16(kh, ql[s], c);
        c = mfma16(kh, qh[s], c);
      }
      sc[kb] = c;
      // keep the scheduler from hoisting every key block's K reads ahead (register pressure at 2 waves per SIMD)
      if (kb & 1) __builtin_amdgcn_sched_barrier(0);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < NTB; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = (kb * 16 + 4 * g + r < L) ? sc[kb][r] : -INFINITY;
        sc[kb][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = xor32_max(xor16_max(mx));
    const float mc = -mx * c2;
    float sum = 0.f;
#pragma unroll
    for (int kb = 0; kb < NTB; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float e = __builtin_amdgcn_exp2f(fmaf(sc[kb][r], c2, mc));
        sc[kb][r] = e;
        sum += e;
      }
    const float inv = __builtin_amdgcn_rcpf(xor32_sum(xor16_sum(sum))) * (1.0f / WSC);  // V is x64
    f32x4 o[HD / 16];
#pragma unroll
    for (int db = 0; db < HD / 16; ++db) o[db] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s2 = 0; s2 < (NTB + 1) / 2; ++s2) {
      uint2 h0, l0, h1 = make_uint2(0u, 0u), l1 = make_uint2(0u, 0u);
      split4(sc[2 * s2], h0, l0);
      if (2 * s2 + 1 < NTB) split4(sc[2 * s2 + 1], h1, l1);
      const f16x8_t ph = __builtin_bit_cast(f16x8_t, make_uint4(h0.x, h0.y, h1.x, h1.y));
      const f16x8_t pl = __builtin_bit_cast(f16x8_t, make_uint4(l0.x, l0.y, l1.x, l1.y));
#pragma unroll
      for (int db = 0; db < HD / 16; ++db) {
        const h16_t* vr = Vt + (db * 16 + l15) * PSV + 32 * s2 + 4 * g;
        const uint2 a0 = *reinterpret_cast<const uint2*>(vr);
        const uint2 b0 = *reinterpret_cast<const uint2*>(vr + VPL);
        uint2 a1 = make_uint2(0u, 0u), b1 = make_uint2(0u, 0u);
        if (2 * s2 + 1 < NTB) {
          a1 = *reinterpret_cast<const uint2*>(vr + 16);
          b1 = *reinterpret_cast<const uint2*>(vr + VPL + 16);
        }
        const f16x8_t vh = __builtin_bit_cast(f16x8_t, make_uint4(a0.x, a0.y, a1.x, a1.y));
        const f16x8_t vl = __builtin_bit_cast(f16x8_t, make_uint4(b0.x, b0.y, b1.x, b1.y));
        f32x4 c = mfma16(vl, ph, o[db]);
        c = mfma16(vh, pl, c);
        o[db] = mfma16(vh, ph, c);
      }
    }
    // O^T lane: dims db*16 + 4g + r of query qb*16 + l15
    const int q = qb * 16 + l15;
    if (q < L) {
      float* dst = p.O + ((long)img * L + q) * C + h * HD + 4 * g;
#pragma unroll
      for (int db = 0; db < HD / 16; ++db) {
        const f32x4 v = o[db] * inv;
        rng = range_acc(rng, v);  // P x V at fp32 accuracy; also catches a NaN from upstream
        *reinterpret_cast<f32x4*>(dst + db * 16) = v;
      }
    }
  }
  range_report(p.range_flag, rng);
  if (p.prep_flag && p.range_flag && blockIdx.x == 0 && threadIdx.x == 0 && *p.prep_flag) *p.range_flag = 1u;
}

// ---- proj 1x1 conv (BN folded) + SiLU + adaptive row pooling to the area tokens, one kernel ----------------------
// a2_attn.py:39-48: x_proj = SiLU(conv1x1(x)) (Conv with folded BN), pooled = adaptive_avg_pool2d(x_proj, (A, W)),
// seq = pooled.flatten(2).transpose(1, 2). One 512-thread workgroup per (image, 64 output channels, area group)
// computes the [64][pixels] tile of x_proj over the rows its areas pool on fp16-split MFMA (weights = the A operand,
// pixels = B), keeps it in LDS and averages the row bins [floor(a H / A), ceil((a + 1) H / A)) straight into the
// token-major S rows: x_proj never reaches HBM (the decomposed path wrote and re-read it, 26 MB each way at bs 32).
// Area group q of G takes areas [q A / G, (q + 1) A / G) and the rows [floor(a0 H / A), ceil(a1 H / A)) they pool
// (a row shared by two bins at a group edge is computed by both groups): at 20x20 / 8 areas two groups of 10 rows
// halve the tile, so two workgroups share a CU and hide each other's load latency (one per CU waited on memory half
// of its cycles): the half-tile kernel runs 4 waves (each with the column blocks and registers of a wave of the
// one-tile kernel), so a CU holds two independent workgroups. The x tile of each 32-channel k step is staged as 4x4
// (k, pixel) blocks transposed in registers into [pixel][k] fp16 planes (double-buffered).
constexpr int PMAXHW = 400;   // pixels per area group the tile holds (20x20 at 640^2 in one group)
constexpr int PPS = 40;       // staged plane row stride (halves): 32 k + 8
struct PoolGroup {
  int a0, a1, r0, r1;  // areas [a0, a1), rows [r0, r1)
};
__host__ __device__ inline PoolGroup pool_group(int q, int G, int A, int H) {
  PoolGroup g;
  g.a0 = (q * A) / G;
  g.a1 = ((q + 1) * A) / G;
  g.r0 = (g.a0 * H) / A;
  g.r1 = (g.a1 * H + A - 1) / A;
  return g;
}
template <int NCB, int NW>  // 16-pixel column blocks per area group, waves; (13, 4): two workgroups per CU
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void a2_proj_pool_kernel(const float* __restrict__ x,
                                                                              const h16_t* __restrict__ wp,
                                                                              const float* __restrict__ bp,
                                                                              float* __restrict__ S, int C, int H,
                                                                              int W, int A, int G,
                                                                              unsigned* range_flag,
                                                                              const unsigned* prep_flag) {
  constexpr int NPX = NCB * 16;                 // padded pixels
  constexpr int PPL = NPX * PPS;                // plane (halves)
  constexpr int STG_B = 2 * 2 * PPL * 2;        // two buffers x two planes
  constexpr int HWP = NPX + 1;                  // fp32 tile row stride (odd: conflict-free per-channel reads)
  constexpr int T_B = 64 * HWP * 4;
  constexpr int R_B = STG_B > T_B ? STG_B : T_B;
  constexpr int NT = 64 * NW;
  constexpr int CBW = (NCB + NW - 1) / NW;      // column blocks per wave
  static_assert(R_B <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[R_B];
  h16_t* Pl = reinterpret_cast<h16_t*>(smem);   // [2 buf][2 plane][NPX][PPS]
  float* Tt = reinterpret_cast<float*>(smem);   // [64][HWP] after the K loop

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, g = lane >> 4;
  const int HW = H * W;
  const int ncb64 = C / 64;
  const int nblk = gridDim.x;
  // XCD-aware: consecutive wg (the channel blocks and area groups of one image) on one XCD
  const int wg = (nblk & 7) ? (int)blockIdx.x : (int)(blockIdx.x & 7) * (nblk >> 3) + (int)(blockIdx.x >> 3);
  const int img = wg / (ncb64 * G), rem = wg - img * ncb64 * G;
  const int grp = rem / ncb64, co = (rem - grp * ncb64) * 64;
  const PoolGroup pg = pool_group(grp, G, A, H);
  const int npx = (pg.r1 - pg.r0) * W;  // the group's pixels (a multiple of 4: W % 4 == 0 when G > 1)
  const float* xb = x + (long)img * C * HW + pg.r0 * W;
  float rng = 0.f;

  // staging: (4 k x 4 pixel) blocks of the 32 x NPX step tile; 8 * NPX / 4 blocks
  constexpr int NBLK = 8 * (NPX / 4);
  constexpr int NIT = (NBLK + NT - 1) / NT;
  // the x tile of step s is loaded two steps ahead (two register sets), stored split at the end of step s - 1
  float4 sA[NIT][4], sB[NIT][4];
  auto load_step = [&](float4 (&stg)[NIT][4], int s) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      // every load unconditional, its pixel clamped into the group: a load under a branch merges into a phi, and
      // the merge waited for every load in flight (vmcnt(0) between the load pairs of a step). Blocks past NBLK are
      // not stored; pixels past npx land in the tile's padding columns, whose outputs nothing reads.
      const int e = tid + NT * i;
      const int kq = e & 7, pq = e >> 3;  // k group fastest: the LDS stores of 8 lanes fill one 64-byte row run
      const int k = 32 * s + 4 * kq, px = min(4 * pq, npx - 4);
#pragma unroll
      for (int r = 0; r < 4; ++r) stg[i][r] = *reinterpret_cast<const float4*>(xb + (long)(k + r) * HW + px);
    }
  };
  auto store_step = [&](const float4 (&stg)[NIT][4], int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int e = tid + NT * i;
      if (e < NBLK) {
        const int kq = e & 7, pq = e >> 3;
        const float4* v = stg[i];
        // pixel 4pq + j: k 4kq .. 4kq + 3
        const f32x4 col[4] = {f32x4{v[0].x, v[1].x, v[2].x, v[3].x}, f32x4{v[0].y, v[1].y, v[2].y, v[3].y},
                              f32x4{v[0].z, v[1].z, v[2].z, v[3].z}, f32x4{v[0].w, v[1].w, v[2].w, v[3].w}};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          uint2 hh, ll;
          split4x(col[j], hh, ll);  // loaded x: the 3-VALU split (common.h split2x)
          rng = range_acc(rng, col[j]);
          h16_t* d = Pl + (buf * 2) * PPL + (4 * pq + j) * PPS + 4 * kq;
          *reinterpret_cast<uint2*>(d) = hh;
          *reinterpret_cast<uint2*>(d + PPL) = ll;
        }
      }
    }
  };
  // weight fragments (A operand): output rows co + 16 rb + l15, k = 32 s + 8g .. +7, fragment-major planes of W'
  const int nk32 = C / 32;
  const long pst = (long)C * C;
  auto wfrag = [&](int rb, int s, int pl) {
    return *reinterpret_cast<const f16x8_t*>(wp + pl * pst + ((long)(((co >> 4) + rb) * nk32 + s) * 64 + lane) * 8);
  };
  f32x4 acc[4][CBW];
#pragma unroll
  for (int rb = 0; rb < 4; ++rb)
#pragma unroll
    for (int j = 0; j < CBW; ++j) acc[rb][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f16x8_t wa[4][2], wb[4][2];
#pragma unroll
  for (int rb = 0; rb < 4; ++rb) {
    wa[rb][0] = wfrag(rb, 0, 0);
    wa[rb][1] = wfrag(rb, 0, 1);
  }
  auto step = [&](int s, float4 (&stored)[NIT][4], float4 (&next)[NIT][4]) __attribute__((always_inline)) {
    // entry: step s's planes are stored (buffer s & 1), `next` holds step s + 1's loads in flight, `stored` is free
    const int buf = s & 1;
    // unconditional (clamped) loads: a register set written on some trips only becomes a phi whose copies wait
    // for the loads in flight. The next step's weight fragments go out before the x tile two steps ahead: the
    // vmcnt queue is in order, so waiting for the weights (one step of lookahead) would otherwise also wait for the
    // x loads issued with them, and the x tile would get one step of latency, not two.
    const int sw = s + 1 < nk32 ? s + 1 : nk32 - 1;
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      wb[rb][0] = wfrag(rb, sw, 0);
      wb[rb][1] = wfrag(rb, sw, 1);
    }
    load_step(stored, s + 2 < nk32 ? s + 2 : nk32 - 1);
    __syncthreads();  // step s's planes stored; every wave is done with step s - 1's buffer
    const h16_t* b0 = Pl + (buf * 2) * PPL + l15 * PPS + 8 * g;
#pragma unroll
    for (int j = 0; j < CBW; ++j) {
      const int cb = wid + NW * j;
      if (cb < NCB) {
        const f16x8_t xh = *reinterpret_cast<const f16x8_t*>(b0 + cb * 16 * PPS);
        const f16x8_t xl = *reinterpret_cast<const f16x8_t*>(b0 + cb * 16 * PPS + PPL);
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          f32x4 c = mfma16(wa[rb][1], xh, acc[rb][j]);
          c = mfma16(wa[rb][0], xl, c);
          acc[rb][j] = mfma16(wa[rb][0], xh, c);
        }
      }
    }
    if (s + 1 < nk32) store_step(next, buf ^ 1);
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      wa[rb][0] = wb[rb][0];
      wa[rb][1] = wb[rb][1];
    }
  };
  load_step(sA, 0);
  load_step(sB, nk32 > 1 ? 1 : 0);
  store_step(sA, 0);
  for (int s = 0; s < nk32; s += 2) {
    step(s, sA, sB);
    if (s + 1 < nk32) step(s + 1, sB, sA);
  }
  __syncthreads();  // the staging planes are free: the SiLU tile takes the region
  // lane (g, l15) of (rb, j): channel co + 16 rb + 4g + r, pixel (wid + 8j) * 16 + l15
#pragma unroll
  for (int rb = 0; rb < 4; ++rb) {
    const f32x4 bias = *reinterpret_cast<const f32x4*>(bp + co + 16 * rb + 4 * g);
#pragma unroll
    for (int j = 0; j < CBW; ++j) {
      const int cb = wid + NW * j;
      if (cb < NCB) {
        const int px = cb * 16 + l15;
#pragma unroll
        for (int r = 0; r < 4; ++r) Tt[(16 * rb + 4 * g + r) * HWP + px] = silu_fast_(acc[rb][j][r] * (1.0f / WSC) + bias[r]);
      }
    }
  }
  __syncthreads();
  // pooled tokens: thread (c = tid % 64, column group tid / 64) averages its channel's bins in row order (as the
  // reference's CPU pooling) for the columns w = tid / 64 + 8 i of every area of the group
  const int c = tid & 63;
  const float* trow = Tt + c * HWP - pg.r0 * W;
  float* Sb = S + (long)img * A * W * C + co + c;
  for (int a = pg.a0; a < pg.a1; ++a) {
    const int r0 = (a * H) / A, r1 = ((a + 1) * H + A - 1) / A;
    const float cnt = (float)(r1 - r0);
    for (int w = tid >> 6; w < W; w += NW) {
      float sum = 0.f;
      for (int r = r0; r < r1; ++r) sum += trow[r * W + w];
      Sb[(long)(a * W + w) * C] = sum / cnt;
    }
  }
  range_report(range_flag, rng);
  // the prepared proj planes were range-checked once, at preparation: re-raise that result on every call (the
  // attention kernel does the same for the in_proj planes, but it does not run when L > 160)
  if (prep_flag && range_flag && blockIdx.x == 0 && threadIdx.x == 0 && *prep_flag) *range_flag = 1u;
}

// The same proj + SiLU + pooling with NRB * 16 output channels per workgroup (128 or 256 instead of 64), 8 waves, one
// workgroup per CU: the kernel above reads each image's x once per 64-channel block, 8 times at C = 512, and at that
// volume (8 x 26 MB per call at n640) it ran at the rate the L2 misses are served (~4 TB/s), not at its products'.
// Here x is read C / (16 NRB) times (twice at n640) from smaller area groups (e.g. 4 groups of 5 rows at 20x20). Wave w
// owns row blocks [w RBW, (w + 1) RBW) and every column block of the group: the weight fragments (A) stay in
// registers across the column blocks, the staged x planes (B) are read once per row-block pair.
template <int NCB, int NRB>
__global__ __launch_bounds__(512, 1) void a2_proj_pool_wide_kernel(const float* __restrict__ x,
                                                                  const h16_t* __restrict__ wp,
                                                                  const float* __restrict__ bp, float* __restrict__ S,
                                                                  int C, int H, int W, int A, int G,
                                                                  unsigned* range_flag, const unsigned* prep_flag) {
  constexpr int NW = 8, NT = 512;
  constexpr int CH = NRB * 16;                  // output channels per workgroup
  constexpr int RBW = NRB / NW;                 // row blocks per wave
  constexpr int NPX = NCB * 16;                 // padded pixels
  constexpr int PPL = NPX * PPS;                // plane (halves)
  constexpr int STG_B = 2 * 2 * PPL * 2;        // two buffers x two planes
  constexpr int HWP = NPX + 1;                  // fp32 tile row stride (odd: conflict-free per-channel reads)
  constexpr int T_B = CH * HWP * 4;
  constexpr int R_B = STG_B > T_B ? STG_B : T_B;
  static_assert(NRB % NW == 0, "row blocks per wave");
  static_assert(R_B <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[R_B];
  h16_t* Pl = reinterpret_cast<h16_t*>(smem);   // [2 buf][2 plane][NPX][PPS]
  float* Tt = reinterpret_cast<float*>(smem);   // [CH][HWP] after the K loop

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, g = lane >> 4;
  const int HW = H * W;
  const int nch = C / CH;
  const int nblk = gridDim.x;
  // XCD-aware: consecutive wg (the channel blocks and area groups of one image) on one XCD
  const int wgi = (nblk & 7) ? (int)blockIdx.x : (int)(blockIdx.x & 7) * (nblk >> 3) + (int)(blockIdx.x >> 3);
  const int img = wgi / (nch * G), rem = wgi - img * nch * G;
  const int grp = rem / nch, co = (rem - grp * nch) * CH;
  const PoolGroup pg = pool_group(grp, G, A, H);
  const int npx = (pg.r1 - pg.r0) * W;  // the group's pixels (a multiple of 4: W % 4 == 0 when G > 1)
  const float* xb = x + (long)img * C * HW + pg.r0 * W;
  float rng = 0.f;

  // staging: (4 k x 4 pixel) blocks of the 32 x NPX step tile; 8 * NPX / 4 blocks
  constexpr int NBLK = 8 * (NPX / 4);
  constexpr int NIT = (NBLK + NT - 1) / NT;
  // x tiles and weight fragments of steps s + 1 .. s + D - 1 are in flight in a register ring while step s computes
  // (D = 3 measured slower: 36 -> 42 us at n640)
  constexpr int D = 2;
  float4 xr[D][NIT][4];
  auto load_step = [&](float4 (&stg)[NIT][4], int s) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      // unconditional loads, pixel clamped into the group (see a2_proj_pool_kernel)
      const int e = tid + NT * i;
      const int kq = e & 7, pq = e >> 3;
      const int k = 32 * s + 4 * kq, px = min(4 * pq, npx - 4);
#pragma unroll
      for (int r = 0; r < 4; ++r) stg[i][r] = *reinterpret_cast<const float4*>(xb + (long)(k + r) * HW + px);
    }
  };
  auto store_step = [&](const float4 (&stg)[NIT][4], int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int e = tid + NT * i;
      if (e < NBLK) {
        const int kq = e & 7, pq = e >> 3;
        const float4* v = stg[i];
        const f32x4 col[4] = {f32x4{v[0].x, v[1].x, v[2].x, v[3].x}, f32x4{v[0].y, v[1].y, v[2].y, v[3].y},
                              f32x4{v[0].z, v[1].z, v[2].z, v[3].z}, f32x4{v[0].w, v[1].w, v[2].w, v[3].w}};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          uint2 hh, ll;
          split4x(col[j], hh, ll);  // loaded x: the 3-VALU split (common.h split2x)
          rng = range_acc(rng, col[j]);
          h16_t* d = Pl + (buf * 2) * PPL + (4 * pq + j) * PPS + 4 * kq;
          *reinterpret_cast<uint2*>(d) = hh;
          *reinterpret_cast<uint2*>(d + PPL) = ll;
        }
      }
    }
  };
  // weight fragments (A operand): output rows co + 16 (wid RBW + rb) + l15, k = 32 s + 8g .. +7, fragment-major planes
  const int nk32 = C / 32;
  const long pst = (long)C * C;
  const int rbase = (co >> 4) + wid * RBW;
  auto wfrag = [&](int rb, int s, int pl) {
    return *reinterpret_cast<const f16x8_t*>(wp + pl * pst + ((long)((rbase + rb) * nk32 + s) * 64 + lane) * 8);
  };
  f32x4 acc[RBW][NCB];
#pragma unroll
  for (int rb = 0; rb < RBW; ++rb)
#pragma unroll
    for (int j = 0; j < NCB; ++j) acc[rb][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f16x8_t wr[D][RBW][2];
  auto load_w = [&](f16x8_t (&w)[RBW][2], int s) __attribute__((always_inline)) {
#pragma unroll
    for (int rb = 0; rb < RBW; ++rb) {
      w[rb][0] = wfrag(rb, s, 0);
      w[rb][1] = wfrag(rb, s, 1);
    }
  };
  // ring slot i holds step s with s % D == i; unconditional (clamped) loads past the last step
#pragma unroll
  for (int i = 0; i < D; ++i) {
    load_step(xr[i], i < nk32 ? i : nk32 - 1);
    load_w(wr[i], i < nk32 ? i : nk32 - 1);
  }
  store_step(xr[0], 0);
  for (int s0 = 0; s0 < nk32; s0 += D) {
#pragma unroll
    for (int i = 0; i < D; ++i) {
      const int s = s0 + i;
      if (s < nk32) {
        const int buf = s & 1;
        __syncthreads();  // step s's planes stored; every wave is done with step s - 1's buffer
        const h16_t* b0 = Pl + (buf * 2) * PPL + l15 * PPS + 8 * g;
#pragma unroll
        for (int j = 0; j < NCB; ++j) {
          const f16x8_t xh = *reinterpret_cast<const f16x8_t*>(b0 + j * 16 * PPS);
          const f16x8_t xl = *reinterpret_cast<const f16x8_t*>(b0 + j * 16 * PPS + PPL);
#pragma unroll
          for (int rb = 0; rb < RBW; ++rb) {
            f32x4 c = mfma16(wr[i][rb][1], xh, acc[rb][j]);
            c = mfma16(wr[i][rb][0], xl, c);
            acc[rb][j] = mfma16(wr[i][rb][0], xh, c);
          }
        }
        if (s + 1 < nk32) store_step(xr[(i + 1) % D], buf ^ 1);
        const int sn = s + D < nk32 ? s + D : nk32 - 1;
        load_step(xr[i], sn);
        load_w(wr[i], sn);
      }
    }
  }
  __syncthreads();  // the staging planes are free: the SiLU tile takes the region
  // lane (g, l15) of (rb, j): channel co + 16 (wid RBW + rb) + 4g + r, pixel 16 j + l15
#pragma unroll
  for (int rb = 0; rb < RBW; ++rb) {
    const int cl = 16 * (wid * RBW + rb) + 4 * g;
    const f32x4 bias = *reinterpret_cast<const f32x4*>(bp + co + cl);
#pragma unroll
    for (int j = 0; j < NCB; ++j) {
      const int px = j * 16 + l15;
#pragma unroll
      for (int r = 0; r < 4; ++r) Tt[(cl + r) * HWP + px] = silu_fast_(acc[rb][j][r] * (1.0f / WSC) + bias[r]);
    }
  }
  __syncthreads();
  // pooled tokens: thread (c = tid % CH, column group tid / CH) averages its channel's bins in row order (as the
  // reference's CPU pooling) for the columns w = tid / CH + (NT / CH) i of every area of the group
  constexpr int NCG = NT / CH;  // column groups
  const int c = tid % CH;
  const float* trow = Tt + c * HWP - pg.r0 * W;
  float* Sb = S + (long)img * A * W * C + co + c;
  for (int a = pg.a0; a < pg.a1; ++a) {
    const int r0 = (a * H) / A, r1 = ((a + 1) * H + A - 1) / A;
    const float cnt = (float)(r1 - r0);
    for (int w = tid / CH; w < W; w += NCG) {
      float sum = 0.f;
      for (int r = r0; r < r1; ++r) sum += trow[r * W + w];
      Sb[(long)(a * W + w) * C] = sum / cnt;
    }
  }
  range_report(range_flag, rng);
  if (prep_flag && range_flag && blockIdx.x == 0 && threadIdx.x == 0 && *prep_flag) *range_flag = 1u;
}

// Weight preparation, one wave per output row: rows [0, 3C) = in_proj with the LN affine folded (W' = W diag(gamma),
// b' = b + W beta), rows [3C, 4C) = the proj 1x1 conv (BN folded by the caller); both split into fp16 planes (x64,
// fragment-major: element (n, k) of [N][C] at ((n/16 * C/32 + k/32) * 64 + (k%32)/8 * 16 + n%16) * 8 + k%8)
__global__ __launch_bounds__(256) void a2_prep_kernel(const float* __restrict__ w, const float* __restrict__ bias,
                                                      const float* __restrict__ ln_w, const float* __restrict__ ln_b,
                                                      const float* __restrict__ pw, int C, h16_t* __restrict__ planes,
                                                      float* __restrict__ bf, h16_t* __restrict__ pplanes,
                                                      unsigned* range_flag, unsigned* prep_flag) {
  const int lane = threadIdx.x & 63;
  int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= 4 * C) return;
  const bool proj = n >= 3 * C;
  if (proj) n -= 3 * C;
  const float* row = (proj ? pw : w) + (long)n * C;
  const long N = proj ? (long)C : 3L * C;
  h16_t* dst = proj ? pplanes : planes;
  float bacc = 0.f, wmax = 0.f;
  for (int k = lane; k < C; k += 64) {
    const float wv = row[k];
    float v = wv * WSC;
    if (!proj) {
      bacc = fmaf(wv, ln_b[k], bacc);
      v = wv * ln_w[k] * WSC;
    }
    const _Float16 hh = (_Float16)v;
    const _Float16 ll = (_Float16)(v - (float)hh);
    wmax = nmax_(wmax, fabsf(v));
    const long fi = ((long)((n >> 4) * (C >> 5) + (k >> 5)) * 64 + (((k & 31) >> 3) << 4) + (n & 15)) * 8 + (k & 7);
    dst[fi] = __builtin_bit_cast(h16_t, hh);
    dst[N * C + fi] = __builtin_bit_cast(h16_t, ll);
  }
  if (!proj) {
    bacc = wave_sum(bacc);
    if (lane == 0) bf[n] = bias[n] + bacc;
  }
  range_report(range_flag, wmax);
  range_report(prep_flag, wmax);
}

}  // namespace a2f
}  // namespace ys

using namespace ys;

// the fused kernels (default; the test hook below runs the decomposed GEMM path on the same split products)
static int g_a2_fused = 1;
static bool a2_fused_env() { return g_a2_fused != 0; }
// Test hook: A2 through the fused kernels (1) or the decomposed path (0); returns the previous state.
YS_EXPORT int yolosod_debug_set_a2_fused(int on) {
  const int prev = a2_fused_env() ? 1 : 0;
  g_a2_fused = on ? 1 : 0;
  return prev;
}

// the LN / QKV / attention kernel's shapes: head dim 64, C a multiple of 64 (<= 1024), L = areas * W <= 160
bool yolosod_a2_fused_ok(int C, int num_heads, int L) {
  const bool on = a2_fused_env();
  return on && num_heads > 0 && C == a2f::HD * num_heads && C % a2f::KS == 0 && C <= 1024 && L >= 1 &&
         L <= a2f::MAXTB * 16;
}

size_t yolosod_a2_fused_prep_bytes(int C) {
  Sizer s;
  s.take<h16_t>((size_t)2 * 3 * C * C);  // in_proj planes (LN folded)
  s.take<float>((size_t)3 * C);          // folded in_proj bias
  s.take<h16_t>((size_t)2 * C * C);      // proj planes
  s.take<unsigned>(1);                   // the weights' split-range word
  return s.off;
}

struct A2Prep {
  h16_t* planes;
  float* bf;
  h16_t* pplanes;
  unsigned* pflag;
};
static bool a2f_carve(void* buf, size_t bytes, int C, A2Prep& q) {
  Carver cv(buf, bytes);
  q.planes = cv.take<h16_t>((size_t)2 * 3 * C * C);
  q.bf = cv.take<float>((size_t)3 * C);
  q.pplanes = cv.take<h16_t>((size_t)2 * C * C);
  q.pflag = cv.take<unsigned>(1);
  return q.pflag != nullptr;
}

int yolosod_a2_fused_prepare(int C, const float* proj_w, const float* ln_w, const float* ln_b, const float* in_w,
                             const float* in_b, void* prep, size_t prep_bytes, hipStream_t st) {
  A2Prep q;
  YS_CHECK_ARG(a2f_carve(prep, prep_bytes, C, q), "a2 prep: buffer too small (%zu)", prep_bytes);
  if (hipMemsetAsync(q.pflag, 0, sizeof(unsigned), st) != hipSuccess) {
    set_error("a2 prep: flag reset failed");
    return -1;
  }
  hipLaunchKernelGGL(a2f::a2_prep_kernel, dim3((4 * C + 3) / 4), dim3(256), 0, st, in_w, in_b, ln_w, ln_b, proj_w, C,
                     q.planes, q.bf, q.pplanes, range_flag_dev(), q.pflag);
  YS_CHECK_LAUNCH("a2_prep");
  return 0;
}

// Area groups of the proj + SiLU + pooling kernel: the fewest groups whose row bands fit `cap` pixels (0: none fit).
// Groups > 1 need W % 4 == 0 (16-byte aligned band starts).
static int g_a2_pool_cap = 208;  // pixels per group the launcher aims for (208: 2 workgroups / CU)
static int a2_pool_cap() { return g_a2_pool_cap; }
static int a2_pool_groups(int H, int W, int A, int cap, int* max_px) {
  for (int G = 1; G <= A; ++G) {
    if (G > 1 && W % 4 != 0) break;
    int mx = 0;
    for (int q = 0; q < G; ++q) {
      const a2f::PoolGroup g = a2f::pool_group(q, G, A, H);
      const int px = (g.r1 - g.r0) * W;
      mx = px > mx ? px : mx;
    }
    if (mx <= cap && mx % 4 == 0) {
      if (max_px) *max_px = mx;
      return G;
    }
  }
  return 0;
}
// Test hook: pixels per area group of the proj / pool kernel (0: the default); returns the previous cap.
YS_EXPORT int yolosod_debug_set_a2_pool_px(int px) {
  const int prev = a2_pool_cap();
  g_a2_pool_cap = (px <= 0 || px > a2f::PMAXHW) ? 208 : px;
  return prev;
}

// the proj + SiLU + pooling kernel's shapes: C a multiple of 64, every area group's rows within the LDS tile
bool yolosod_a2_proj_pool_ok(int C, int H, int W, int A) {
  const bool on = a2_fused_env();
  return on && C % 64 == 0 && C <= 1024 && A > 0 &&
         (a2_pool_groups(H, W, A, a2_pool_cap(), nullptr) > 0 || a2_pool_groups(H, W, A, a2f::PMAXHW, nullptr) > 0);
}

// The wide proj / pool kernel (default; the test hook keeps the 64-channel one): its (column blocks, row
// blocks per workgroup) instances and the configuration for a shape - the first instance whose area groups fit and
// that gives >= 256 workgroups, else the one with the most workgroups (0: none fits).
static int g_a2_pool_wide = 1;
static bool a2_pool_wide_env() { return g_a2_pool_wide != 0; }
// Test hook: the wide proj / pool kernel on (1) or off (0); returns the previous state.
YS_EXPORT int yolosod_debug_set_a2_pool_wide(int on) {
  const int prev = a2_pool_wide_env() ? 1 : 0;
  g_a2_pool_wide = on ? 1 : 0;
  return prev;
}
struct A2PoolWide {
  int ncb, nrb, G;
};
static A2PoolWide a2_pool_wide_cfg(int B, int C, int H, int W, int A) {
  static const int inst[][2] = {{7, 16}, {13, 8}, {7, 8}};
  A2PoolWide best{0, 0, 0};
  long best_n = 0;
  if (!a2_pool_wide_env()) return best;
  for (const auto& in : inst) {
    if (C % (16 * in[1])) continue;
    int mx = 0;
    const int G = a2_pool_groups(H, W, A, in[0] * 16, &mx);
    if (G == 0) continue;
    const long n = (long)B * G * (C / (16 * in[1]));
    if (n >= 256) return A2PoolWide{in[0], in[1], G};
    if (n > best_n) {
      best_n = n;
      best = A2PoolWide{in[0], in[1], G};
    }
  }
  return best;
}

// x -> S (token-major pooled SiLU(proj x + bp)). Returns < 0 on error.
int yolosod_a2_proj_pool_run(const float* x, const float* proj_b, float* S, int B, int C, int H, int W, int A,
                             const void* prep, size_t prep_bytes, hipStream_t st) {
  A2Prep q;
  YS_CHECK_ARG(a2f_carve(const_cast<void*>(prep), prep_bytes, C, q), "a2: prepared block too small");
  YS_CHECK_ARG(yolosod_a2_proj_pool_ok(C, H, W, A), "a2: proj/pool shape C=%d %dx%d A=%d not fused", C, H, W, A);
  YS_CHECK_ARG(((uintptr_t)x & 15) == 0, "a2: x must be 16-byte aligned");
  const A2PoolWide wc = a2_pool_wide_cfg(B, C, H, W, A);
  if (wc.G > 0) {
    const long nw = (long)B * wc.G * (C / (16 * wc.nrb));
    YS_CHECK_ARG(nw < (1L << 31), "a2: too many workgroups");
#define YS_A2PW(N, R)                                                                                               \
  if (wc.ncb == N && wc.nrb == R) {                                                                                 \
    hipLaunchKernelGGL((a2f::a2_proj_pool_wide_kernel<N, R>), dim3((unsigned)nw), dim3(512), 0, st, x, q.pplanes,  \
                       proj_b, S, C, H, W, A, wc.G, range_flag_dev(), q.pflag);                                     \
    YS_CHECK_LAUNCH("a2_proj_pool_wide");                                                                            \
    return 0;                                                                                                        \
  }
    YS_A2PW(7, 16) YS_A2PW(13, 8) YS_A2PW(7, 8)
#undef YS_A2PW
  }
  int mx = 0;
  int G = a2_pool_groups(H, W, A, a2_pool_cap(), &mx);
  if (G == 0) G = a2_pool_groups(H, W, A, a2f::PMAXHW, &mx);
  const long nwg = (long)B * (C / 64) * G;
  YS_CHECK_ARG(nwg < (1L << 31), "a2: too many workgroups");
  const int ncb = (mx + 15) / 16;
#define YS_A2P(N, NW)                                                                                                \
  if (ncb <= N) {                                                                                                     \
    hipLaunchKernelGGL((a2f::a2_proj_pool_kernel<N, NW>), dim3((unsigned)nwg), dim3(64 * NW), 0, st, x, q.pplanes,   \
                       proj_b, S, C, H, W, A, G, range_flag_dev(), q.pflag);                                                 \
    YS_CHECK_LAUNCH("a2_proj_pool");                                                                                  \
    return 0;                                                                                                         \
  }
  YS_A2P(4, 4) YS_A2P(8, 4) YS_A2P(13, 4) YS_A2P(16, 8) YS_A2P(25, 8)
#undef YS_A2P
  YS_CHECK_ARG(false, "a2: %dx%d pixels too many for the proj/pool kernel", H, W);
  return -1;
}

// LN -> QKV -> attention of all (image, head) pairs: S / stats -> O ([B*L][C]). Returns < 0 on error.
int yolosod_a2_fused_run(const float* S, const float* stats, float* O, int B, int L, int C, int num_heads,
                         const void* prep, size_t prep_bytes, hipStream_t st) {
  A2Prep q;
  YS_CHECK_ARG(a2f_carve(const_cast<void*>(prep), prep_bytes, C, q), "a2: prepared block too small");
  YS_CHECK_ARG(yolosod_a2_fused_ok(C, num_heads, L), "a2: shape C=%d heads=%d L=%d not fused", C, num_heads, L);
  const long nwg = (long)B * num_heads;
  YS_CHECK_ARG(nwg < (1L << 31), "a2: too many (image, head) pairs");
  a2f::Args a{S, stats, q.planes, q.bf, O, L, C, 1.0f / sqrtf((float)a2f::HD), range_flag_dev(), q.pflag};
  const int ntb = (L + 15) / 16;
#define YS_A2F(N)                                                                                         \
  case N:                                                                                                 \
    hipLaunchKernelGGL((a2f::a2_qkv_attn_kernel<N>), dim3((unsigned)nwg), dim3(512), 0, st, a); \
    break;
  switch (ntb) {
    YS_A2F(1) YS_A2F(2) YS_A2F(3) YS_A2F(4) YS_A2F(5) YS_A2F(6) YS_A2F(7) YS_A2F(8) YS_A2F(9) YS_A2F(10)
    default: YS_CHECK_ARG(false, "a2: L=%d too long for the fused kernel", L);
  }
#undef YS_A2F
  YS_CHECK_LAUNCH("a2_qkv_attn");
  return 0;
}
