// A2_Attn's LayerNorm -> QKV projection -> multi-head attention in one kernel per (image, head), on the fp16 matrix
// cores at fp32 accuracy (the two-term split of swin_x3.hip: v = h + l, a.b ~ ah.bh + ah.bl + al.bh).
//
// Reference: ultralytics/nn/modules/a2_attn.py:50-53 - seq_norm = layer_norm(seq); attention(seq_norm, seq_norm,
// seq_norm) with nn.MultiheadAttention (batch_first): q, k, v = seq_norm @ W_in^T + b_in split in three; per head
// softmax(q k^T / sqrt(64)) v. The out-projection of the MHA is folded with the output 1x1 conv (A2_Attn._fused_out)
// and runs as the following token GEMM; the pooling before it is a2_pool_tokens_kernel.
//
// Why one kernel: the decomposed path wrote the normalised tokens, then Q/K/V [tokens][3C] (31 MB at bs 32) to HBM
// and read them back in the attention kernel, over three launches. Here one 256-thread workgroup per (image, head)
// keeps everything of its head on chip:
//   1. K loop over the C input channels in 32-wide steps: the step's slice of the pooled tokens [L][32] is read from
//      HBM / L2, normalised with the per-token (mean, rstd) of row_stats_kernel (the LN affine is folded into the
//      prepared weights: W' = W diag(gamma), b' = b + W beta) and stored as two fp16 planes in LDS (double-buffered);
//      wave w owns head-local column block w of Q, K and V (16 output dims each) for all L tokens - its weight
//      fragments stream from L2 in the fragment-major layout of the prep kernel, one step ahead.
//   2. Q and K go to LDS as [token][d] planes, V as V^T [d][token] planes (computed with the operands swapped, so a
//      lane holds 4 consecutive tokens of one dim).
//   3. Attention: wave w takes query blocks w, w+4, w+8: S^T = K Q^T per 16-key block (the Q fragments read with the
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
constexpr int KS = 32;          // k step
constexpr int PSA = KS + 8;     // activation plane row stride (halves): 5 16-byte quads, conflict-free b128 reads
constexpr int PSQ = HD + 8;     // Q / K plane row stride
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
__global__ __launch_bounds__(256, 1) void a2_qkv_attn_kernel(Args p) {
  constexpr int NL = NTB * 16;          // padded tokens
  constexpr int APL = NL * PSA;         // activation plane (halves)
  constexpr int QPL = NL * PSQ;         // Q / K plane
  constexpr int PSV = NL + 8;           // V^T row stride
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
  const int C = p.C, L = p.L;
  const int heads = C / HD;
  // XCD-aware: the heads of one image run on one XCD (they read the same pooled tokens from its L2)
  const int nblk = gridDim.x;
  const int wg = (nblk & 7) ? (int)blockIdx.x : (int)(blockIdx.x & 7) * (nblk >> 3) + (int)(blockIdx.x >> 3);
  const int img = wg / heads, h = wg - img * heads;
  float rng = 0.f;

  const float* Sb = p.S + (long)img * L * C;
  for (int t = tid; t < NL; t += 256) {
    const float2 v = t < L ? *reinterpret_cast<const float2*>(p.stats + 2 * ((long)img * L + t)) : make_float2(0.f, 0.f);
    st[t] = v;
  }
  // this thread's staging items: token rows of the 32-wide k slice as float4 (NL * 8 float4 per step)
  constexpr int NIT = (NL * 8 + 255) / 256;
  float4 stg[NIT];
  auto load_step = [&](int s) {
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int e = tid + 256 * i;
      const int t = e >> 3, q = e & 7;
      stg[i] = (e < NL * 8 && t < L) ? *reinterpret_cast<const float4*>(Sb + (long)t * C + KS * s + 4 * q)
                                     : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_step = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int e = tid + 256 * i;
      if (e < NL * 8) {
        const int t = e >> 3, q = e & 7;
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
  // weight fragments of this wave's column block w of Q, K, V (rows h*64 + 16w + [0,16) of each third)
  const int nsteps = C / KS;
  const long pst = (long)3 * C * C;  // plane stride
  int nbr[3];
#pragma unroll
  for (int m = 0; m < 3; ++m) nbr[m] = (m * C + h * HD) / 16 + wid;
  auto wfrag = [&](int m, int s, int pl) {
    return *reinterpret_cast<const f16x8_t*>(p.w + pl * pst + ((long)(nbr[m] * nsteps + s) * 64 + lane) * 8);
  };
  f16x8_t wc[3][2], wn[3][2];
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    wc[m][0] = wfrag(m, 0, 0);
    wc[m][1] = wfrag(m, 0, 1);
  }
  // accumulators: Q, K (lane: token tb*16 + l15, dims 16w + 4g + r) and V swapped (lane: dim 16w + l15, tokens
  // tb*16 + 4g + r); start from 64 b'
  f32x4 acc[3][NTB];
  {
    const f32x4 bq = *reinterpret_cast<const f32x4*>(p.b + h * HD + 16 * wid + 4 * g) * WSC;
    const f32x4 bk = *reinterpret_cast<const f32x4*>(p.b + C + h * HD + 16 * wid + 4 * g) * WSC;
    const float bv = p.b[2 * C + h * HD + 16 * wid + l15] * WSC;
#pragma unroll
    for (int tb = 0; tb < NTB; ++tb) {
      acc[0][tb] = bq;
      acc[1][tb] = bk;
      acc[2][tb] = f32x4{bv, bv, bv, bv};
    }
  }
  load_step(0);
  __syncthreads();  // stats in LDS
  store_step(0);
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    if (s + 1 < nsteps) {
      load_step(s + 1);
#pragma unroll
      for (int m = 0; m < 3; ++m) {
        wn[m][0] = wfrag(m, s + 1, 0);
        wn[m][1] = wfrag(m, s + 1, 1);
      }
    }
    __syncthreads();  // step s's planes stored; every wave is done with step s - 1's buffer
    const h16_t* a0 = Ab + (buf * 2) * APL + l15 * PSA + 8 * g;
#pragma unroll
    for (int tb = 0; tb < NTB; ++tb) {
      const f16x8_t xh = *reinterpret_cast<const f16x8_t*>(a0 + tb * 16 * PSA);
      const f16x8_t xl = *reinterpret_cast<const f16x8_t*>(a0 + tb * 16 * PSA + APL);
#pragma unroll
      for (int m = 0; m < 2; ++m) {  // Q, K: weights as the A operand (rows = dims), tokens as B
        f32x4 c = mfma16(wc[m][1], xh, acc[m][tb]);
        c = mfma16(wc[m][0], xl, c);
        acc[m][tb] = mfma16(wc[m][0], xh, c);
      }
      {  // V: tokens as the A operand, weights as B (lane: 4 consecutive tokens of one dim)
        f32x4 c = mfma16(xh, wc[2][1], acc[2][tb]);
        c = mfma16(xl, wc[2][0], c);
        acc[2][tb] = mfma16(xh, wc[2][0], c);
      }
    }
    if (s + 1 < nsteps) {
      store_step(buf ^ 1);
#pragma unroll
      for (int m = 0; m < 3; ++m) {
        wc[m][0] = wn[m][0];
        wc[m][1] = wn[m][1];
      }
    }
  }
  __syncthreads();  // every wave is done with the activation planes (Q / K / V^T reuse the region)
  // Q, K -> [token][d] planes, V -> V^T [d][token] planes (all x64); padded tokens hold finite values
#pragma unroll
  for (int tb = 0; tb < NTB; ++tb) {
    const int tok = tb * 16 + l15;
    uint2 hh, ll;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const f32x4 v = acc[m][tb];
      rng = range_acc(rng, v);
      split4(v, hh, ll);
      h16_t* d = (m == 0 ? Qp : Kp) + tok * PSQ + 16 * wid + 4 * g;
      *reinterpret_cast<uint2*>(d) = hh;
      *reinterpret_cast<uint2*>(d + QPL) = ll;
    }
    rng = range_acc(rng, acc[2][tb]);
    split4(acc[2][tb], hh, ll);
    h16_t* d = Vt + (16 * wid + l15) * PSV + tb * 16 + 4 * g;
    *reinterpret_cast<uint2*>(d) = hh;
    *reinterpret_cast<uint2*>(d + VPL) = ll;
  }
  __syncthreads();

  // attention: S^T[key][q] per 16-key block; slot j of lane group g in 32-d step s is head dim 32s + 4g + j (j < 4)
  // or 32s + 16 + 4g + j - 4 for both the Q (B) and K (A) fragments
  const float c2 = p.scale * 1.44269504088896341f * (1.0f / (WSC * WSC));
  for (int qb = wid; qb < NTB; qb += 4) {
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

// in_proj with the LN affine folded, split into fp16 planes (x64, fragment-major: element (n, k) of W' [3C][C] at
// ((n/16 * C/32 + k/32) * 64 + (k%32)/8 * 16 + n%16) * 8 + k%8), folded bias b' = b + W beta; one wave per row
__global__ __launch_bounds__(256) void a2_prep_kernel(const float* __restrict__ w, const float* __restrict__ bias,
                                                      const float* __restrict__ ln_w, const float* __restrict__ ln_b,
                                                      int C, h16_t* __restrict__ planes, float* __restrict__ bf,
                                                      unsigned* range_flag, unsigned* prep_flag) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= 3 * C) return;
  const float* row = w + (long)n * C;
  const long N = 3L * C;
  float bacc = 0.f, wmax = 0.f;
  for (int k = lane; k < C; k += 64) {
    const float wv = row[k];
    bacc = fmaf(wv, ln_b[k], bacc);
    const float v = wv * ln_w[k] * WSC;
    const _Float16 hh = (_Float16)v;
    const _Float16 ll = (_Float16)(v - (float)hh);
    wmax = nmax_(wmax, fabsf(v));
    const long fi = ((long)((n >> 4) * (C >> 5) + (k >> 5)) * 64 + (((k & 31) >> 3) << 4) + (n & 15)) * 8 + (k & 7);
    planes[fi] = __builtin_bit_cast(h16_t, hh);
    planes[N * C + fi] = __builtin_bit_cast(h16_t, ll);
  }
  bacc = wave_sum(bacc);
  if (lane == 0) bf[n] = bias[n] + bacc;
  range_report(range_flag, wmax);
  range_report(prep_flag, wmax);
}

}  // namespace a2f
}  // namespace ys

using namespace ys;

// the fused kernel's shapes: head dim 64, C a multiple of 64 (<= 1024), L = areas * W <= 160
bool yolosod_a2_fused_ok(int C, int num_heads, int L) {
  static const bool on = [] { const char* e = getenv("YOLOSOD_A2_FUSED"); return !(e && e[0] == '0'); }();
  return on && num_heads > 0 && C == a2f::HD * num_heads && C <= 1024 && L >= 1 && L <= a2f::MAXTB * 16;
}

size_t yolosod_a2_fused_prep_bytes(int C) {
  Sizer s;
  s.take<h16_t>((size_t)2 * 3 * C * C);
  s.take<float>((size_t)3 * C);
  s.take<unsigned>(1);
  return s.off;
}

static bool a2f_carve(void* buf, size_t bytes, int C, h16_t*& planes, float*& bf, unsigned*& pflag) {
  Carver cv(buf, bytes);
  planes = cv.take<h16_t>((size_t)2 * 3 * C * C);
  bf = cv.take<float>((size_t)3 * C);
  pflag = cv.take<unsigned>(1);
  return pflag != nullptr;
}

int yolosod_a2_fused_prepare(int C, const float* ln_w, const float* ln_b, const float* in_w, const float* in_b,
                             void* prep, size_t prep_bytes, hipStream_t st) {
  h16_t* planes;
  float* bf;
  unsigned* pflag;
  YS_CHECK_ARG(a2f_carve(prep, prep_bytes, C, planes, bf, pflag), "a2 prep: buffer too small (%zu)", prep_bytes);
  if (hipMemsetAsync(pflag, 0, sizeof(unsigned), st) != hipSuccess) {
    set_error("a2 prep: flag reset failed");
    return -1;
  }
  hipLaunchKernelGGL(a2f::a2_prep_kernel, dim3((3 * C + 3) / 4), dim3(256), 0, st, in_w, in_b, ln_w, ln_b, C, planes,
                     bf, range_flag_dev(), pflag);
  YS_CHECK_LAUNCH("a2_prep");
  return 0;
}

// LN -> QKV -> attention of all (image, head) pairs: S / stats -> O ([B*L][C]). Returns < 0 on error.
int yolosod_a2_fused_run(const float* S, const float* stats, float* O, int B, int L, int C, int num_heads,
                         const void* prep, size_t prep_bytes, hipStream_t st) {
  h16_t* planes;
  float* bf;
  unsigned* pflag;
  YS_CHECK_ARG(a2f_carve(const_cast<void*>(prep), prep_bytes, C, planes, bf, pflag), "a2: prepared block too small");
  YS_CHECK_ARG(yolosod_a2_fused_ok(C, num_heads, L), "a2: shape C=%d heads=%d L=%d not fused", C, num_heads, L);
  const long nwg = (long)B * num_heads;
  YS_CHECK_ARG(nwg < (1L << 31), "a2: too many (image, head) pairs");
  a2f::Args a{S, stats, planes, bf, O, L, C, 1.0f / sqrtf((float)a2f::HD), range_flag_dev(), pflag};
  const int ntb = (L + 15) / 16;
#define YS_A2F(N)                                                                                         \
  case N:                                                                                                 \
    hipLaunchKernelGGL((a2f::a2_qkv_attn_kernel<N>), dim3((unsigned)nwg), dim3(256), 0, st, a); \
    break;
  switch (ntb) {
    YS_A2F(1) YS_A2F(2) YS_A2F(3) YS_A2F(4) YS_A2F(5) YS_A2F(6) YS_A2F(7) YS_A2F(8) YS_A2F(9) YS_A2F(10)
    default: YS_CHECK_ARG(false, "a2: L=%d too long for the fused kernel", L);
  }
#undef YS_A2F
  YS_CHECK_LAUNCH("a2_qkv_attn");
  return 0;
}
