// Fused SwinBlock for the wide P4 instance (L9: C = 256, 4 heads of 64, 7x7 windows, MLP hidden 2C).
//
// One 512-thread workgroup (8 waves, 2 per SIMD, up to 256 VGPRs each) processes one window; the window's 49
// tokens stay in LDS from the depthwise conv to the final pw1x1+BN+SiLU+residual, so HBM sees read x (+ halo)
// once and write y once - the decomposed path moved ~1.7 GB of token-major scratch per call at 640^2 bs=32.
// At C = 256 the whole QKV tile (49 x 768) does not fit next to the residual stream, so:
//   * attention runs on head pairs: QKV of two heads (49 x 384) -> S^T / softmax / O^T per (head, 16-query
//     block) wave -> the out-projection's partial product over those 128 input channels is accumulated in
//     registers (the residual stream must stay LN1's input until every head has read it);
//   * the MLP runs on two hidden chunks of 256: GELU(LN2(T) W1_chunk^T) -> LDS -> MLP2 partial accumulated in
//     registers; T += the accumulators at the end;
//   * weights (3 MB per window, L2-resident) are streamed per wave in 8-k chunks with one chunk of lookahead.
// Token rows 0..47 are three 16-row MFMA blocks; token 48 is computed on the VALU from the same weight fragments
// (see swin_fused.hip), keys 0..47 on MFMA and key 48 as a rank-1 term.
//
// Stages (ultralytics/nn/modules/blocks_transformer.py): dw3x3 (:160) + zero pad + partition (:31-46) -> LN1
// (:112) -> MHA in_proj / softmax(QK^T/sqrt(hd)) V / out_proj + residual (:115-119) -> LN2 -> Linear-GELU-Linear +
// residual (:92-98,122) -> window reverse + crop (:125-129) -> x + SiLU(BN(pw1x1)) (:166-171).
#include "common.h"
#include <math.h>
#include <stdlib.h>

namespace ys {

namespace wide {

constexpr int C = 256;
constexpr int HD = 64;
constexpr int ROWS = 49;
constexpr int XR = 48;          // VALU token row
constexpr int LT = C + 4;       // residual stream row stride (== 4 mod 64: conflict-free b128 row reads)
constexpr int LQ2 = 3 * 128 + 4;  // QKV of a head pair [q(128) | k(128) | v(128)]
constexpr int LHC = 256 + 4;    // MLP hidden chunk
constexpr int HPW = 12;         // halo row stride
constexpr int HALF = 128;       // channels per halo half
constexpr int WK_ELEMS = ROWS * LQ2;
static_assert(54 * ((HALF + 5) / 6) * HPW <= WK_ELEMS && ROWS * LHC <= WK_ELEMS, "work region");
constexpr int NT = 512;         // threads

struct Args {
  const float* x;
  float* y;
  int B, H, W, nWx, nWin;
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
__device__ __forceinline__ float group4_sum(float v) { return xor32_sum(xor16_sum(v)); }
__device__ __forceinline__ float comp(const float4& v, int c) { return c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w; }

// Accumulate, for NJ weight rows per lane (wrow[j] -> W[row_j][kbase + g*K/4 ...], row_j = out column of lane l15):
//   !TRANS: acc[rb][j] += A'[token rows rb*16 + ..][K] . W[row_j][K]   (D[token][col])
//    TRANS: acc[rb][j] += W[row_j][K] . A'[token rows]^T                (D[col][token])
// and ext[j] += the lane's partial of A'[48] . W[row_j] (caller sums over the lane groups once at the end).
// MFMA k permuted: lane group g owns k in [g*K/4, (g+1)*K/4); W fragments streamed in chunks of 8 k per group
// (2 float4 per j) with one chunk of lookahead. A: LDS [ROWS][lda] (+ LayerNorm from stats / LDS params).
template <int K, int NJ, bool LN, bool TRANS>
__device__ __forceinline__ void gemm_stream(const float* __restrict__ As, int lda, const float* const (&wrow)[NJ],
                                            f32x4 (&acc)[3][NJ], float (&ext)[NJ], const float* stats,
                                            const float* lnw, const float* lnb, int lane) {
  constexpr int KQ = K / 4;
  constexpr int CK = 2;  // float4 per j per chunk
  constexpr int NCH = KQ / (4 * CK);
  const int l15 = lane & 15, g = lane >> 4;
  const float* arow[4];
  float rs[4], nmr[4];  // LN: A' = (a*rs - mu*rs) * w + b, two packed FMAs per pair of elements
#pragma unroll
  for (int rb = 0; rb < 4; ++rb) {
    const int r = rb < 3 ? rb * 16 + l15 : XR;
    arow[rb] = As + r * lda + g * KQ;
    if (LN) {
      rs[rb] = stats[2 * r + 1];
      nmr[rb] = -stats[2 * r] * rs[rb];
    }
  }
  float4 wb0[NJ][CK], wb1[NJ][CK];
  auto load_chunk = [&](float4 (&wb)[NJ][CK], int ch) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int u = 0; u < CK; ++u) wb[j][u] = *reinterpret_cast<const float4*>(wrow[j] + 4 * CK * ch + 4 * u);
  };
  auto mma_chunk = [&](const float4 (&wb)[NJ][CK], int ch) {
#pragma unroll
    for (int u = 0; u < CK; ++u) {
      const int ko = 4 * CK * ch + 4 * u;
      float4 a[4];
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) a[rb] = *reinterpret_cast<const float4*>(arow[rb] + ko);
      if (LN) {
        const float4 w = *reinterpret_cast<const float4*>(lnw + g * KQ + ko);
        const float4 bb = *reinterpret_cast<const float4*>(lnb + g * KQ + ko);
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          const f32x2 r2 = {rs[rb], rs[rb]}, m2 = {nmr[rb], nmr[rb]};
          const f32x2 lo = __builtin_elementwise_fma(
              __builtin_elementwise_fma(f32x2{a[rb].x, a[rb].y}, r2, m2), f32x2{w.x, w.y}, f32x2{bb.x, bb.y});
          const f32x2 hi = __builtin_elementwise_fma(
              __builtin_elementwise_fma(f32x2{a[rb].z, a[rb].w}, r2, m2), f32x2{w.z, w.w}, f32x2{bb.z, bb.w});
          a[rb] = make_float4(lo.x, lo.y, hi.x, hi.y);
        }
      }
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int rb = 0; rb < 3; ++rb)
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            const float av = comp(a[rb], c), bv = comp(wb[j][u], c);
            acc[rb][j] = TRANS ? mfma4(bv, av, acc[rb][j]) : mfma4(av, bv, acc[rb][j]);
          }
#pragma unroll
      for (int j = 0; j < NJ; ++j) ext[j] = dot4_acc(a[3], wb[j][u], ext[j]);
    }
  };
  static_assert(NCH % 2 == 0, "chunk pairs");
  load_chunk(wb0, 0);
  // ping-pong over chunk pairs (rolled: a fully unrolled K loop lets the scheduler hoist every chunk's loads)
#pragma unroll 1
  for (int ch = 0; ch < NCH; ch += 2) {
    load_chunk(wb1, ch + 1);
    mma_chunk(wb0, ch);
    if (ch + 2 < NCH) load_chunk(wb0, ch + 2);
    mma_chunk(wb1, ch + 1);
  }
}

// LayerNorm statistics of rows [0, ROWS) of S[ROWS][LT] over C: 8 lanes per row (512 threads = 64 rows).
__device__ __forceinline__ void row_stats8(const float* S, float* stats, float eps, int tid) {
  const int r = tid >> 3, part = tid & 7;
  const bool valid = r < ROWS;
  float4 v[C / 32];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < C / 32; ++i) {
    v[i] = valid ? *reinterpret_cast<const float4*>(S + r * LT + part * (C / 8) + 4 * i) : make_float4(0.f, 0.f, 0.f, 0.f);
    s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  }
  s = quad_sum(s);
  s += __shfl_xor(s, 4, 64);
  const float mean = s / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < C / 32; ++i) {
    const float a0 = v[i].x - mean, a1 = v[i].y - mean, a2 = v[i].z - mean, a3 = v[i].w - mean;
    q += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
  }
  q = quad_sum(q);
  q += __shfl_xor(q, 4, 64);
  if (part == 0 && valid) {
    stats[2 * r] = mean;
    stats[2 * r + 1] = 1.0f / sqrtf(q / (float)C + eps);
  }
}

__global__ __launch_bounds__(NT, 1) void swin_wide_kernel(Args p) {
  __shared__ __attribute__((aligned(16))) float smem[ROWS * LT + WK_ELEMS + 2 * 64 + 4 * C];
  float* T = smem;                   // residual stream [ROWS][LT]
  float* WK = T + ROWS * LT;         // halo half / QKV of a head pair / MLP hidden chunk
  float* stats = WK + WK_ELEMS;      // [64][2]
  float* lnp = stats + 2 * 64;       // [ln1_w | ln1_b | ln2_w | ln2_b]

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, g = lane >> 4;
  const int H = p.H, W = p.W;
  const long HWl = (long)H * W;

  const long nwin_total = (long)p.B * p.nWin;
  const long per_xcd = (nwin_total + 7) >> 3;
  const long gw = (long)(blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  if (gw >= nwin_total) return;
  const int gwi = __builtin_amdgcn_readfirstlane((int)gw);  // window counts < 2^31 (launcher)
  const int img = gwi / p.nWin, win = gwi - (gwi / p.nWin) * p.nWin;
  const int wy = win / p.nWx, wx = win - (win / p.nWx) * p.nWx;
  const float* xb = p.x + (long)img * C * HWl;
  const int h0 = wy * 7 - 1, w0 = wx * 7 - 1;

  // halo of both channel halves into registers: lane = 9 * row + column (lane 63 idle), so a wave-instruction
  // reads 7 row segments of 9 floats. Row slot s = 7*wid + row < 54 is (channel 6i + s/9, patch row s%9) at step
  // i: a lane's byte offset is fixed, the step and the half go into the scalar soffset, and out-of-image lanes
  // get an out-of-range voffset (the buffer load returns 0) - no per-load VALU. Slots 54, 55 idle.
  constexpr int NR = (HALF + 5) / 6;
  constexpr unsigned OOB = 0x80000000u;
  float hv[2][NR];
  const int hl_r = lane / 9, hl_px = lane - (lane / 9) * 9;
  const int hslot = 7 * wid + hl_r;
  {
    const int hcs = hslot / 9, hpy = hslot - (hslot / 9) * 9;
    const int wc = w0 + hl_px, hh = h0 + hpy;
    const bool ok = hl_r < 7 && hslot < 54 && wc >= 0 && wc < W && (unsigned)hh < (unsigned)H;
    const int HWi = H * W;
    const unsigned voff = ok ? (unsigned)((hcs * HWi + hh * W + wc) * 4) : OOB;
    const unsigned vlast = (6 * (NR - 1) + hcs < HALF) ? voff : OOB;
    const unsigned long long xa = (unsigned long long)xb;
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(xa >> 32)) << 32) |
                (unsigned)__builtin_amdgcn_readfirstlane((unsigned)xa)),
        (short)0, __builtin_amdgcn_readfirstlane(C * HWi * 4), 0x00020000);
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)
#pragma unroll
      for (int i = 0; i < NR; ++i)
        hv[hf][i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                  rx, i == NR - 1 ? vlast : voff, (hf * HALF + 6 * i) * HWi * 4, 0));
  }
  {
    static_assert((4 * C) % NT == 0, "LN parameter staging");
    constexpr int NPT = 4 * C / NT;
    float pv[NPT];  // every load first, then the LDS stores
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int e = tid + NT * i;
      const int which = e / C, c = e - which * C;
      const float* src = which == 0 ? p.ln1_w : which == 1 ? p.ln1_b : which == 2 ? p.ln2_w : p.ln2_b;
      pv[i] = src[c];
    }
#pragma unroll
    for (int i = 0; i < NPT; ++i) lnp[tid + NT * i] = pv[i];
  }

  // ---- depthwise 3x3 per channel half: halo -> LDS [c][py][HPW], one output row of 7 tokens per item ----
  const int dc = tid % HALF;
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    float dwk[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) dwk[i] = p.dw[(hf * HALF + dc) * 9 + i];
    if (hf) __syncthreads();  // previous half's dw reads done
    if (hl_r < 7 && hslot < 54) {  // patch row 9*(6i + s/9) + s%9 = 54i + s; rows of channels >= HALF unused
#pragma unroll
      for (int i = 0; i < NR; ++i) WK[(54 * i + hslot) * HPW + hl_px] = hv[hf][i];
    }
    __syncthreads();
    for (int item = tid; item < HALF * 7; item += NT) {
      const int iy = item / HALF;  // item % HALF == dc
      const float* hp = WK + (dc * 9 + iy) * HPW;
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
        T[(iy * 7 + ix) * LT + hf * HALF + dc] = (rowok && wx * 7 + ix < W) ? v : 0.f;
      }
    }
  }
  __syncthreads();

  // ---- LN1 statistics ----
  row_stats8(T, stats, p.ln1_eps, tid);
  __syncthreads();

  // ---- attention on head pairs; out-projection partials accumulated in registers ----
  f32x4 acc_o[3][2];
  float bo_[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) bo_[j] = p.bo[(wid + 8 * j) * 16 + l15];
  float ext_o[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    ext_o[j] = 0.f;
#pragma unroll
    for (int rb = 0; rb < 3; ++rb) acc_o[rb][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll 1
  for (int hp = 0; hp < 2; ++hp) {
    // QKV of heads 2hp, 2hp+1: local column nl = part*128 + within -> in_proj row part*C + hp*128 + within
    {
      f32x4 acc[3][3];
      float ext[3];
      const float* wrow[3];
      int nl[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        nl[j] = (wid + 8 * j) * 16 + l15;
        const int part = nl[j] >> 7, within = nl[j] & 127;
        wrow[j] = p.win + (long)(part * C + hp * 128 + within) * C + g * (C / 4);
        ext[j] = 0.f;
#pragma unroll
        for (int rb = 0; rb < 3; ++rb) acc[rb][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      // biases loaded before the weight stream: after it, each one was an exposed L2 round trip
      float bq[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) bq[j] = p.bin[(nl[j] >> 7) * C + hp * 128 + (nl[j] & 127)];
      gemm_stream<C, 3, true, false>(T, LT, wrow, acc, ext, stats, lnp, lnp + C, lane);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const float bias = bq[j];
        const float e = group4_sum(ext[j]);
#pragma unroll
        for (int rb = 0; rb < 3; ++rb)
#pragma unroll
          for (int r = 0; r < 4; ++r) WK[(rb * 16 + 4 * g + r) * LQ2 + nl[j]] = acc[rb][j][r] + bias;
        if (g == 0) WK[XR * LQ2 + nl[j]] = e + bias;
      }
    }
    __syncthreads();
    // wave = (local head lh, 16-query block qb); O overwrites the wave's own query columns
    {
      const int lh = wid >> 2, qb = wid & 3;
      int qrow = qb * 16 + l15;
      qrow = qrow < XR ? qrow : XR;
      constexpr int DQ = HD / 4;
      const int qo = lh * HD, ko = 128 + lh * HD, vo = 256 + lh * HD;
      f32x4 st[3];
      float s48 = 0.f;
#pragma unroll
      for (int kb = 0; kb < 3; ++kb) st[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < DQ / 4; ++t) {
        const float4 qv = *reinterpret_cast<const float4*>(WK + qrow * LQ2 + qo + g * DQ + 4 * t);
        float4 kv[3];
#pragma unroll
        for (int kb = 0; kb < 3; ++kb)
          kv[kb] = *reinterpret_cast<const float4*>(WK + (kb * 16 + l15) * LQ2 + ko + g * DQ + 4 * t);
        const float4 k48 = *reinterpret_cast<const float4*>(WK + XR * LQ2 + ko + g * DQ + 4 * t);
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int kb = 0; kb < 3; ++kb) st[kb] = mfma4(comp(kv[kb], c), comp(qv, c), st[kb]);
        s48 = dot4_acc(k48, qv, s48);
      }
      // softmax over the 49 keys (lane: keys kb*16 + 4g + r for query l15; key 48 after the group sum) on the raw
      // scores, exp2 with scale*log2(e) folded into one FMA, 1/sum applied to O (per query = per lane)
      const float c2 = p.scale * 1.44269504088896341f;
      const float sv48 = group4_sum(s48);
      float mx = sv48;
#pragma unroll
      for (int kb = 0; kb < 3; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, st[kb][r]);
      mx = xor32_max(xor16_max(mx));
      const float mc = -mx * c2;
      float sum = 0.f;
#pragma unroll
      for (int kb = 0; kb < 3; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __builtin_amdgcn_exp2f(fmaf(st[kb][r], c2, mc));
          st[kb][r] = e;
          sum += e;
        }
      const float e48 = __builtin_amdgcn_exp2f(fmaf(sv48, c2, mc));
      sum += (g == 0) ? e48 : 0.f;
      const float inv = __builtin_amdgcn_rcpf(group4_sum(sum));
      f32x4 o[HD / 16];
#pragma unroll
      for (int db = 0; db < HD / 16; ++db) o[db] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < 3; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float* vrow = WK + (kb * 16 + 4 * g + r) * LQ2 + vo + l15;
#pragma unroll
          for (int db = 0; db < HD / 16; ++db) o[db] = mfma4(vrow[db * 16], st[kb][r], o[db]);
        }
#pragma unroll
      for (int db = 0; db < HD / 16; ++db) {
        const float4 v48 = *reinterpret_cast<const float4*>(WK + XR * LQ2 + vo + db * 16 + 4 * g);
        o[db][0] = fmaf(v48.x, e48, o[db][0]) * inv;
        o[db][1] = fmaf(v48.y, e48, o[db][1]) * inv;
        o[db][2] = fmaf(v48.z, e48, o[db][2]) * inv;
        o[db][3] = fmaf(v48.w, e48, o[db][3]) * inv;
      }
      const int q = qb * 16 + l15;
      if (q < ROWS) {
#pragma unroll
        for (int db = 0; db < HD / 16; ++db)
          *reinterpret_cast<f32x4*>(WK + q * LQ2 + qo + db * 16 + 4 * g) = o[db];
      }
    }
    __syncthreads();
    // out-projection partial over this pair's 128 input channels: acc_o += O_pair Wo[:, hp*128 .. +128]^T
    {
      const float* wrow[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) wrow[j] = p.wo + (long)((wid + 8 * j) * 16 + l15) * C + hp * 128 + g * 32;
      gemm_stream<128, 2, false, false>(WK, LQ2, wrow, acc_o, ext_o, nullptr, nullptr, nullptr, lane);
    }
    __syncthreads();  // WK is overwritten by the next pair's QKV
  }
  // T += O Wo^T + bo
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = (wid + 8 * j) * 16 + l15;
    const float bias = bo_[j];
    const float e = group4_sum(ext_o[j]);
#pragma unroll
    for (int rb = 0; rb < 3; ++rb)
#pragma unroll
      for (int r = 0; r < 4; ++r) T[(rb * 16 + 4 * g + r) * LT + n] += acc_o[rb][j][r] + bias;
    if (g == 0) T[XR * LT + n] += e + bias;
  }
  __syncthreads();

  // ---- LN2 statistics ----
  row_stats8(T, stats, p.ln2_eps, tid);
  __syncthreads();

  // ---- MLP in two hidden chunks of 256; MLP2 partials accumulated in registers ----
  f32x4 acc_m[3][2];
  float ext_m[2];
  float b2_[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) b2_[j] = p.b2[(wid + 8 * j) * 16 + l15];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    ext_m[j] = 0.f;
#pragma unroll
    for (int rb = 0; rb < 3; ++rb) acc_m[rb][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll 1
  for (int ck = 0; ck < 2; ++ck) {
    {
      f32x4 acc[3][2];
      float ext[2];
      const float* wrow[2];
      int nl[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        nl[j] = (wid + 8 * j) * 16 + l15;
        wrow[j] = p.w1 + (long)(ck * 256 + nl[j]) * C + g * (C / 4);
        ext[j] = 0.f;
#pragma unroll
        for (int rb = 0; rb < 3; ++rb) acc[rb][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      float b1_[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) b1_[j] = p.b1[ck * 256 + nl[j]];
      gemm_stream<C, 2, true, false>(T, LT, wrow, acc, ext, stats, lnp + 2 * C, lnp + 3 * C, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float bias = b1_[j];
        const float e = group4_sum(ext[j]);
#pragma unroll
        for (int rb = 0; rb < 3; ++rb)
#pragma unroll
          for (int r = 0; r < 4; r += 2) {
            const f32x2 hv2 = gelu2_fast_(f32x2{acc[rb][j][r], acc[rb][j][r + 1]} + bias);
            WK[(rb * 16 + 4 * g + r) * LHC + nl[j]] = hv2.x;
            WK[(rb * 16 + 4 * g + r + 1) * LHC + nl[j]] = hv2.y;
          }
        if (g == 0) WK[XR * LHC + nl[j]] = gelu_fast_(e + bias);
      }
    }
    __syncthreads();
    {
      const float* wrow[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) wrow[j] = p.w2 + (long)((wid + 8 * j) * 16 + l15) * (2 * C) + ck * 256 + g * 64;
      gemm_stream<256, 2, false, false>(WK, LHC, wrow, acc_m, ext_m, nullptr, nullptr, nullptr, lane);
    }
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = (wid + 8 * j) * 16 + l15;
    const float bias = b2_[j];
    const float e = group4_sum(ext_m[j]);
#pragma unroll
    for (int rb = 0; rb < 3; ++rb)
#pragma unroll
      for (int r = 0; r < 4; ++r) T[(rb * 16 + 4 * g + r) * LT + n] += acc_m[rb][j][r] + bias;
    if (g == 0) T[XR * LT + n] += e + bias;
  }
  __syncthreads();

  // ---- y = x + SiLU(BN(Wpw T^T)) on the valid tokens: D[c][tok], c = cb*16 + 4g + r, tok = tb*16 + l15 ----
  // residual loads / y stores are buffer ops: fixed per-lane voffset (token; channel row 4g of block wid, + l15 for
  // token 48), out-of-image tokens get an out-of-range voffset (loads return 0, stores are dropped), the channel
  // offset ((cb - wid)*16 + r planes) goes into the scalar soffset
  {
    const int HWi = H * W;
    constexpr unsigned OOB = 0x80000000u;
    auto rsrc = [&](const float* base) {
      const unsigned long long a = (unsigned long long)base;
      return __builtin_amdgcn_make_buffer_rsrc(
          (void*)(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(a >> 32)) << 32) |
                  (unsigned)__builtin_amdgcn_readfirstlane((unsigned)a)),
          (short)0, __builtin_amdgcn_readfirstlane(C * HWi * 4), 0x00020000);
    };
    const __amdgpu_buffer_rsrc_t rx = rsrc(xb), ry = rsrc(p.y + (long)img * C * HWl);
    unsigned vtok[3];
#pragma unroll
    for (int tb = 0; tb < 3; ++tb) {
      const int tok = tb * 16 + l15;
      const int iy = tok / 7, ix = tok - iy * 7;
      const int hh = wy * 7 + iy, wc = wx * 7 + ix;
      vtok[tb] = (hh < H && wc < W) ? (unsigned)(((wid * 16 + 4 * g) * HWi + hh * W + wc) * 4) : OOB;
    }
    const unsigned v48 = (wy * 7 + 6 < H && wx * 7 + 6 < W && g == 0)
                             ? (unsigned)(((wid * 16 + l15) * HWi + (wy * 7 + 6) * W + wx * 7 + 6) * 4) : OOB;
    float xr[2][3][4], bsc[2][4], bsh[2][4], x48[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int cb = wid + 8 * j;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        bsc[j][r] = p.bn_scale[cb * 16 + 4 * g + r];
        bsh[j][r] = p.bn_shift[cb * 16 + 4 * g + r];
#pragma unroll
        for (int tb = 0; tb < 3; ++tb)
          xr[j][tb][r] = __builtin_bit_cast(
              float, __builtin_amdgcn_raw_buffer_load_b32(rx, vtok[tb], (128 * j + r) * HWi * 4, 0));
      }
      x48[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, v48, 128 * j * HWi * 4, 0));
    }
    f32x4 acc[3][2];
    float ext[2];
    const float* wrow[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      wrow[j] = p.wpw + (long)((wid + 8 * j) * 16 + l15) * C + g * (C / 4);
      ext[j] = 0.f;
#pragma unroll
      for (int rb = 0; rb < 3; ++rb) acc[rb][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    gemm_stream<C, 2, false, true>(T, LT, wrow, acc, ext, nullptr, nullptr, nullptr, lane);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
#pragma unroll
      for (int tb = 0; tb < 3; ++tb)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          __builtin_amdgcn_raw_buffer_store_b32(
              __builtin_bit_cast(unsigned, xr[j][tb][r] + silu_fast_(acc[tb][j][r] * bsc[j][r] + bsh[j][r])), ry,
              vtok[tb], (128 * j + r) * HWi * 4, 0);
      const float e = group4_sum(ext[j]);
      const int c48 = (wid + 8 * j) * 16 + l15;
      __builtin_amdgcn_raw_buffer_store_b32(
          __builtin_bit_cast(unsigned, x48[j] + silu_fast_(e * p.bn_scale[c48] + p.bn_shift[c48])), ry, v48,
          128 * j * HWi * 4, 0);
    }
  }
}

}  // namespace wide
}  // namespace ys

using namespace ys;

// returns 1 if launched, 0 if the shape is not handled (C != 256, heads != 4, window != 7x7, hidden != 2C), <0 on
// error. bn_scale / bn_shift: the pw BatchNorm folded to a per-channel affine (fold_bn_kernel).
int yolosod_swin_wide_launch(const float* x, float* y, int B, int C, int H, int W, int num_heads, int wh, int ww,
                             int nWx, int nWin, const float* dw_w, const float* ln1_w, const float* ln1_b,
                             float ln1_eps, const float* in_proj_w, const float* in_proj_b, const float* out_proj_w,
                             const float* out_proj_b, const float* ln2_w, const float* ln2_b, float ln2_eps,
                             const float* mlp1_w, const float* mlp1_b, int mlp_hidden, const float* mlp2_w,
                             const float* mlp2_b, const float* pw_w, const float* bn_scale, const float* bn_shift,
                             hipStream_t st) {
  if (C != wide::C || num_heads != C / wide::HD || wh != 7 || ww != 7 || mlp_hidden != 2 * C) return 0;
  if ((long)C * H * W >= (1L << 30) || (long)B * nWin >= (1L << 31)) return 0;  // 32-bit byte offsets / indices
  wide::Args a{x, y, B, H, W, nWx, nWin, dw_w, ln1_w, ln1_b, ln1_eps, in_proj_w, in_proj_b, out_proj_w, out_proj_b,
               ln2_w, ln2_b, ln2_eps, mlp1_w, mlp1_b, mlp2_w, mlp2_b, pw_w, bn_scale, bn_shift,
               1.0f / sqrtf((float)wide::HD)};
  const long nwin = (long)B * nWin;
  if (nwin == 0) return 1;
  hipLaunchKernelGGL(wide::swin_wide_kernel, dim3((unsigned)(8 * ((nwin + 7) / 8))), dim3(wide::NT), 0, st, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("swin_wide: launch failed: %s", hipGetErrorString(e));
    return -1;
  }
  return 1;
}
