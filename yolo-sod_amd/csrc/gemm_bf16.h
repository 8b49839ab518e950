// bf16 MFMA GEMM for gfx950 (the bf16 model config), fp32 accumulation, fused prologue / epilogue.
//
//   out(b, m, n) = epilogue( sum_k A'(b, m, k) * B(b, k, n) )      out, res: bf16; bias / BN / LN params: fp32
//   A(b,m,k) = A[b*a_bs + m*lda + k]        (K-contiguous: token-major activations or weights)
//   A'      = A, or bf16(LayerNorm_k(A)) when ln_w != nullptr, from per-row (mean, rstd) computed once by
//             row_stats_bf16_kernel; applied in fp32 while staging the A tile, rounded once to bf16 for the MFMA
//   B_KC:  B(b,k,n) = B[b*b_bs + n*ldb + k]  (K-contiguous: nn.Linear / 1x1-conv weights, token-major acts)
//   !B_KC: B(b,k,n) = B[b*b_bs + k*ldb + n]  (N-contiguous: NCHW activations; transposed while staging to LDS)
//
// Tiling: 4 waves, each an (MI*32)x(NI*32) block of v_mfma_f32_32x32x16_bf16 accumulators; BK = 64 (4 MFMA k-steps);
// LDS double buffer + register prefetch of the next k block (one barrier per k block). LDS images are [row][k] with
// a 72-element (144-byte) row stride: lane (r = l&31, h = l>>5) reads its 8 k-consecutive bf16 operand elements
// (k = 8h .. 8h+7 of the 16-wide step) as one ds_read_b128, and the 16 rows of a read group land on distinct banks.
// Tile order is XCD-aware (workgroup i runs on XCD i % 8: contiguous row-major tile ranges per XCD). The epilogue
// stages the fp32 accumulators through LDS and stores 4 consecutive n per lane (8 bytes of bf16); the Swin variant
// scatters token columns to NCHW pixels (window reverse is the identity here: tokens are in padded raster order).
#pragma once
#include "common.h"
#include <stdlib.h>

namespace ys {

struct EpiB {
  const float* bias;   // bias_mode 1: per-row m, 2: per-col n
  int bias_mode;
  const float* scale;  // folded BN:  v = v*scale + shift, bn_mode 1: per-row, 2: per-col
  const float* shift;
  int bn_mode;
  int act;             // 0 none, 1 SiLU, 2 GELU(erf), 3 ReLU
  const bf16_t* res;   // residual added after activation (same indexing as out)
  long res_bs;
  int ldr;
  bf16_t* out;
  long out_bs;
  int ldc;
  // Swin output: n = token of the padded raster [img][Hp][Wp], m = channel; out / res are NCHW [img][M][H][W],
  // tokens in the padding (h >= H or w >= W) are dropped (blocks_transformer.py:125-129 crop)
  int swin;
  int sw_H, sw_W, sw_Hp, sw_Wp;
  int vec;             // set by launch_gemm_bf16: 4-wide epilogue legal (alignment / strides)
  int pair;            // set by launch_gemm_bf16: Swin output as token pairs (4-byte stores; W, Wp even)
};

struct GemmB {
  const bf16_t* A;
  long a_bs;
  int lda;
  const bf16_t* B;
  long b_bs;
  int ldb;
  int M, N, K;
  const float* ln_w;      // optional LayerNorm of A rows (fp32 params)
  const float* ln_b;
  const float* ln_stats;  // [M][2] = (mean, rstd) from row_stats_bf16_kernel, required with ln_w
  int tiles_n, tiles;     // set by launch_gemm_bf16
  EpiB epi;
};

// Per-row LayerNorm statistics (mean, 1/sqrt(var + eps)) of a K-contiguous bf16 [rows][K] matrix: one wave per
// row, values widened to fp32 in registers (K <= 1024), two passes (mean, then centred sum of squares).
template <int VPL>
__global__ __launch_bounds__(256) void row_stats_bf16_kernel(const bf16_t* __restrict__ x, int ld, long rows, int K,
                                                             float eps, float* __restrict__ stats) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const bf16_t* xr = x + row * ld;
  const int K4 = K >> 2;
  f32x4 v[VPL];
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < VPL; ++u) {
    const int c = lane + 64 * u;
    v[u] = ld4(xr + 4 * (c < K4 ? c : K4 - 1));  // unconditional: a predicated load waited in turn
    if (c >= K4) v[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    s += (v[u].x + v[u].y) + (v[u].z + v[u].w);
  }
  const float mean = wave_sum(s) / (float)K;
  float q = 0.f;
#pragma unroll
  for (int u = 0; u < VPL; ++u) {
    if (lane + 64 * u < K4) {
      const f32x4 d = v[u] - mean;
      q += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
    }
  }
  const float var = wave_sum(q) / (float)K;
  if (lane == 0) {
    stats[2 * row] = mean;
    stats[2 * row + 1] = 1.0f / sqrtf(var + eps);
  }
}

static inline int launch_row_stats_bf16(const bf16_t* x, int ld, long rows, int K, float eps, float* stats,
                                        hipStream_t st) {
  YS_CHECK_ARG(K % 4 == 0 && K <= 1024 && ld % 4 == 0, "row_stats_bf16: K=%d ld=%d unsupported", K, ld);
  if (rows == 0) return 0;
  const dim3 grid((unsigned)((rows + 3) / 4));
  if (K <= 256) hipLaunchKernelGGL((row_stats_bf16_kernel<1>), grid, dim3(256), 0, st, x, ld, rows, K, eps, stats);
  else if (K <= 512) hipLaunchKernelGGL((row_stats_bf16_kernel<2>), grid, dim3(256), 0, st, x, ld, rows, K, eps, stats);
  else hipLaunchKernelGGL((row_stats_bf16_kernel<4>), grid, dim3(256), 0, st, x, ld, rows, K, eps, stats);
  YS_CHECK_LAUNCH("row_stats_bf16");
  return 0;
}

// LayerNorm of K-contiguous bf16 rows, written back as bf16 rows for a GEMM without an A prologue: the statistics
// exactly as row_stats_bf16_kernel, then bf16(fma((x - mean) * rstd, w, b)) - the expression the LN prologue of
// gemm_bf16_kernel evaluates. Applying it once per row instead of in every N tile's staging (QKV: 12 tiles of 128 at
// C = 512) took the VALU of the LN off those GEMMs' main loops.
template <int VPL>
__global__ __launch_bounds__(256) void ln_rows_bf16_kernel(const bf16_t* __restrict__ x, int ld, long rows, int K,
                                                           float eps, const float* __restrict__ w,
                                                           const float* __restrict__ b, bf16_t* __restrict__ out,
                                                           int ldo) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const bf16_t* xr = x + row * ld;
  const int K4 = K >> 2;
  f32x4 v[VPL];
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < VPL; ++u) {
    const int c = lane + 64 * u;
    v[u] = ld4(xr + 4 * (c < K4 ? c : K4 - 1));  // unconditional: a predicated load waited in turn
    if (c >= K4) v[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    s += (v[u].x + v[u].y) + (v[u].z + v[u].w);
  }
  const float mean = wave_sum(s) / (float)K;
  float q = 0.f;
#pragma unroll
  for (int u = 0; u < VPL; ++u) {
    if (lane + 64 * u < K4) {
      const f32x4 d = v[u] - mean;
      q += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
    }
  }
  const float var = wave_sum(q) / (float)K;
  const float rs = 1.0f / sqrtf(var + eps);
#pragma unroll
  for (int u = 0; u < VPL; ++u) {
    const int c = lane + 64 * u;
    if (c < K4) {
      const f32x4 lw = *reinterpret_cast<const f32x4*>(w + 4 * c), lb = *reinterpret_cast<const f32x4*>(b + 4 * c);
      f32x4 o;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = fmaf((v[u][i] - mean) * rs, lw[i], lb[i]);
      st4(out + row * ldo + 4 * c, o);
    }
  }
}

static inline int launch_ln_rows_bf16(const bf16_t* x, int ld, long rows, int K, float eps, const float* w,
                                      const float* b, bf16_t* out, int ldo, hipStream_t st) {
  YS_CHECK_ARG(K % 4 == 0 && K <= 1024 && ld % 4 == 0 && ldo % 4 == 0, "ln_rows_bf16: K=%d ld=%d unsupported", K, ld);
  YS_CHECK_ARG(((uintptr_t)w | (uintptr_t)b) % 16 == 0, "ln_rows_bf16: LN params must be 16-byte aligned");
  if (rows == 0) return 0;
  const dim3 grid((unsigned)((rows + 3) / 4));
#define YS_LNR(V_) hipLaunchKernelGGL((ln_rows_bf16_kernel<V_>), grid, dim3(256), 0, st, x, ld, rows, K, eps, w, b, out, ldo)
  if (K <= 256) YS_LNR(1);
  else if (K <= 512) YS_LNR(2);
  else YS_LNR(4);
#undef YS_LNR
  YS_CHECK_LAUNCH("ln_rows_bf16");
  return 0;
}

__device__ __forceinline__ float act_b(float v, int act) {
  if (act == 1) return silu_fast_(v);
  if (act == 2) return gelu_fast_(v);
  if (act == 3) return fmaxf(v, 0.f);
  return v;
}

template <int WM, int WN, int MI, int NI, bool B_KC, bool A_LN>
__global__ __launch_bounds__(256, A_LN ? 2 : 3) void gemm_bf16_kernel(GemmB g) {
  constexpr int BM = WM * MI * 32;
  constexpr int BN = WN * NI * 32;
  constexpr int BK = 64;
  constexpr int SK = BK + 8;                  // [row][k] image stride (bf16 elements): 144 B
  constexpr int A_ELEMS = BM * SK;
  constexpr int B_ELEMS = BN * SK;
  constexpr int NA = BM * BK / 8 / 256;       // 16-byte chunks per thread per A tile
  constexpr int NB = BN * BK / 8 / 256;
  // an N-contiguous B tile as one 4x8 (k, n) block per thread (BN / 8 column chunks x BK / 4 row quads = 256)
  constexpr bool BT = !B_KC && NB == 4 && (BN / 8) * (BK / 4) == 256;
  constexpr int SC = BN + 4;                  // epilogue staging row stride (fp32)
  // one LDS image of the A / B tiles (the next tile waits in registers, so a second LDS buffer bought nothing but
  // occupancy lost) and the C staging in two row halves: 37 KB per workgroup instead of 74, 3 workgroups per CU
  constexpr int MAIN_BYTES = (A_ELEMS + B_ELEMS) * 2;
  constexpr int HB = BM / 2;                  // staged rows per epilogue pass
  constexpr int STAGE_BYTES = HB * SC * 4;
  constexpr int SMEM_BYTES = (MAIN_BYTES > STAGE_BYTES ? MAIN_BYTES : STAGE_BYTES) + (A_LN ? 8 * BM : 0);
  static_assert(WM * WN == 4, "4 waves");
  static_assert(NA >= 1 && NB >= 1, "tile too small");
  static_assert(MI * 32 <= BM / 2, "a wave's rows lie in one epilogue half");
  __shared__ __attribute__((aligned(16))) char smem[SMEM_BYTES];
  bf16_t* As = reinterpret_cast<bf16_t*>(smem);
  bf16_t* Bs = As + A_ELEMS;
  float* s_mean = reinterpret_cast<float*>(smem + SMEM_BYTES - (A_LN ? 8 * BM : 0));
  float* s_rstd = s_mean + BM;

  const int tpx = (g.tiles + 7) >> 3;
  const int t = (blockIdx.x & 7) * tpx + (blockIdx.x >> 3);
  if (t >= g.tiles) return;
  const int m0 = (t / g.tiles_n) * BM, n0 = (t % g.tiles_n) * BN;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int bz = blockIdx.z;
  const bf16_t* A = g.A + (long)bz * g.a_bs;
  const bf16_t* B = g.B + (long)bz * g.b_bs;
  const int M = g.M, N = g.N, K = g.K;

  if (A_LN) {
    for (int r = tid; r < BM; r += 256) {
      const int m = m0 + r;
      const float2 st = (m < M) ? *reinterpret_cast<const float2*>(g.ln_stats + 2L * m) : make_float2(0.f, 0.f);
      s_mean[r] = st.x;
      s_rstd[r] = st.y;
    }
  }

  // rb as a native vector: a uint4 (struct) element copied global -> array -> LDS stays a memcpy through a stack
  // array once its load is unconditional (scratch round trip per tile)
  uint4 ra[NA];
  u32x4_t rb[NB];
  int cur_k0 = 0;  // k offset of the tile held in ra / rb (LN params of the A prologue)
  // Every tile load is unconditional: rows past M / N read row M-1 / N-1 and an N-contiguous chunk past N reads
  // column 0, whose products land in output rows / columns the epilogue never stores. A load under a per-lane
  // predicate merges into a phi whose copy waited for every load in flight (vmcnt(0) after each load of a tile).
  // A partial N-contiguous chunk (n < N < n + 8) reads up to ldb (ldb % 8 == 0): in bounds, and its columns past N
  // only feed unstored outputs.
  auto load_tiles = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int idx = tid + 256 * i;
      const int m = m0 + (idx >> 3);
      ra[i] = *reinterpret_cast<const uint4*>(A + (long)(m < M ? m : M - 1) * g.lda + k0 + (idx & 7) * 8);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int idx = tid + 256 * i;
      if (B_KC) {
        const int n = n0 + (idx >> 3);
        rb[i] = *reinterpret_cast<const u32x4_t*>(B + (long)(n < N ? n : N - 1) * g.ldb + k0 + (idx & 7) * 8);
      } else {
        // BT: thread t loads k rows 4 (t / (BN/8)) + i of its 8-column chunk (t % (BN/8)): a 4x8 (k, n) block that
        // store_tiles writes as 8 [n][k] rows of 4 k (8-byte LDS stores instead of 32 2-byte ones)
        const int kl = BT ? 4 * (tid / (BN / 8)) + i : idx / (BN / 8);
        const int n = n0 + ((BT ? tid : idx) % (BN / 8)) * 8;
        rb[i] = *reinterpret_cast<const u32x4_t*>(B + (long)(k0 + kl) * g.ldb + (n < N ? n : 0));
      }
    }
  };
  auto store_tiles = [&]() {
    bf16_t* Ab = As;
    bf16_t* Bb = Bs;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int idx = tid + 256 * i;
      const int r = idx >> 3, kc = (idx & 7) * 8;
      uint4 v = ra[i];
      if (A_LN) {
        // LN params of this chunk's 8 k (L1-resident)
        float f[8];
        unpack8(v, f);
        const float mu = s_mean[r], rs = s_rstd[r];
        const float* lw = g.ln_w + cur_k0 + kc;
        const float* lb = g.ln_b + cur_k0 + kc;
#pragma unroll
        for (int q = 0; q < 8; ++q) f[q] = fmaf((f[q] - mu) * rs, lw[q], lb[q]);
        v = pack8(f);
      }
      *reinterpret_cast<uint4*>(&Ab[r * SK + kc]) = v;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int idx = tid + 256 * i;
      if (B_KC) {
        const int r = idx >> 3, kc = (idx & 7) * 8;
        *reinterpret_cast<u32x4_t*>(&Bb[r * SK + kc]) = rb[i];
      } else if (BT) {  // the thread's 4x8 block: n = nc + j gets k = kq .. kq + 3 as one 8-byte store
        if (i == 0) {
          const int kq = 4 * (tid / (BN / 8)), nc = (tid % (BN / 8)) * 8;
          const uint32_t w[4][4] = {{rb[0].x, rb[0].y, rb[0].z, rb[0].w}, {rb[1].x, rb[1].y, rb[1].z, rb[1].w},
                                    {rb[2].x, rb[2].y, rb[2].z, rb[2].w}, {rb[3].x, rb[3].y, rb[3].z, rb[3].w}};
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int sh = (j & 1) * 16;  // element j of a row: 32-bit word j / 2, half j % 2
            const uint32_t e0 = (w[0][j >> 1] >> sh) & 0xffffu, e1 = (w[1][j >> 1] >> sh) & 0xffffu;
            const uint32_t e2 = (w[2][j >> 1] >> sh) & 0xffffu, e3 = (w[3][j >> 1] >> sh) & 0xffffu;
            *reinterpret_cast<uint2*>(&Bb[(nc + j) * SK + kq]) = make_uint2(e0 | (e1 << 16), e2 | (e3 << 16));
          }
        }
      } else {  // 8 n-consecutive values of one k row -> column k of 8 [n][k] rows
        const int kl = idx / (BN / 8), nc = (idx % (BN / 8)) * 8;
        const uint32_t w[4] = {rb[i].x, rb[i].y, rb[i].z, rb[i].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          Bb[(nc + 2 * q) * SK + kl] = (bf16_t)(w[q] & 0xffffu);
          Bb[(nc + 2 * q + 1) * SK + kl] = (bf16_t)(w[q] >> 16);
        }
      }
    }
  };

  f32x16 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nk = K / BK;
  const int lr = lane & 31, lh = lane >> 5;
  load_tiles(0);
  if (A_LN) __syncthreads();  // s_mean / s_rstd
  store_tiles();
  __syncthreads();
  for (int kb = 0; kb < nk; ++kb) {
    load_tiles((kb + 1 < nk ? kb + 1 : kb) * BK);  // unconditional (the last trip reloads its own tile)
    // keep the next tile's loads ahead of this tile's MFMAs (the scheduler otherwise sinks them to the barrier)
    __builtin_amdgcn_sched_barrier(0);
    const bf16_t* Ab = As + (wm * MI * 32 + lr) * SK + lh * 8;
    const bf16_t* Bb = Bs + (wn * NI * 32 + lr) * SK + lh * 8;
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      bf16x8_t a[MI], b[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) a[i] = *reinterpret_cast<const bf16x8_t*>(Ab + i * 32 * SK + 16 * kk);
#pragma unroll
      for (int j = 0; j < NI; ++j) b[j] = *reinterpret_cast<const bf16x8_t*>(Bb + j * 32 * SK + 16 * kk);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
    if (kb + 1 < nk) {
      cur_k0 = (kb + 1) * BK;
      store_tiles();
      __syncthreads();
    }
  }

  const EpiB& e = g.epi;
  // stage C through LDS in two row halves (the main-loop buffer is free after the last barrier); a wave's rows lie
  // in one half. C/D map of 32x32: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  float* Cs = reinterpret_cast<float*>(smem);
  // scalar epilogue (Swin: consecutive raster tokens = consecutive pixels of an output row): a thread's column is
  // the same in every row pass (256 % BN == 0), so its output offset (token -> pixel, crop) is computed once; rows
  // advance by the channel plane
  static_assert(256 % BN == 0, "column per thread");
  const int col = tid % BN, ncol = n0 + col;
  bool col_ok = ncol < N;
  long o0 = 0, r0_ = 0, m_str = 0, r_str = 0;
  if (!e.vec && col_ok) {
    if (e.swin) {
      const long per_img = (long)e.sw_Hp * e.sw_Wp;
      const int img = (int)(ncol / per_img);
      const int rr = (int)(ncol - img * per_img);
      const int h = rr / e.sw_Wp, w = rr - (rr / e.sw_Wp) * e.sw_Wp;
      col_ok = h < e.sw_H && w < e.sw_W;  // crop of the padded border
      m_str = (long)e.sw_H * e.sw_W;      // out / res NCHW [img][M][H][W]
      o0 = (long)img * M * m_str + (long)h * e.sw_W + w;
      r0_ = o0;
      r_str = m_str;
    } else {
      m_str = e.ldc;
      r_str = e.ldr;
      o0 = (long)bz * e.out_bs + ncol;
      r0_ = (long)bz * e.res_bs + ncol;
    }
  }
  // residual operands of a half are loaded before its staging barrier, all at once: in the loops below each
  // iteration's residual load was a separate HBM round trip (the out-projection / MLP2 / pw GEMMs spent as long in
  // their epilogues as in their main loops)
  constexpr int NQ = BN / 4;
  constexpr int VIT = HB * NQ / 256;         // vector-epilogue iterations per half
  constexpr int SIT = HB / (256 / BN);       // scalar-epilogue rows per thread and half
  static_assert(HB * NQ % 256 == 0 && SIT % 8 == 0, "epilogue split");
  const bf16_t* resb = e.res ? e.res + (long)bz * e.res_bs : nullptr;
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    const int mh = m0 + hf * HB;
    uint2 rv[VIT];
    if (resb && e.vec) {
#pragma unroll
      for (int it = 0; it < VIT; ++it) {
        const int idx = tid + 256 * it;
        const int m = mh + idx / NQ, n = n0 + 4 * (idx % NQ);
        // unconditional, clamped (a predicated load's phi copy waited for the loads before it)
        rv[it] = *reinterpret_cast<const uint2*>(resb + (long)(m < M ? m : M - 1) * e.ldr + (n < N ? n : N - 4));
      }
    }
    if (hf) __syncthreads();  // the first half's epilogue has read Cs
    if ((wm * MI * 32) / HB == hf) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            Cs[(wm * MI * 32 - hf * HB + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh) * SC + wn * NI * 32 + j * 32 + lr] =
                acc[i][j][r];
    }
    __syncthreads();
    if (e.vec) {
      bf16_t* outb = e.out + (long)bz * e.out_bs;
#pragma unroll
      for (int it = 0; it < VIT; ++it) {
        const int idx = tid + 256 * it;
        const int row = idx / NQ, c4 = idx % NQ;
        const int m = mh + row;
        const int n = n0 + 4 * c4;
        if (m >= M || n >= N) continue;
        f32x4 v = *reinterpret_cast<const f32x4*>(&Cs[row * SC + 4 * c4]);
        if (e.bias_mode == 1) v += e.bias[m];
        else if (e.bias_mode == 2) v += *reinterpret_cast<const f32x4*>(e.bias + n);
        if (e.bn_mode == 1) v = v * e.scale[m] + e.shift[m];
        else if (e.bn_mode == 2)
          v = v * *reinterpret_cast<const f32x4*>(e.scale + n) + *reinterpret_cast<const f32x4*>(e.shift + n);
        v.x = act_b(v.x, e.act); v.y = act_b(v.y, e.act); v.z = act_b(v.z, e.act); v.w = act_b(v.w, e.act);
        if (resb)
          v += f32x4{__uint_as_float(rv[it].x << 16), __uint_as_float(rv[it].x & 0xffff0000u),
                     __uint_as_float(rv[it].y << 16), __uint_as_float(rv[it].y & 0xffff0000u)};
        st4(outb + (long)m * e.ldc + n, v);
      }
    } else if (BN == 128 && e.pair) {
      // Swin output as token pairs: thread (rsub, pc) owns tokens n0 + 2 pc, +1 (same image row: W and Wp are even,
      // so a pair is cropped whole or not at all) for rows rsub + 4 it - one 4-byte residual load and one 4-byte
      // store per pair instead of two 2-byte accesses per element
      static_assert(HB % 4 == 0, "pair epilogue: 4 rows per pass");
      const int pc = tid & 63, rsub = tid >> 6;  // BN == 128: 64 pairs per row
      const long tok = (long)n0 + 2 * pc;
      const long per_img = (long)e.sw_Hp * e.sw_Wp;
      const int img = (int)(tok / per_img);
      const int rr = (int)(tok - img * per_img);
      const int h = rr / e.sw_Wp, w = rr - (rr / e.sw_Wp) * e.sw_Wp;
      if (tok < N && h < e.sw_H && w < e.sw_W) {
        const long HWo = (long)e.sw_H * e.sw_W;
        const long o0p = (long)img * M * HWo + (long)h * e.sw_W + w;
        constexpr int PIT = HB / 4;
        uint32_t rp[PIT];
#pragma unroll
        for (int it = 0; it < PIT; ++it) {
          const int m = mh + rsub + 4 * it;
          rp[it] = e.res ? *reinterpret_cast<const uint32_t*>(e.res + o0p + (long)(m < M ? m : M - 1) * HWo) : 0u;
        }
#pragma unroll
        for (int it = 0; it < PIT; ++it) {
          const int row = rsub + 4 * it;
          const int m = mh + row;
          if (m >= M) continue;
          const float2 c2 = *reinterpret_cast<const float2*>(&Cs[row * SC + 2 * pc]);
          float v0 = c2.x, v1 = c2.y;
          if (e.bias_mode == 1) { v0 += e.bias[m]; v1 += e.bias[m]; }
          if (e.bn_mode == 1) { v0 = v0 * e.scale[m] + e.shift[m]; v1 = v1 * e.scale[m] + e.shift[m]; }
          v0 = act_b(v0, e.act);
          v1 = act_b(v1, e.act);
          if (e.res) {
            v0 += __uint_as_float(rp[it] << 16);
            v1 += __uint_as_float(rp[it] & 0xffff0000u);
          }
          *reinterpret_cast<uint32_t*>(e.out + o0p + (long)m * HWo) = pack_bf16x2(v0, v1);
        }
      }
    } else if (col_ok) {
      const float bn_ = e.bias_mode == 2 ? e.bias[ncol] : 0.f;
      const float sc_n = e.bn_mode == 2 ? e.scale[ncol] : 1.f, sh_n = e.bn_mode == 2 ? e.shift[ncol] : 0.f;
      // rows in batches of 8: the batch's residual loads go out together
      for (int it0 = 0; it0 < SIT; it0 += 8) {
        bf16_t r8[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int m = mh + tid / BN + (it0 + u) * (256 / BN);
          r8[u] = e.res ? e.res[r0_ + (long)(m < M ? m : M - 1) * r_str] : (bf16_t)0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int row = tid / BN + (it0 + u) * (256 / BN);
          const int m = mh + row;
          if (m < M) {
            float v = Cs[row * SC + col];
            if (e.bias_mode == 1) v += e.bias[m];
            else if (e.bias_mode == 2) v += bn_;
            if (e.bn_mode == 1) v = v * e.scale[m] + e.shift[m];
            else if (e.bn_mode == 2) v = v * sc_n + sh_n;
            v = act_b(v, e.act);
            if (e.res) v += bf2f(r8[u]);
            e.out[o0 + (long)m * m_str] = f2bf(v);
          }
        }
      }
    }
  }
}

static inline bool al_b(const void* p, int bytes) { return ((uintptr_t)p & (bytes - 1)) == 0; }

static inline int launch_gemm_bf16(const GemmB& g0, int batch, bool b_kc, hipStream_t st) {
  GemmB g = g0;
  YS_CHECK_ARG(g.K % 64 == 0, "gemm_bf16: K=%d must be a multiple of 64", g.K);
  YS_CHECK_ARG(g.lda % 8 == 0 && g.ldb % 8 == 0 && g.a_bs % 8 == 0 && g.b_bs % 8 == 0,
               "gemm_bf16: lda / ldb / batch strides must be multiples of 8");
  YS_CHECK_ARG(al_b(g.A, 16) && al_b(g.B, 16), "gemm_bf16: A/B must be 16-byte aligned");
  YS_CHECK_ARG(!g.ln_w || (g.ln_b && g.ln_stats && al_b(g.ln_stats, 8)),
               "gemm_bf16: LN params must come with row statistics");
  if (g.M == 0 || g.N == 0 || batch == 0) return 0;
  const EpiB& e = g.epi;
  g.epi.pair = e.swin && e.sw_W % 2 == 0 && e.sw_Wp % 2 == 0 && e.bias_mode != 2 && e.bn_mode != 2 && al_b(e.out, 4) &&
               (!e.res || al_b(e.res, 4));
  g.epi.vec = !e.swin && g.N % 4 == 0 && e.ldc % 4 == 0 && e.out_bs % 4 == 0 && al_b(e.out, 8) &&
              (!e.res || (e.ldr % 4 == 0 && e.res_bs % 4 == 0 && al_b(e.res, 8))) &&
              (e.bias_mode != 2 || al_b(e.bias, 16)) && (e.bn_mode != 2 || (al_b(e.scale, 16) && al_b(e.shift, 16)));
  const bool ln = g.ln_w != nullptr;
#define YS_GEMMB_LAUNCH(WM_, WN_, MI_, NI_)                                                                     \
  do {                                                                                                          \
    constexpr int bm = WM_ * MI_ * 32, bn = WN_ * NI_ * 32;                                                     \
    g.tiles_n = (g.N + bn - 1) / bn;                                                                            \
    g.tiles = g.tiles_n * ((g.M + bm - 1) / bm);                                                                \
    dim3 grid((unsigned)(8 * ((g.tiles + 7) / 8)), 1, batch);                                                   \
    if (b_kc) {                                                                                                 \
      if (ln) hipLaunchKernelGGL((gemm_bf16_kernel<WM_, WN_, MI_, NI_, true, true>), grid, dim3(256), 0, st, g); \
      else hipLaunchKernelGGL((gemm_bf16_kernel<WM_, WN_, MI_, NI_, true, false>), grid, dim3(256), 0, st, g);  \
    } else {                                                                                                    \
      hipLaunchKernelGGL((gemm_bf16_kernel<WM_, WN_, MI_, NI_, false, false>), grid, dim3(256), 0, st, g);      \
    }                                                                                                           \
  } while (0)
  YS_CHECK_ARG(b_kc || !ln, "gemm_bf16: LN prologue needs a K-contiguous B");
  // 128x64 tiles when N is narrow or 128x128 would leave CUs idle; 128x128 otherwise
  const long t128 = (long)((g.M + 127) / 128) * ((g.N + 127) / 128) * batch;
  constexpr int force = 0;  // A/B builds: 1 = 128x64 everywhere, 2 = 128x128 everywhere
  if (force == 1 || (force != 2 && (g.N <= 64 || t128 < 512))) YS_GEMMB_LAUNCH(4, 1, 1, 2);
  else YS_GEMMB_LAUNCH(2, 2, 2, 2);
#undef YS_GEMMB_LAUNCH
  YS_CHECK_LAUNCH("gemm_bf16");
  return 0;
}

static inline EpiB epib_plain(bf16_t* out, long out_bs, int ldc) {
  EpiB e{};
  e.out = out;
  e.out_bs = out_bs;
  e.ldc = ldc;
  return e;
}

}  // namespace ys
