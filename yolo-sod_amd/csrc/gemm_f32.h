// Exact-fp32 MFMA GEMM for gfx950 with fused prologue / epilogue (used by the Swin and A2 drivers).
//
//   out(b, m, n) = epilogue( sum_k A'(b, m, k) * B(b, k, n) )
//   A(b,m,k) = A[b*a_bs + m*lda + k]       (K-contiguous)
//   A'      = A, or LayerNorm_k(A) when ln_w != nullptr: per-row (mean, rstd) come precomputed from
//             row_stats_kernel (one read of A); the normalisation is applied while staging the A tile, so the
//             normalised activations never exist in HBM
//   B_KC:  B(b,k,n) = B[b*b_bs + n*ldb + k]  (K-contiguous: nn.Linear / 1x1-conv weights, token-major acts)
//   !B_KC: B(b,k,n) = B[b*b_bs + k*ldb + n]  (N-contiguous: NCHW activations)
//
// Tiling: 4 waves, each an (MI*32)x(NI*32) output block of v_mfma_f32_32x32x2_f32 accumulators (128x128 tiles with
// 2x2 per wave, or 128x64 with 1x2 for narrow N); block tile x BK=32; LDS double-buffered with register prefetch (one barrier per K block).
// The MFMA's k index is permuted: lane half h takes k = h*16 + s (s = 0..15) of each 32-deep block, so the A and
// K-contiguous B fragments are 16-byte ds_read_b128 along k from a [row][k] LDS image whose 36-float row stride
// keeps each 16-lane read group conflict-free. The summation order differs from a plain k loop only by rounding.
// Tile order is XCD-aware: workgroup i runs on XCD i % 8, so the tiles are dealt to XCDs in contiguous row-major
// ranges and the N-tiles that share an A row-block hit the same XCD L2. The epilogue stages the accumulators
// through LDS and stores whole rows with 16-byte coalesced stores (bias / BN / act / residual fused).
#pragma once
#include "common.h"
#include <stdlib.h>

namespace ys {

struct Epi {
  const float* bias;   // bias_mode 1: per-row m, 2: per-col n
  int bias_mode;
  const float* scale;  // folded BN:  v = v*scale + shift, bn_mode 1: per-row, 2: per-col
  const float* shift;
  int bn_mode;
  int act;             // 0 none, 1 SiLU, 2 GELU(erf), 3 ReLU
  const float* res;    // residual added after activation (same indexing as out)
  long res_bs;
  int ldr;
  float* out;
  long out_bs;
  int ldc;
  // window-reverse output (SwinBlock): n = global token, m = channel; out/res are NCHW [img][M][H][W]
  int swin;
  int sw_H, sw_W, sw_wh, sw_ww, sw_nWx, sw_nWin;
  int vec;             // set by launch_gemm: 16-byte epilogue legal (alignment / strides)
};

struct GemmArgs {
  const float* A;
  long a_bs;
  int lda;
  const float* B;
  long b_bs;
  int ldb;
  int M, N, K;
  const float* ln_w;      // optional LayerNorm of A rows
  const float* ln_b;
  const float* ln_stats;  // [M][2] = (mean, rstd) from row_stats_kernel, required with ln_w
  int tiles_n, tiles;     // set by launch_gemm
  Epi epi;
  int nimg;               // set by launch_gemm: > 0 = batch folded into N (N-contiguous B, nimg columns per image)
  int nmajor;             // set by launch_gemm: tiles in column-major (n-major) order
  int bfold;              // set by launch_gemm: > 0 = batch folded into the tile index (bfold images, n-major inside)
  int x2;                 // 1: products as fp16 two-term splits on v_mfma_f32_32x32x16_f16 (fp32 accuracy)
  float x2_sa, x2_sb;     // x2: exact power-of-two scales of A / B at the split (a weight operand: 64, keeps its
                          // low terms out of fp16's subnormal range); the accumulators are scaled back before the
                          // epilogue. 0 = 1
  unsigned* range_flag;   // x2: split-range guard (common.h range_report); set by launch_gemm
};

// Per-row LayerNorm statistics (mean, 1/sqrt(var + eps)) of a K-contiguous [rows][K] matrix: one wave per row,
// the row held in registers (K <= 1024), two passes (mean, then centred sum of squares) as torch does.
template <int VPL>
__global__ __launch_bounds__(256) void row_stats_kernel(const float* __restrict__ x, int ld, long rows, int K,
                                                        float eps, float* __restrict__ stats) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float4* xr = reinterpret_cast<const float4*>(x + row * ld);
  const int K4 = K >> 2;
  float4 v[VPL];
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < VPL; ++u) {
    const int c = lane + 64 * u;
    v[u] = xr[c < K4 ? c : K4 - 1];  // unconditional: a predicated load waited in turn
    if (c >= K4) v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    s += (v[u].x + v[u].y) + (v[u].z + v[u].w);
  }
  const float mean = wave_sum(s) / (float)K;
  float q = 0.f;
#pragma unroll
  for (int u = 0; u < VPL; ++u) {
    if (lane + 64 * u < K4) {
      const float a = v[u].x - mean, b = v[u].y - mean, c = v[u].z - mean, d = v[u].w - mean;
      q += (a * a + b * b) + (c * c + d * d);
    }
  }
  const float var = wave_sum(q) / (float)K;
  if (lane == 0) {
    stats[2 * row] = mean;
    stats[2 * row + 1] = 1.0f / sqrtf(var + eps);
  }
}

static inline int launch_row_stats(const float* x, int ld, long rows, int K, float eps, float* stats, hipStream_t st) {
  YS_CHECK_ARG(K % 4 == 0 && K <= 1024 && ld % 4 == 0, "row_stats: K=%d ld=%d unsupported", K, ld);
  if (rows == 0) return 0;
  const dim3 grid((unsigned)((rows + 3) / 4));
  if (K <= 256) hipLaunchKernelGGL((row_stats_kernel<1>), grid, dim3(256), 0, st, x, ld, rows, K, eps, stats);
  else if (K <= 512) hipLaunchKernelGGL((row_stats_kernel<2>), grid, dim3(256), 0, st, x, ld, rows, K, eps, stats);
  else hipLaunchKernelGGL((row_stats_kernel<4>), grid, dim3(256), 0, st, x, ld, rows, K, eps, stats);
  YS_CHECK_LAUNCH("row_stats");
  return 0;
}

// LayerNorm of K-contiguous fp32 rows written out as rows (the A operand of a GEMM without an LN prologue): the
// statistics exactly as row_stats_kernel, then fma((x - mean) * rstd, w, b). For an A operand that many N tiles stage
// (A2's QKV GEMM: 12 tiles of 128 at C = 512) this normalises each element once instead of once per tile.
template <int VPL>
__global__ __launch_bounds__(256) void ln_rows_kernel(const float* __restrict__ x, int ld, long rows, int K, float eps,
                                                      const float* __restrict__ w, const float* __restrict__ b,
                                                      float* __restrict__ out, int ldo) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float4* xr = reinterpret_cast<const float4*>(x + row * ld);
  const int K4 = K >> 2;
  float4 v[VPL];
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < VPL; ++u) {
    const int c = lane + 64 * u;
    v[u] = xr[c < K4 ? c : K4 - 1];  // unconditional: a predicated load waited in turn
    if (c >= K4) v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    s += (v[u].x + v[u].y) + (v[u].z + v[u].w);
  }
  const float mean = wave_sum(s) / (float)K;
  float q = 0.f;
#pragma unroll
  for (int u = 0; u < VPL; ++u) {
    if (lane + 64 * u < K4) {
      const float a = v[u].x - mean, bb = v[u].y - mean, c = v[u].z - mean, d = v[u].w - mean;
      q += (a * a + bb * bb) + (c * c + d * d);
    }
  }
  const float var = wave_sum(q) / (float)K;
  const float rs = 1.0f / sqrtf(var + eps);
#pragma unroll
  for (int u = 0; u < VPL; ++u) {
    const int c = lane + 64 * u;
    if (c < K4) {
      const float4 lw = reinterpret_cast<const float4*>(w)[c], lb = reinterpret_cast<const float4*>(b)[c];
      reinterpret_cast<float4*>(out + row * ldo)[c] =
          make_float4(fmaf((v[u].x - mean) * rs, lw.x, lb.x), fmaf((v[u].y - mean) * rs, lw.y, lb.y),
                      fmaf((v[u].z - mean) * rs, lw.z, lb.z), fmaf((v[u].w - mean) * rs, lw.w, lb.w));
    }
  }
}

static inline int launch_ln_rows(const float* x, int ld, long rows, int K, float eps, const float* w, const float* b,
                                 float* out, int ldo, hipStream_t st) {
  YS_CHECK_ARG(K % 4 == 0 && K <= 1024 && ld % 4 == 0 && ldo % 4 == 0, "ln_rows: K=%d ld=%d unsupported", K, ld);
  YS_CHECK_ARG(((uintptr_t)w | (uintptr_t)b | (uintptr_t)x | (uintptr_t)out) % 16 == 0, "ln_rows: 16-byte alignment");
  if (rows == 0) return 0;
  const dim3 grid((unsigned)((rows + 3) / 4));
  if (K <= 256) hipLaunchKernelGGL((ln_rows_kernel<1>), grid, dim3(256), 0, st, x, ld, rows, K, eps, w, b, out, ldo);
  else if (K <= 512) hipLaunchKernelGGL((ln_rows_kernel<2>), grid, dim3(256), 0, st, x, ld, rows, K, eps, w, b, out, ldo);
  else hipLaunchKernelGGL((ln_rows_kernel<4>), grid, dim3(256), 0, st, x, ld, rows, K, eps, w, b, out, ldo);
  YS_CHECK_LAUNCH("ln_rows");
  return 0;
}

__device__ __forceinline__ float apply_act(float v, int act) {
  if (act == 1) return siluf_(v);
  if (act == 2) return geluf_(v);
  if (act == 3) return fmaxf(v, 0.f);
  return v;
}

__device__ __forceinline__ float epi_value(const Epi& e, int m, int n, float v) {
  if (e.bias_mode == 1) v += e.bias[m];
  else if (e.bias_mode == 2) v += e.bias[n];
  if (e.bn_mode == 1) v = v * e.scale[m] + e.shift[m];
  else if (e.bn_mode == 2) v = v * e.scale[n] + e.shift[n];
  return apply_act(v, e.act);
}

// X2: the A tile (and a K-contiguous B tile) is split into fp16 hi / lo terms while staging: row r of the LDS image
// holds, per 8-k group j8, 8 hi halves then 8 lo halves (72 halves = the 144 B of the fp32 image's row, so the same
// buffers; ds_read_b128 row reads stay conflict-free). A lane (half lh) of v_mfma_f32_32x32x16_f16 step s takes k
// group 2*lh + s. An N-contiguous B tile stays fp32 [k][n] in LDS and is split in registers after 8 strided reads.
template <int WM, int WN, int MI, int NI, bool B_KC, bool A_LN, bool X2 = false>
__global__ __launch_bounds__(256, 2) void gemm_f32_kernel(GemmArgs g) {
  constexpr int BM = WM * MI * 32;
  constexpr int BN = WN * NI * 32;
  constexpr int BK = 32;
  constexpr int SK = BK + 4;                     // [row][k] images
  constexpr int SBN = BN + 4;                    // [k][n] image (N-contiguous B)
  constexpr int NA = BM * BK / 4 / 256;          // float4 per thread per A tile
  constexpr int NB = BN * BK / 4 / 256;
  // X2 with an N-contiguous B whose tile is one 4x4 (k, n) block per thread: the block is loaded as four float4 rows,
  // transposed in registers and split once into the same [n][k] hi / lo image as a K-contiguous B, so the MFMA loop
  // reads whole 16-byte fragments (the [k][n] fp32 image took 8 strided reads and a split per fragment and wave)
  constexpr bool BT = X2 && !B_KC && NB == 4 && BN / 4 * (BK / 4) == 256;
  constexpr bool B_IMG = B_KC || BT;             // B staged as a [n][k] image
  constexpr int A_ELEMS = BM * SK;
  constexpr int B_ELEMS = B_IMG ? BN * SK : BK * SBN;
  constexpr int SC = BN + 4;                     // epilogue staging row stride
  constexpr int MAIN_ELEMS = 2 * A_ELEMS + 2 * B_ELEMS;
  constexpr int SMEM = (MAIN_ELEMS > BM * SC ? MAIN_ELEMS : BM * SC) + (A_LN ? 2 * BM : 0);
  static_assert(WM * WN == 4, "4 waves");
  __shared__ __attribute__((aligned(16))) float smem[SMEM];
  float* As = smem;
  float* Bs = smem + 2 * A_ELEMS;
  float* s_mean = smem + (SMEM - (A_LN ? 2 * BM : 0));
  float* s_rstd = s_mean + BM;

  // XCD-aware tile order (gridDim.x = 8 * ceil(tiles / 8)); see header comment
  const int ntiles = g.bfold ? g.tiles * g.bfold : g.tiles;
  const int tpx = (ntiles + 7) >> 3;
  int t = (blockIdx.x & 7) * tpx + (blockIdx.x >> 3);
  if (t >= ntiles) return;
  int bz = blockIdx.z;
  if (g.bfold) {  // batch in the tile index: an image's tiles are contiguous, so they share one XCD's L2
    bz = t / g.tiles;
    t -= bz * g.tiles;
  }
  int m0, n0;
  if (g.nmajor) {  // all M tiles of an N column on one XCD: an N-contiguous B (NCHW activations) is read once
    const int tiles_m = g.tiles / g.tiles_n;
    m0 = (t % tiles_m) * BM;
    n0 = (t / tiles_m) * BN;
  } else {
    m0 = (t / g.tiles_n) * BM;
    n0 = (t % g.tiles_n) * BN;
  }

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const float* A = g.A + (long)bz * g.a_bs;
  const float* B = g.B + (long)bz * g.b_bs;
  const int M = g.M, N = g.N, K = g.K;
  const bool vec_b = (g.ldb & 3) == 0 && (g.b_bs & 3) == 0;
  // folded batch: column n -> image n / nimg, column n % nimg (a float4 never straddles images: nimg % 4 == 0);
  // this thread's B columns are the same in every k block, so their offsets are computed once
  long bcol[B_KC ? 1 : NB];
  int bn_[B_KC ? 1 : NB];  // unclamped first column of the thread's B quad (X2: columns past N are zeroed at the split)
  if (!B_KC) {
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      bn_[i] = n0 + ((BT ? tid : tid + 256 * i) % (BN / 4)) * 4;
      const int n = bn_[i] < N ? bn_[i] : 0;  // a quad past N reads column 0 (in bounds; its outputs are dropped)
      if (g.nimg > 0) {
        const int img = n / g.nimg;
        bcol[i] = (long)img * g.b_bs + (n - img * g.nimg);
      } else {
        bcol[i] = n;
      }
    }
  }

  if (A_LN) {
    for (int r = tid; r < BM; r += 256) {
      const int m = m0 + r;
      const float2 st = (m < M) ? *reinterpret_cast<const float2*>(g.ln_stats + 2L * m) : make_float2(0.f, 0.f);
      s_mean[r] = st.x;
      s_rstd[r] = st.y;
    }
  }

  // native vectors: a float4 (struct) copied global -> array -> LDS stays a memcpy through a stack array
  f32x4 ra[NA], rb[NB], lw, lb;
  float rng = 0.f;  // X2: largest magnitude split (scaled operands), split-range guard
  const float sa = (X2 && g.x2_sa != 0.f) ? g.x2_sa : 1.f, sb = (X2 && g.x2_sb != 0.f) ? g.x2_sb : 1.f;
  // per-thread operand pointers at k = 0 (a k block adds k0 or k0 * ldb); rows past M / N clamped
  const float* pa[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int idx = tid + 256 * i;
    const int m = m0 + (idx >> 3);
    pa[i] = A + (long)(m < M ? m : M - 1) * g.lda + (idx & 7) * 4;
  }
  const float* pb[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int idx = tid + 256 * i;
    if (B_KC) {
      const int n = n0 + (idx >> 3);
      pb[i] = B + (long)(n < N ? n : N - 1) * g.ldb + (idx & 7) * 4;
    } else {
      const int kl = BT ? 4 * (tid / (BN / 4)) + i : idx / (BN / 4);
      pb[i] = B + (long)kl * g.ldb + bcol[i];
    }
  }
  // Tile loads without per-lane predicates: rows past M / N read the clamped row (pa / pb), an N-contiguous quad
  // past N reads column 0 and a partial quad reads on to ldb (ldb % 4 == 0: in bounds); those products only reach
  // outputs the epilogue never stores. A predicated load merges into a phi whose copy waited for every load in
  // flight (vmcnt(0) after each load of a ragged tile).
  auto load_tiles = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NA; ++i) ra[i] = *reinterpret_cast<const f32x4*>(pa[i] + k0);
    if (A_LN) {  // every A float4 of this thread sits at the same k offset (256 % 8 == 0)
      lw = *reinterpret_cast<const f32x4*>(g.ln_w + k0 + (tid & 7) * 4);
      lb = *reinterpret_cast<const f32x4*>(g.ln_b + k0 + (tid & 7) * 4);
    }
    if (B_KC || vec_b) {
#pragma unroll
      for (int i = 0; i < NB; ++i)
        rb[i] = *reinterpret_cast<const f32x4*>(pb[i] + (B_KC ? (long)k0 : (long)k0 * g.ldb));
      return;
    }
    // an N-contiguous B whose rows are not 16-byte aligned (odd H*W; off the hot path): predicated element loads
    // (BT: thread t loads rows 4 (t / (BN/4)) + i of its column quad 4 (t % (BN/4)))
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int n = bn_[i];
      const float* src = pb[i] + (long)k0 * g.ldb;
      rb[i].x = (n < N) ? src[0] : 0.f;
      rb[i].y = (n + 1 < N) ? src[1] : 0.f;
      rb[i].z = (n + 2 < N) ? src[2] : 0.f;
      rb[i].w = (n + 3 < N) ? src[3] : 0.f;
    }
  };
  auto store_tiles = [&](int buf) {
    float* Ab = As + buf * A_ELEMS;
    float* Bb = Bs + buf * B_ELEMS;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int idx = tid + 256 * i;
      const int r = idx >> 3, kq = (idx & 7) * 4;
      f32x4 v = ra[i];
      if (A_LN) {
        const float mu = s_mean[r], rs = s_rstd[r];
        v.x = (v.x - mu) * rs * lw.x + lb.x;
        v.y = (v.y - mu) * rs * lw.y + lb.y;
        v.z = (v.z - mu) * rs * lw.z + lb.z;
        v.w = (v.w - mu) * rs * lw.w + lb.w;
      }
      if (X2) {
        uint2 h, l;
        split4(f32x4{v.x, v.y, v.z, v.w} * sa, h, l);
        rng = range_acc(rng, f32x4{v.x, v.y, v.z, v.w} * sa);
        h16_t* d = reinterpret_cast<h16_t*>(Ab) + r * (2 * SK) + 16 * (kq >> 3) + (kq & 7);
        *reinterpret_cast<uint2*>(d) = h;
        *reinterpret_cast<uint2*>(d + 8) = l;
      } else {
        *reinterpret_cast<f32x4*>(&Ab[r * SK + kq]) = v;
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int idx = tid + 256 * i;
      if (BT) {
        if (i == 0) {  // the whole 4x4 block: column quad 4 (tid % (BN/4)), k rows kq .. kq + 3
          const int nq = (tid % (BN / 4)) * 4, kq = 4 * (tid / (BN / 4));
          const f32x4 r4[4] = {f32x4{rb[0].x, rb[0].y, rb[0].z, rb[0].w}, f32x4{rb[1].x, rb[1].y, rb[1].z, rb[1].w},
                               f32x4{rb[2].x, rb[2].y, rb[2].z, rb[2].w}, f32x4{rb[3].x, rb[3].y, rb[3].z, rb[3].w}};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            // columns past N (read from column 0 or past the row end) are zeroed here, after the wait the split
            // needs anyway, so the range guard sees operand values only
            const f32x4 col = bn_[0] + j < N ? f32x4{r4[0][j], r4[1][j], r4[2][j], r4[3][j]} * sb
                                              : f32x4{0.f, 0.f, 0.f, 0.f};
            uint2 h, l;
            split4(col, h, l);
            rng = range_acc(rng, col);
            h16_t* d = reinterpret_cast<h16_t*>(Bb) + (nq + j) * (2 * SK) + 16 * (kq >> 3) + (kq & 7);
            *reinterpret_cast<uint2*>(d) = h;
            *reinterpret_cast<uint2*>(d + 8) = l;
          }
        }
      } else if (B_KC && X2) {
        const int r = idx >> 3, kq = (idx & 7) * 4;
        uint2 h, l;
        split4(f32x4{rb[i].x, rb[i].y, rb[i].z, rb[i].w} * sb, h, l);
        rng = range_acc(rng, f32x4{rb[i].x, rb[i].y, rb[i].z, rb[i].w} * sb);
        h16_t* d = reinterpret_cast<h16_t*>(Bb) + r * (2 * SK) + 16 * (kq >> 3) + (kq & 7);
        *reinterpret_cast<uint2*>(d) = h;
        *reinterpret_cast<uint2*>(d + 8) = l;
      } else if (B_KC) {
        const int r = idx >> 3, kq = (idx & 7) * 4;
        *reinterpret_cast<f32x4*>(&Bb[r * SK + kq]) = rb[i];
      } else {
        const int kl = idx / (BN / 4), nq = (idx % (BN / 4)) * 4;
        f32x4 v = rb[i];
        if (X2) {  // the split reads these columns from LDS: columns past N zeroed for the range guard
          const int n = bn_[i];
          v = f32x4{n < N ? v.x : 0.f, n + 1 < N ? v.y : 0.f, n + 2 < N ? v.z : 0.f, n + 3 < N ? v.w : 0.f};
        }
        *reinterpret_cast<f32x4*>(&Bb[kl * SBN + nq]) = v;
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

#ifdef YS_GEMM_HALFK  // diagnostic builds only: half the k blocks (timing of the main loop vs the rest; wrong results)
  const int nk = K / BK / 2;
#else
  const int nk = K / BK;
#endif
  const int lr = lane & 31, lh = lane >> 5;
  load_tiles(0);
  if (A_LN) __syncthreads();  // s_mean / s_rstd
  store_tiles(0);
  __syncthreads();
  for (int kb = 0; kb < nk; ++kb) {
    const int buf = kb & 1;
    load_tiles((kb + 1 < nk ? kb + 1 : kb) * BK);  // unconditional (the last trip reloads its own tile)
    __builtin_amdgcn_sched_barrier(0);  // the next tile's loads stay ahead of this tile's MFMAs
    const float* Ab = As + buf * A_ELEMS + (wm * MI * 32 + lr) * SK + lh * 16;
    const float* Bb = Bs + buf * B_ELEMS;
    if constexpr (X2) {
      const h16_t* Ah = reinterpret_cast<const h16_t*>(As + buf * A_ELEMS) + (wm * MI * 32 + lr) * (2 * SK);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int ko = 16 * (2 * lh + s2);  // this lane half's k group (2*lh + s2) in the split image
        f16x8_t ah[MI], al[MI], bh[NI], bl[NI];
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          ah[i] = *reinterpret_cast<const f16x8_t*>(Ah + i * 32 * (2 * SK) + ko);
          al[i] = *reinterpret_cast<const f16x8_t*>(Ah + i * 32 * (2 * SK) + ko + 8);
        }
        if constexpr (B_IMG) {
          const h16_t* Bh = reinterpret_cast<const h16_t*>(Bb) + (wn * NI * 32 + lr) * (2 * SK);
#pragma unroll
          for (int j = 0; j < NI; ++j) {
            bh[j] = *reinterpret_cast<const f16x8_t*>(Bh + j * 32 * (2 * SK) + ko);
            bl[j] = *reinterpret_cast<const f16x8_t*>(Bh + j * 32 * (2 * SK) + ko + 8);
          }
        } else {
#pragma unroll
          for (int j = 0; j < NI; ++j) {
            const float* col = Bb + (8 * (2 * lh + s2)) * SBN + wn * NI * 32 + j * 32 + lr;
            const f32x4 c0 = f32x4{col[0], col[SBN], col[2 * SBN], col[3 * SBN]} * sb;
            const f32x4 c1 = f32x4{col[4 * SBN], col[5 * SBN], col[6 * SBN], col[7 * SBN]} * sb;
            split8(c0, c1, bh[j], bl[j]);
            rng = range_acc(range_acc(rng, c0), c1);
          }
        }
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
          }
      }
    } else
#pragma unroll
    for (int t4 = 0; t4 < 4; ++t4) {
      float4 a[MI], b[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) a[i] = *reinterpret_cast<const float4*>(Ab + i * 32 * SK + 4 * t4);
      if (B_KC) {
#pragma unroll
        for (int j = 0; j < NI; ++j)
          b[j] = *reinterpret_cast<const float4*>(Bb + (wn * NI * 32 + j * 32 + lr) * SK + lh * 16 + 4 * t4);
      } else {
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          const float* col = Bb + (lh * 16 + 4 * t4) * SBN + wn * NI * 32 + j * 32 + lr;
          b[j] = make_float4(col[0], col[SBN], col[2 * SBN], col[3 * SBN]);
        }
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].x, b[j].x, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].y, b[j].y, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].z, b[j].z, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].w, b[j].w, acc[i][j], 0, 0, 0);
        }
    }
    if (kb + 1 < nk) store_tiles(buf ^ 1);
    __syncthreads();
  }

  if (X2) range_report(g.range_flag, rng);
  if (X2 && sa * sb != 1.f) {
    const float inv = 1.0f / (sa * sb);  // exact: powers of two
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc[i][j] *= inv;
  }
  const Epi& e = g.epi;
  if (e.vec) {
    // stage C through LDS (the main-loop buffers are free after the last barrier), then 16-byte row stores.
    // C/D map of 32x32: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
    float* Cs = smem;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          Cs[(wm * MI * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh) * SC + wn * NI * 32 + j * 32 + lr] =
              acc[i][j][r];
    __syncthreads();
    constexpr int NQ = BN / 4;
    float* outb = e.out + (long)bz * e.out_bs;
    const float* resb = e.res ? e.res + (long)bz * e.res_bs : nullptr;
#pragma unroll 4
    for (int idx = tid; idx < BM * NQ; idx += 256) {
      const int row = idx / NQ, c4 = idx % NQ;
      const int m = m0 + row;
      int n = n0 + 4 * c4;
      if (m >= M || n >= N) continue;
      float* ob = outb;
      const float* rb_ = resb;
      if (g.nimg > 0) {  // folded batch (bias / BN per row only)
        const int img = n / g.nimg;
        n -= img * g.nimg;
        ob += (long)img * e.out_bs;
        if (rb_) rb_ += (long)img * e.res_bs;
      }
      f32x4 v = *reinterpret_cast<const f32x4*>(&Cs[row * SC + 4 * c4]);
      if (e.bias_mode == 1) v += e.bias[m];
      else if (e.bias_mode == 2) v += *reinterpret_cast<const f32x4*>(e.bias + n);
      if (e.bn_mode == 1) v = v * e.scale[m] + e.shift[m];
      else if (e.bn_mode == 2)
        v = v * *reinterpret_cast<const f32x4*>(e.scale + n) + *reinterpret_cast<const f32x4*>(e.shift + n);
      v.x = apply_act(v.x, e.act); v.y = apply_act(v.y, e.act); v.z = apply_act(v.z, e.act); v.w = apply_act(v.w, e.act);
      if (rb_) v += *reinterpret_cast<const f32x4*>(rb_ + (long)m * e.ldr + n);
      *reinterpret_cast<f32x4*>(ob + (long)m * e.ldc + n) = v;
    }
    return;
  }

  // scalar epilogue (window-reverse scatter of the Swin pw conv, or unaligned outputs)
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int n = n0 + wn * NI * 32 + j * 32 + lr;
    if (n >= N) continue;
    long col_off;  // output offset of (m = 0, n)
    long m_stride;
    if (!e.swin) {
      col_off = (long)bz * e.out_bs + n;
      m_stride = e.ldc;
    } else {
      const int L = e.sw_wh * e.sw_ww;
      const int per_img = e.sw_nWin * L;
      const int img = n / per_img;
      const int rr = n - img * per_img;
      const int win = rr / L, tok = rr - win * L;
      const int wy = win / e.sw_nWx, wx = win - wy * e.sw_nWx;
      const int iy = tok / e.sw_ww, ix = tok - iy * e.sw_ww;
      const int h = wy * e.sw_wh + iy, w = wx * e.sw_ww + ix;
      if (h >= e.sw_H || w >= e.sw_W) continue;  // crop of the zero-padded border (blocks_transformer.py:125-129)
      m_stride = (long)e.sw_H * e.sw_W;
      col_off = (long)img * e.ldc * m_stride + (long)h * e.sw_W + w;  // ldc = channels
    }
    const long rcol_off = e.swin ? col_off : (long)bz * e.res_bs + n;
    const long r_stride = e.swin ? m_stride : e.ldr;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * MI * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m >= M) continue;
        float v = epi_value(e, m, n, acc[i][j][r]);
        if (e.res) v += e.res[rcol_off + (long)m * r_stride];
        e.out[col_off + (long)m * m_stride] = v;
      }
  }
}

static inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// test hook state: 1 = every gemm_f32 call takes the fp16-split products (yolosod_debug_set_gemm_x2), -1 = as asked
inline int& gemm_x2_forced() {
  static int v = -1;
  return v;
}

static inline int launch_gemm(const GemmArgs& g0, int batch, bool b_kc, hipStream_t st) {
  GemmArgs g = g0;
  YS_CHECK_ARG(g.K % 32 == 0, "gemm: K=%d must be a multiple of 32", g.K);
  YS_CHECK_ARG(g.lda % 4 == 0 && (!b_kc || g.ldb % 4 == 0),
               "gemm: lda (and ldb of a K-contiguous B) must be multiples of 4");
  YS_CHECK_ARG(al16(g.A) && al16(g.B), "gemm: A/B must be 16-byte aligned");
  YS_CHECK_ARG(!g.ln_w || (al16(g.ln_w) && al16(g.ln_b) && g.ln_stats && ((uintptr_t)g.ln_stats & 7) == 0),
               "gemm: LN params must be 16-byte aligned and come with row statistics");
  if (g.M == 0 || g.N == 0 || batch == 0) return 0;
  const Epi& e = g.epi;
  g.epi.vec = !e.swin && g.N % 4 == 0 && e.ldc % 4 == 0 && e.out_bs % 4 == 0 && al16(e.out) &&
              (!e.res || (e.ldr % 4 == 0 && e.res_bs % 4 == 0 && al16(e.res))) &&
              (e.bias_mode != 2 || al16(e.bias)) && (e.bn_mode != 2 || (al16(e.scale) && al16(e.shift)));
  const bool ln = g.ln_w != nullptr;
  const bool x2 = g.x2 != 0 || gemm_x2_forced() == 1;
  // N-contiguous B with a per-image N that is not a multiple of 128 (A2 at 640: H*W = 400): fold the batch into N so
  // the tiles run across image boundaries instead of padding every image's last tile column
  g.nimg = 0;
  g.nmajor = 0;
  g.bfold = 0;
  if (!b_kc && batch > 1 && g.a_bs == 0 && g.N % 128 != 0 && g.N % 4 == 0 && g.epi.vec && e.bias_mode != 2 && e.bn_mode != 2 &&
      g.ldb % 4 == 0 && g.b_bs % 4 == 0 && (long)g.N * batch < (1L << 31)) {
    g.nimg = g.N;
    g.nmajor = 1;
    g.N *= batch;
    batch = 1;
  }
  // K-contiguous per-image B with a shared A (the A2 output GEMM: B = the image's tokens): the batch goes into the
  // tile index and the tiles run n-major, so the M tiles reading one B column block sit on one XCD (B read once)
  const int batch0 = batch;
  if (b_kc && batch > 1 && g.a_bs == 0 && (long)batch * ((g.M + 63) / 64) * ((g.N + 63) / 64) < (1L << 30)) {
    g.bfold = batch;
    g.nmajor = 1;
    batch = 1;
  }
  g.range_flag = x2 ? range_flag_dev() : nullptr;
  // N tiles of 64 when N is not a multiple of 128 (e.g. 3C = 192) or small; 128 otherwise
  const bool narrow = (g.N % 128 != 0) && (g.N <= 256);
#define YS_GEMM_LAUNCH(WM_, WN_, MI_, NI_)                                                                     \
  do {                                                                                                         \
    constexpr int bm = WM_ * MI_ * 32, bn = WN_ * NI_ * 32;                                                    \
    g.tiles_n = (g.N + bn - 1) / bn;                                                                           \
    g.tiles = g.tiles_n * ((g.M + bm - 1) / bm);                                                               \
    const long nt_ = (long)g.tiles * (g.bfold ? g.bfold : 1);                                                  \
    dim3 grid((unsigned)(8 * ((nt_ + 7) / 8)), 1, batch);                                                      \
    if (x2) {                                                                                                  \
      if (b_kc) {                                                                                              \
        if (ln) hipLaunchKernelGGL((gemm_f32_kernel<WM_, WN_, MI_, NI_, true, true, true>), grid, dim3(256), 0, st, g); \
        else hipLaunchKernelGGL((gemm_f32_kernel<WM_, WN_, MI_, NI_, true, false, true>), grid, dim3(256), 0, st, g); \
      } else {                                                                                                 \
        if (ln) hipLaunchKernelGGL((gemm_f32_kernel<WM_, WN_, MI_, NI_, false, true, true>), grid, dim3(256), 0, st, g); \
        else hipLaunchKernelGGL((gemm_f32_kernel<WM_, WN_, MI_, NI_, false, false, true>), grid, dim3(256), 0, st, g); \
      }                                                                                                        \
    } else if (b_kc) {                                                                                         \
      if (ln) hipLaunchKernelGGL((gemm_f32_kernel<WM_, WN_, MI_, NI_, true, true>), grid, dim3(256), 0, st, g); \
      else hipLaunchKernelGGL((gemm_f32_kernel<WM_, WN_, MI_, NI_, true, false>), grid, dim3(256), 0, st, g);  \
    } else {                                                                                                   \
      if (ln) hipLaunchKernelGGL((gemm_f32_kernel<WM_, WN_, MI_, NI_, false, true>), grid, dim3(256), 0, st, g); \
      else hipLaunchKernelGGL((gemm_f32_kernel<WM_, WN_, MI_, NI_, false, false>), grid, dim3(256), 0, st, g); \
    }                                                                                                          \
  } while (0)
  constexpr int forced = 0;  // tile choice (A/B builds: 1 = 128x64, 2 = 128x128, 3 = 64x256)
  // 128x64 tiles also when 128x128 would leave CUs idle (fewer tiles than CUs) or waste > 10% of a tile column
  // on a ragged N (e.g. N = H*W = 400): more, smaller workgroups for the small A2 / MHA GEMMs
  const long t128 = (long)((g.M + 127) / 128) * ((g.N + 127) / 128) * batch0;
  const bool ragged = (long)((g.N + 127) / 128) * 128 - g.N > g.N / 10;
  const bool small = !narrow && g.M > 64 && (t128 < 256 || ragged);
  if (forced == 1 || (!forced && (narrow || small))) YS_GEMM_LAUNCH(4, 1, 1, 2);
  else if (forced == 3 || (!forced && g.M <= 64)) YS_GEMM_LAUNCH(1, 4, 2, 2);  // 64 x 256 tiles
  else YS_GEMM_LAUNCH(2, 2, 2, 2);
#undef YS_GEMM_LAUNCH
  YS_CHECK_LAUNCH("gemm_f32");
  return 0;
}

static inline Epi epi_plain(float* out, long out_bs, int ldc) {
  Epi e{};
  e.out = out;
  e.out_bs = out_bs;
  e.ldc = ldc;
  return e;
}

}  // namespace ys
