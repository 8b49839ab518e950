// Channel / spatial / coordinate attention of the Multi-Attention Fusion Neck: SE_Block, CBAM_Block, CA_Block.
//
// All three are HBM-bound (a few FLOPs per byte). Layout is the reference's NCHW fp32. Each op is split into
//   (1) a per-(b,c)-plane reduction pass (global-avg / global-max / row+column means),
//   (2) a tiny per-image gate computation folded into the prologue of the next pass, and
//   (3) one streaming apply pass that reads x once and writes y once (float4, coalesced).
// To keep the apply pass' re-read of x out of HBM, the host driver walks the batch in image chunks sized to
// stay resident in the 256 MiB Infinity Cache between the reduction pass and the apply pass.
//
// Reference semantics (file:line in quitedob/yolo-sod):
//   SE     ultralytics/nn/modules/smallobj_modules.py:84-92  (x * sigmoid(fc2(relu(fc1(mean_hw x)))))
//   CBAM   ultralytics/nn/modules/cbam_block.py:19-55         ((x*ca)*sa, ca from avg+max MLP, sa = 7x7 conv)
//   CA     ultralytics/nn/modules/ca_block.py:38-59           ((x*a_w)*a_h, h_sigmoid(BN(conv1(.))) gates)
#include "common.h"
#include <stdlib.h>
#include <math.h>

namespace ys {

static size_t mall_chunk_bytes() {
  static size_t v = [] {
    const char* e = getenv("YOLOSOD_MALL_CHUNK_MB");
    long mb = e ? atol(e) : 96;
    return (size_t)(mb < 0 ? 0 : mb) << 20;
  }();
  return v;
}

static int images_per_chunk(int B, size_t bytes_per_image) {
  size_t cap = mall_chunk_bytes();
  if (cap == 0 || bytes_per_image == 0) return B;
  size_t n = cap / bytes_per_image;
  if (n < 1) n = 1;
  if ((int)n > B) n = B;
  return (int)n;
}

// ------------------------------------------------------------------------------------------------
// (1) per-plane sum (+max): one 256-thread workgroup per (b,c) plane, float4 streaming, 4 loads in flight.
// ------------------------------------------------------------------------------------------------
template <bool WITH_MAX>
__global__ __launch_bounds__(256) void plane_stats_kernel(const float* __restrict__ x, long HW,
                                                          float* __restrict__ mean, float* __restrict__ mx) {
  const long plane = blockIdx.x;
  const float* p = x + plane * HW;
  float s = 0.f, m = -INFINITY;
  const int tid = threadIdx.x;
  if ((HW & 3) == 0) {
    const float4* p4 = reinterpret_cast<const float4*>(p);
    const long n4 = HW >> 2;
    long i = tid;
    for (; i + 3 * 256 < n4; i += 4 * 256) {
      float4 a = p4[i], b = p4[i + 256], c = p4[i + 512], d = p4[i + 768];
      s += ((a.x + a.y) + (a.z + a.w)) + ((b.x + b.y) + (b.z + b.w)) + ((c.x + c.y) + (c.z + c.w)) +
           ((d.x + d.y) + (d.z + d.w));
      if (WITH_MAX) {
        m = fmaxf(m, fmaxf(fmaxf(fmaxf(a.x, a.y), fmaxf(a.z, a.w)), fmaxf(fmaxf(b.x, b.y), fmaxf(b.z, b.w))));
        m = fmaxf(m, fmaxf(fmaxf(fmaxf(c.x, c.y), fmaxf(c.z, c.w)), fmaxf(fmaxf(d.x, d.y), fmaxf(d.z, d.w))));
      }
    }
    for (; i < n4; i += 256) {
      float4 a = p4[i];
      s += (a.x + a.y) + (a.z + a.w);
      if (WITH_MAX) m = fmaxf(m, fmaxf(fmaxf(a.x, a.y), fmaxf(a.z, a.w)));
    }
  } else {
    for (long i = tid; i < HW; i += 256) {
      float v = p[i];
      s += v;
      if (WITH_MAX) m = fmaxf(m, v);
    }
  }
  __shared__ float ss[4], sm[4];
  s = wave_sum(s);
  if (WITH_MAX) m = wave_max(m);
  const int w = tid >> 6;
  if ((tid & 63) == 0) {
    ss[w] = s;
    sm[w] = m;
  }
  __syncthreads();
  if (tid == 0) {
    float t = (ss[0] + ss[1]) + (ss[2] + ss[3]);
    mean[plane] = t / (float)HW;
    if (WITH_MAX) mx[plane] = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
  }
}

// ------------------------------------------------------------------------------------------------
// SE apply: gate a[b,c] = sigmoid(W2 relu(W1 m + b1) + b2) recomputed in the block prologue (hidden <= 64,
// C <= 4096), then y = x * a over a chunk of the plane. grid.x = planes * chunks_per_plane.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void se_apply_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                       const float* __restrict__ mean, int C, long HW,
                                                       int chunks, const float* __restrict__ w1,
                                                       const float* __restrict__ b1, const float* __restrict__ w2,
                                                       const float* __restrict__ b2, int hid) {
  const long plane = blockIdx.x / chunks;
  const int chunk = blockIdx.x % chunks;
  const int b = (int)(plane / C), c = (int)(plane % C);
  __shared__ float hsh[64];
  __shared__ float gate;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float* mb = mean + (long)b * C;
  for (int j = wv; j < hid; j += 4) {
    float acc = 0.f;
    for (int k = lane; k < C; k += 64) acc += w1[(long)j * C + k] * mb[k];
    acc = wave_sum(acc);
    if (lane == 0) hsh[j] = fmaxf(acc + b1[j], 0.f);
  }
  __syncthreads();
  if (tid == 0) {
    float z = 0.f;
    for (int j = 0; j < hid; ++j) z += w2[(long)c * hid + j] * hsh[j];
    gate = sigmoidf_(z + b2[c]);
  }
  __syncthreads();
  const float a = gate;
  const float* p = x + plane * HW;
  float* q = y + plane * HW;
  const long per = (HW + chunks - 1) / chunks;
  long s0 = chunk * per, s1 = s0 + per;
  if (s1 > HW) s1 = HW;
  if ((HW & 3) == 0 && (per & 3) == 0) {
    const float4* p4 = reinterpret_cast<const float4*>(p + s0);
    float4* q4 = reinterpret_cast<float4*>(q + s0);
    const long n4 = (s1 - s0) >> 2;
    for (long i = tid; i < n4; i += 256) {
      float4 v = p4[i];
      v.x *= a; v.y *= a; v.z *= a; v.w *= a;
      q4[i] = v;
    }
  } else {
    for (long i = s0 + tid; i < s1; i += 256) q[i] = p[i] * a;
  }
}

static int chunks_for_plane(long HW) {
  // ~16 KiB of x per workgroup keeps >= 8 waves/CU busy even for the smallest planes.
  long c = HW / 4096;
  if (c < 1) c = 1;
  if (c > 64) c = 64;
  // keep chunk length a multiple of 4 floats when possible
  while (c > 1 && ((HW + c - 1) / c) % 4 != 0) --c;
  return (int)c;
}

// ------------------------------------------------------------------------------------------------
// CBAM pass 2: per-pixel channel mean / max of o = ca[c] * x  ->  map[b][0|1][p].
// The block prologue computes ca[b, :] = sigmoid(fc(avg) + fc(max)) into LDS (fc = W2 relu(W1 .), no bias);
// block (0, b) also publishes ca to global for pass 3.
// ------------------------------------------------------------------------------------------------
template <int MAXC>
__device__ void cbam_channel_gate(const float* avg, const float* mx, const float* w1, const float* w2, int C, int hid,
                                  float* ca_sh, float* hsh) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // hidden activations of both branches: hsh[j] (avg), hsh[64+j] (max)
  for (int j = wv; j < 2 * hid; j += 4) {
    const int jj = j % hid;
    const float* v = (j < hid) ? avg : mx;
    float acc = 0.f;
    for (int k = lane; k < C; k += 64) acc += w1[(long)jj * C + k] * v[k];
    acc = wave_sum(acc);
    if (lane == 0) hsh[(j < hid ? 0 : 64) + jj] = fmaxf(acc, 0.f);
  }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    float za = 0.f, zm = 0.f;
    for (int j = 0; j < hid; ++j) {
      const float wcj = w2[(long)c * hid + j];
      za += wcj * hsh[j];
      zm += wcj * hsh[64 + j];
    }
    ca_sh[c] = sigmoidf_(za + zm);
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void cbam_pixel_stats_kernel(const float* __restrict__ x, const float* __restrict__ avg,
                                                               const float* __restrict__ mx, const float* __restrict__ w1,
                                                               const float* __restrict__ w2, int C, int hid, long HW,
                                                               float* __restrict__ ca_out, float* __restrict__ map) {
  __shared__ float ca_sh[4096];
  __shared__ float hsh[128];
  const int b = blockIdx.y;
  cbam_channel_gate<4096>(avg + (long)b * C, mx + (long)b * C, w1, w2, C, hid, ca_sh, hsh);
  if (blockIdx.x == 0)
    for (int c = threadIdx.x; c < C; c += 256) ca_out[(long)b * C + c] = ca_sh[c];
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= HW) return;
  const float* xb = x + (long)b * C * HW + p;
  float s = 0.f, m = -INFINITY;
  int c = 0;
  for (; c + 8 <= C; c += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = xb[(long)(c + u) * HW];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float o = ca_sh[c + u] * v[u];
      s += o;
      m = fmaxf(m, o);
    }
  }
  for (; c < C; ++c) {
    const float o = ca_sh[c] * xb[(long)c * HW];
    s += o;
    m = fmaxf(m, o);
  }
  float* mp = map + (long)b * 2 * HW;
  mp[p] = s / (float)C;
  mp[HW + p] = m;
}

// CBAM pass 3: sa = sigmoid(conv7x7([mean;max]), pad 3, no bias); y = sa * (ca[c] * x).
__global__ __launch_bounds__(256) void cbam_apply_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                         const float* __restrict__ ca, const float* __restrict__ map,
                                                         const float* __restrict__ wsa, int C, int H, int W) {
  __shared__ float wk[98];
  if (threadIdx.x < 98) wk[threadIdx.x] = wsa[threadIdx.x];
  __syncthreads();
  const int b = blockIdx.y;
  const long HW = (long)H * W;
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= HW) return;
  const int py = (int)(p / W), px = (int)(p % W);
  const float* mp = map + (long)b * 2 * HW;
  float z = 0.f;
  for (int ci = 0; ci < 2; ++ci) {
    const float* m = mp + ci * HW;
    for (int ky = 0; ky < 7; ++ky) {
      const int yy = py + ky - 3;
      if (yy < 0 || yy >= H) continue;
      for (int kx = 0; kx < 7; ++kx) {
        const int xx = px + kx - 3;
        if (xx < 0 || xx >= W) continue;
        z += wk[ci * 49 + ky * 7 + kx] * m[(long)yy * W + xx];
      }
    }
  }
  const float sa = sigmoidf_(z);
  const float* xb = x + (long)b * C * HW + p;
  float* yb = y + (long)b * C * HW + p;
  const float* cab = ca + (long)b * C;
  int c = 0;
  for (; c + 8 <= C; c += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = xb[(long)(c + u) * HW];
#pragma unroll
    for (int u = 0; u < 8; ++u) yb[(long)(c + u) * HW] = sa * (cab[c + u] * v[u]);
  }
  for (; c < C; ++c) yb[(long)c * HW] = sa * (cab[c] * xb[(long)c * HW]);
}

// ------------------------------------------------------------------------------------------------
// CA pass 1: row means (over W) and column means (over H) of each (b,c) plane -> yin[b][c][0..H+W).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void ca_pool_kernel(const float* __restrict__ x, int H, int W, float* __restrict__ yin) {
  const long plane = blockIdx.x;
  const float* p = x + plane * (long)H * W;
  float* o = yin + plane * (long)(H + W);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int h = wv; h < H; h += 4) {
    float s = 0.f;
    for (int w = lane; w < W; w += 64) s += p[(long)h * W + w];
    s = wave_sum(s);
    if (lane == 0) o[h] = s / (float)W;
  }
  for (int w = tid; w < W; w += 256) {
    float s = 0.f;
    for (int h = 0; h < H; ++h) s += p[(long)h * W + w];
    o[H + w] = s / (float)H;
  }
}

// CA pass 2: per position p of the concatenated (H+W) axis:
//   t[j]   = h_sigmoid(BN(sum_c W1[j][c] yin[c][p] + b1[j]))        (conv1 + bn1 + act; BN eval, eps given)
//   gate[c][p] = sigmoid(sum_j Wx[c][j] t[j] + bx[c]),  Wx = conv_h for p < H, conv_w otherwise.
// grid = (ceil((H+W)/16), B); 256 threads.
__global__ __launch_bounds__(256) void ca_gate_kernel(const float* __restrict__ yin, int C, int H, int W, int mip,
                                                      const float* __restrict__ w1, const float* __restrict__ b1,
                                                      const float* __restrict__ bn_w, const float* __restrict__ bn_b,
                                                      const float* __restrict__ bn_m, const float* __restrict__ bn_v,
                                                      float bn_eps, const float* __restrict__ wh,
                                                      const float* __restrict__ bh, const float* __restrict__ ww,
                                                      const float* __restrict__ bw, float* __restrict__ gate) {
  constexpr int P = 16;
  __shared__ float t_sh[P][65];
  const int b = blockIdx.y;
  const int L = H + W;
  const int p0 = blockIdx.x * P;
  const int tid = threadIdx.x;
  const float* yb = yin + (long)b * C * L;
  // t: P x mip outputs, one thread each (mip <= 64 -> P*mip <= 1024, loop)
  for (int o = tid; o < P * mip; o += 256) {
    const int pp = o / mip, j = o % mip;
    const int p = p0 + pp;
    if (p >= L) continue;
    float acc = 0.f;
    for (int c = 0; c < C; ++c) acc += w1[(long)j * C + c] * yb[(long)c * L + p];
    float z = acc + b1[j];
    const float inv = 1.0f / sqrtf(bn_v[j] + bn_eps);
    z = (z - bn_m[j]) * inv * bn_w[j] + bn_b[j];
    z = fminf(fmaxf(z + 3.0f, 0.0f), 6.0f) / 6.0f;
    t_sh[pp][j] = z;
  }
  __syncthreads();
  float* gb = gate + (long)b * C * L;
  for (int o = tid; o < P * C; o += 256) {
    const int c = o / P, pp = o % P;
    const int p = p0 + pp;
    if (p >= L) continue;
    const float* wx = (p < H) ? wh : ww;
    const float bx = (p < H) ? bh[c] : bw[c];
    float acc = 0.f;
    for (int j = 0; j < mip; ++j) acc += wx[(long)c * mip + j] * t_sh[pp][j];
    gb[(long)c * L + p] = sigmoidf_(acc + bx);
  }
}

// CA pass 3: y[b,c,h,w] = (x * a_w[b,c,w]) * a_h[b,c,h]; gate rows are [a_h (H) | a_w (W)].
__global__ __launch_bounds__(256) void ca_apply_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                       const float* __restrict__ gate, int H, int W, long total) {
  const long L = H + W;
  if ((W & 3) == 0) {
    const long n4 = total >> 2;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
      const long e = i << 2;
      const long plane = e / ((long)H * W);
      const long r = e % ((long)H * W);
      const int h = (int)(r / W), w = (int)(r % W);
      const float* g = gate + plane * L;
      const float ah = g[h];
      float4 v = reinterpret_cast<const float4*>(x)[i];
      v.x = (v.x * g[H + w]) * ah;
      v.y = (v.y * g[H + w + 1]) * ah;
      v.z = (v.z * g[H + w + 2]) * ah;
      v.w = (v.w * g[H + w + 3]) * ah;
      reinterpret_cast<float4*>(y)[i] = v;
    }
  } else {
    for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
      const long plane = e / ((long)H * W);
      const long r = e % ((long)H * W);
      const int h = (int)(r / W), w = (int)(r % W);
      const float* g = gate + plane * L;
      y[e] = (x[e] * g[H + w]) * g[h];
    }
  }
}

static int grid_stride_blocks(long work_items) {
  long b = (work_items + 255) / 256;
  if (b > 256L * 16) b = 256L * 16;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace ys

using namespace ys;

// =================================================================================================
// C ABI
// =================================================================================================
YS_EXPORT size_t yolosod_se_workspace(int B, int C, int H, int W) {
  Sizer s;
  s.take<float>((size_t)B * C);
  return s.off;
}

YS_EXPORT int yolosod_se_forward(const float* x, float* y, int B, int C, int H, int W, const float* fc1_w,
                                 const float* fc1_b, const float* fc2_w, const float* fc2_b, int hidden,
                                 void* workspace, size_t workspace_bytes, void* stream) {
  YS_CHECK_ARG(x && y && fc1_w && fc1_b && fc2_w && fc2_b, "se: null pointer");
  YS_CHECK_ARG(B >= 0 && C > 0 && H > 0 && W > 0, "se: bad shape");
  YS_CHECK_ARG(hidden > 0 && hidden <= 64, "se: hidden=%d unsupported (1..64)", hidden);
  if (B == 0) return 0;
  Carver cv(workspace, workspace_bytes);
  float* mean = cv.take<float>((size_t)B * C);
  YS_CHECK_ARG(mean, "se: workspace too small (%zu)", workspace_bytes);
  hipStream_t st = (hipStream_t)stream;
  const long HW = (long)H * W;
  const int chunks = chunks_for_plane(HW);
  const int ipc = images_per_chunk(B, (size_t)C * HW * sizeof(float));
  for (int b0 = 0; b0 < B; b0 += ipc) {
    const int nb = (B - b0 < ipc) ? B - b0 : ipc;
    const long off = (long)b0 * C * HW;
    hipLaunchKernelGGL((plane_stats_kernel<false>), dim3(nb * C), dim3(256), 0, st, x + off, HW, mean + (long)b0 * C,
                       nullptr);
    hipLaunchKernelGGL(se_apply_kernel, dim3((unsigned)(nb * C * chunks)), dim3(256), 0, st, x + off, y + off,
                       mean + (long)b0 * C, C, HW, chunks, fc1_w, fc1_b, fc2_w, fc2_b, hidden);
  }
  YS_CHECK_LAUNCH("se");
  return 0;
}

YS_EXPORT size_t yolosod_cbam_workspace(int B, int C, int H, int W) {
  Sizer s;
  s.take<float>((size_t)B * C);  // avg
  s.take<float>((size_t)B * C);  // max
  s.take<float>((size_t)B * C);  // ca
  s.take<float>((size_t)B * 2 * H * W);  // [mean;max] map
  return s.off;
}

YS_EXPORT int yolosod_cbam_forward(const float* x, float* y, int B, int C, int H, int W, const float* fc0_w,
                                   const float* fc2_w, int hidden, const float* sa_w, void* workspace,
                                   size_t workspace_bytes, void* stream) {
  YS_CHECK_ARG(x && y && fc0_w && fc2_w && sa_w, "cbam: null pointer");
  YS_CHECK_ARG(B >= 0 && C > 0 && C <= 4096 && H > 0 && W > 0, "cbam: bad shape");
  YS_CHECK_ARG(hidden > 0 && hidden <= 64, "cbam: hidden=%d unsupported (1..64)", hidden);
  if (B == 0) return 0;
  Carver cv(workspace, workspace_bytes);
  float* avg = cv.take<float>((size_t)B * C);
  float* mx = cv.take<float>((size_t)B * C);
  float* ca = cv.take<float>((size_t)B * C);
  float* map = cv.take<float>((size_t)B * 2 * H * W);
  YS_CHECK_ARG(map, "cbam: workspace too small (%zu)", workspace_bytes);
  hipStream_t st = (hipStream_t)stream;
  const long HW = (long)H * W;
  const int ipc = images_per_chunk(B, (size_t)C * HW * sizeof(float));
  for (int b0 = 0; b0 < B; b0 += ipc) {
    const int nb = (B - b0 < ipc) ? B - b0 : ipc;
    const long off = (long)b0 * C * HW;
    hipLaunchKernelGGL((plane_stats_kernel<true>), dim3(nb * C), dim3(256), 0, st, x + off, HW,
                       avg + (long)b0 * C, mx + (long)b0 * C);
    dim3 g((unsigned)((HW + 255) / 256), nb);
    hipLaunchKernelGGL(cbam_pixel_stats_kernel, g, dim3(256), 0, st, x + off, avg + (long)b0 * C, mx + (long)b0 * C,
                       fc0_w, fc2_w, C, hidden, HW, ca + (long)b0 * C, map + (long)b0 * 2 * HW);
    hipLaunchKernelGGL(cbam_apply_kernel, g, dim3(256), 0, st, x + off, y + off, ca + (long)b0 * C,
                       map + (long)b0 * 2 * HW, sa_w, C, H, W);
  }
  YS_CHECK_LAUNCH("cbam");
  return 0;
}

YS_EXPORT size_t yolosod_ca_workspace(int B, int C, int H, int W) {
  Sizer s;
  s.take<float>((size_t)B * C * (H + W));  // pooled
  s.take<float>((size_t)B * C * (H + W));  // gates
  return s.off;
}

YS_EXPORT int yolosod_ca_forward(const float* x, float* y, int B, int C, int H, int W, const float* conv1_w,
                                 const float* conv1_b, int mip, const float* bn_w, const float* bn_b,
                                 const float* bn_mean, const float* bn_var, float bn_eps, const float* convh_w,
                                 const float* convh_b, const float* convw_w, const float* convw_b, void* workspace,
                                 size_t workspace_bytes, void* stream) {
  YS_CHECK_ARG(x && y && conv1_w && conv1_b && bn_w && bn_b && bn_mean && bn_var && convh_w && convh_b && convw_w &&
                   convw_b,
               "ca: null pointer");
  YS_CHECK_ARG(B >= 0 && C > 0 && H > 0 && W > 0, "ca: bad shape");
  YS_CHECK_ARG(mip > 0 && mip <= 64, "ca: mip=%d unsupported (1..64)", mip);
  if (B == 0) return 0;
  Carver cv(workspace, workspace_bytes);
  float* yin = cv.take<float>((size_t)B * C * (H + W));
  float* gate = cv.take<float>((size_t)B * C * (H + W));
  YS_CHECK_ARG(gate, "ca: workspace too small (%zu)", workspace_bytes);
  hipStream_t st = (hipStream_t)stream;
  const long HW = (long)H * W;
  const int ipc = images_per_chunk(B, (size_t)C * HW * sizeof(float));
  for (int b0 = 0; b0 < B; b0 += ipc) {
    const int nb = (B - b0 < ipc) ? B - b0 : ipc;
    const long off = (long)b0 * C * HW;
    const long goff = (long)b0 * C * (H + W);
    hipLaunchKernelGGL(ca_pool_kernel, dim3(nb * C), dim3(256), 0, st, x + off, H, W, yin + goff);
    hipLaunchKernelGGL(ca_gate_kernel, dim3((H + W + 15) / 16, nb), dim3(256), 0, st, yin + goff, C, H, W, mip,
                       conv1_w, conv1_b, bn_w, bn_b, bn_mean, bn_var, bn_eps, convh_w, convh_b, convw_w, convw_b,
                       gate + goff);
    const long total = (long)nb * C * HW;
    hipLaunchKernelGGL(ca_apply_kernel, dim3(grid_stride_blocks(((W & 3) == 0) ? total / 4 : total)), dim3(256), 0,
                       st, x + off, y + off, gate + goff, H, W, total);
  }
  YS_CHECK_LAUNCH("ca");
  return 0;
}
