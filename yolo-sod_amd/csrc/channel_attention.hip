// Channel / spatial / coordinate attention of the Multi-Attention Fusion Neck: SE_Block, CBAM_Block, CA_Block.
//
// All three are HBM-bound (a few FLOPs per byte). Layout is the reference's NCHW; storage is fp32 or bf16 (the
// bf16 model config), arithmetic always fp32. Each op is
//   (1) a reduction over x (per-plane sum/max split over several workgroups per plane, or row+column means) -
//       normally emitted by x's producing conv epilogue (conv_epilogue.hip), so no extra pass over x,
//   (2) the gate (the SE / CBAM channel MLP, the CA conv1+BN+h_sigmoid+conv_h/w gates),
//   (3) one streaming apply pass that reads x once and writes y once (coalesced vectors, every lane busy).
// SE recomputes its (tiny) channel MLP inside the apply workgroups: gate + scale is one launch. CBAM is three:
// channel gate + per-pixel channel mean/max of ca*x (per 32-channel group) in one, the 7x7 spatial conv, the apply.
// (A 2-launch CBAM with the spatial conv evaluated inside 1024-pixel apply workgroups - halo rows of the map in LDS,
// first channel slab prefetched across the conv - measured slower on MI355X: L4 0.186 vs 0.132 ms, L18 0.080 vs
// 0.053: far fewer workgroups stream the tensor, and the per-workgroup halo combine over the channel groups
// re-reads the partial maps; it was removed.)
// (Walking the batch in image chunks sized to stay resident in the 256 MiB Infinity Cache between the passes was
// measured on MI355X at the bs=32 640x640 shapes: the apply pass' re-read does hit on-die (7.3 TB/s) but the extra
// launch boundaries and the smaller grids cost more - SE L1 0.269 vs 0.243 ms, CBAM L4 0.199 vs 0.163, CA L32 0.090
// vs 0.073 - so every pass covers the whole batch.)
//
// Reference semantics (file:line in quitedob/yolo-sod):
//   SE     ultralytics/nn/modules/smallobj_modules.py:84-92  (x * sigmoid(fc2(relu(fc1(mean_hw x)))))
//   CBAM   ultralytics/nn/modules/cbam_block.py:19-55         ((x*ca)*sa, ca from avg+max MLP, sa = 7x7 conv)
//   CA     ultralytics/nn/modules/ca_block.py:38-59           ((x*a_w)*a_h, h_sigmoid(BN(conv1(.))) gates)
#include "common.h"
#include <stdlib.h>
#include <math.h>

namespace ys {

constexpr int kMaxParts = 64;

// How many workgroups reduce one plane: one per 8192 elements, so the big early planes (SE at 320x320, CBAM at
// 160x160) still launch thousands of workgroups per chunk. Depends on the plane size only, never on the batch or
// the storage type, so results are bitwise independent of batch size, chunking and sharding.
struct PartPlan {
  int parts;
  long seg;
};
static PartPlan part_plan(long HW) {
  long p = HW / 8192;
  if (p > kMaxParts) p = kMaxParts;
  if (p < 1) p = 1;
  long seg = (HW + p - 1) / p;
  if ((HW & 3) == 0) seg = (seg + 3) & ~3L;
  p = (HW + seg - 1) / seg;
  return {(int)p, seg};
}

// ------------------------------------------------------------------------------------------------
// (1) per-plane partial sum (+max): workgroup (plane, k) reduces x[plane][k*seg, (k+1)*seg) with four vector
// loads in flight per lane; partials land in psum/pmax[plane * parts + k].
// ------------------------------------------------------------------------------------------------
template <bool WITH_MAX, class T>
__global__ __launch_bounds__(256) void plane_part_stats_kernel(const T* __restrict__ x, long HW, int parts,
                                                               long seg, float* __restrict__ psum,
                                                               float* __restrict__ pmax) {
  const long plane = blockIdx.x / parts;
  const int k = blockIdx.x % parts;
  const long s0 = k * seg;
  const long s1 = (s0 + seg < HW) ? s0 + seg : HW;
  const T* p = x + plane * HW;
  float s = 0.f, m = -INFINITY;
  const int tid = threadIdx.x;
  if ((HW & 3) == 0) {
    const T* p4 = p + s0;
    const long n4 = (s1 - s0) >> 2;
    long i = tid;
    for (; i + 3 * 256 < n4; i += 4 * 256) {
      f32x4 a = ld4(p4 + 4 * i), b = ld4(p4 + 4 * (i + 256)), c = ld4(p4 + 4 * (i + 512)), d = ld4(p4 + 4 * (i + 768));
      s += ((a.x + a.y) + (a.z + a.w)) + ((b.x + b.y) + (b.z + b.w)) + ((c.x + c.y) + (c.z + c.w)) +
           ((d.x + d.y) + (d.z + d.w));
      if (WITH_MAX) {
        m = fmaxf(m, fmaxf(fmaxf(fmaxf(a.x, a.y), fmaxf(a.z, a.w)), fmaxf(fmaxf(b.x, b.y), fmaxf(b.z, b.w))));
        m = fmaxf(m, fmaxf(fmaxf(fmaxf(c.x, c.y), fmaxf(c.z, c.w)), fmaxf(fmaxf(d.x, d.y), fmaxf(d.z, d.w))));
      }
    }
    for (; i < n4; i += 256) {
      f32x4 a = ld4(p4 + 4 * i);
      s += (a.x + a.y) + (a.z + a.w);
      if (WITH_MAX) m = fmaxf(m, fmaxf(fmaxf(a.x, a.y), fmaxf(a.z, a.w)));
    }
  } else {
    for (long i = s0 + tid; i < s1; i += 256) {
      float v = ld1(p + i);
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
    psum[blockIdx.x] = (ss[0] + ss[1]) + (ss[2] + ss[3]);
    if (WITH_MAX) pmax[blockIdx.x] = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
  }
}

// ------------------------------------------------------------------------------------------------
// (2) channel gates of one image, computed by one workgroup (256 threads) into LDS:
//   SE:   gate[c] = sigmoid(W2 relu(W1 mean + b1) + b2)
//   CBAM: gate[c] = sigmoid(W2 relu(W1 avg) + W2 relu(W1 max))     (no biases, cbam_block.py:14-17)
// avg / mx: LDS [C] each, hsh: LDS [128]. Only channels [c0, c0 + n) of the output are produced, into out[0, n).
// The summation orders are fixed (partials in k order, the hidden dot products as a wave reduction), so every
// workgroup that recomputes a gate gets the same bits.
// ------------------------------------------------------------------------------------------------
template <bool CBAM>
__device__ __forceinline__ void gate_mlp(const float* __restrict__ psum, const float* __restrict__ pmax, int parts,
                                         int C, float inv_hw, const float* __restrict__ w1,
                                         const float* __restrict__ b1, const float* __restrict__ w2,
                                         const float* __restrict__ b2, int hid, int b, float* avg, float* mx,
                                         float* hsh, int c0, int n, float* out) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int c = tid; c < C; c += 256) {
    // the plane's partials as 8-deep batches of independent loads, accumulated in k order (the same bits as a plain
    // k loop, which waited for each load in turn: up to 64 L2 round trips before the gate could start)
    const float* ps = psum + ((long)b * C + c) * parts;
    const float* pm = CBAM ? pmax + ((long)b * C + c) * parts : nullptr;
    float s = 0.f, m = -INFINITY;
    int k = 0;
    for (; k + 8 <= parts; k += 8) {
      float v[8], w[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        v[u] = ps[k + u];
        if (CBAM) w[u] = pm[k + u];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s += v[u];
        if (CBAM) m = fmaxf(m, w[u]);
      }
    }
    for (; k < parts; ++k) {
      s += ps[k];
      if (CBAM) m = fmaxf(m, pm[k]);
    }
    avg[c] = s * inv_hw;
    if (CBAM) mx[c] = m;
  }
  __syncthreads();
  const int nh = CBAM ? 2 * hid : hid;
  for (int j = wv; j < nh; j += 4) {
    const int jj = j % hid;
    const float* v = (j < hid) ? avg : mx;
    float acc = 0.f;
    for (int k = lane; k < C; k += 64) acc += w1[(long)jj * C + k] * v[k];
    acc = wave_sum(acc);
    if (lane == 0) hsh[(j < hid ? 0 : 64) + jj] = fmaxf(CBAM ? acc : acc + b1[jj], 0.f);
  }
  __syncthreads();
  for (int i = tid; i < n; i += 256) {
    const int c = c0 + i;
    float za = 0.f, zm = 0.f;
    int j = 0;
    for (; j + 4 <= hid; j += 4) {  // 4 weight loads in flight, accumulated in j order
      float wv4[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) wv4[u] = w2[(long)c * hid + j + u];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        za += wv4[u] * hsh[j + u];
        if (CBAM) zm += wv4[u] * hsh[64 + j + u];
      }
    }
    for (; j < hid; ++j) {
      const float wcj = w2[(long)c * hid + j];
      za += wcj * hsh[j];
      if (CBAM) zm += wcj * hsh[64 + j];
    }
    out[i] = CBAM ? sigmoidf_(za + zm) : sigmoidf_(za + b2[c]);
  }
  __syncthreads();
}

// per-image gates into global memory. grid = images, dynamic LDS = (2*C + 128 + C) floats.
template <bool CBAM>
__global__ __launch_bounds__(256) void channel_gate_kernel(const float* __restrict__ psum,
                                                           const float* __restrict__ pmax, int parts, int C,
                                                           float inv_hw, const float* __restrict__ w1,
                                                           const float* __restrict__ b1, const float* __restrict__ w2,
                                                           const float* __restrict__ b2, int hid,
                                                           float* __restrict__ gate) {
  extern __shared__ float sh[];
  const int b = blockIdx.x;
  float* g = sh + 2 * C + 128;
  gate_mlp<CBAM>(psum, pmax, parts, C, inv_hw, w1, b1, w2, b2, hid, b, sh, sh + C, sh + 2 * C, 0, C, g);
  for (int c = threadIdx.x; c < C; c += 256) gate[(long)b * C + c] = g[c];
}

// ------------------------------------------------------------------------------------------------
// (3a) SE apply: y = x * gate[b][c]. Vector path: grid = (ceil(HW / 1024), ceil(C / 8), images), a lane scales
// 4 pixels in 8 consecutive channel planes - 8 independent vector loads in flight before the first store (the
// 4-deep per-plane version streamed at ~4 TB/s, this shape at ~6 like cbam_apply), issued before the fused gate MLP.
// Scalar path otherwise.
// FUSED: the workgroup computes the gates of its 8 channels itself from the plane partials (gate_mlp), so SE is
// one launch after its producer; dynamic LDS = (2*C + 136) floats.
// ------------------------------------------------------------------------------------------------
template <class T, bool FUSED>
__global__ __launch_bounds__(256) void plane_scale_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                          const float* __restrict__ gate, int C, long HW, int rev,
                                                          int se_pre,
                                                          const float* __restrict__ psum, int parts, float inv_hw,
                                                          const float* __restrict__ w1, const float* __restrict__ b1,
                                                          const float* __restrict__ w2, const float* __restrict__ b2,
                                                          int hid) {
  extern __shared__ float sh[];
  const int b = rev ? gridDim.z - 1 - blockIdx.z : blockIdx.z;
  const int c0 = (rev ? gridDim.y - 1 - blockIdx.y : blockIdx.y) * 8;
  const int n = (C - c0 < 8) ? C - c0 : 8;
  // vector path with 8 channels: the lane's 8 loads go out before the gate MLP (they do not depend on it), so its
  // latency chain overlaps them instead of preceding them
  const long p4 = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
  const bool pre = se_pre && (HW & 3) == 0 && n == 8 && p4 < HW;
  f32x4 v[8];
  if (pre) {
    const T* xb = x + ((long)b * C + c0) * HW + p4;
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = ld4(xb + (long)u * HW);
  }
  const float* gb;
  if (FUSED) {
    float* g = sh + 2 * C + 128;
    gate_mlp<false>(psum, nullptr, parts, C, inv_hw, w1, b1, w2, b2, hid, b, sh, nullptr, sh + 2 * C, c0, n, g);
    gb = g;
  } else {
    gb = gate + (long)b * C + c0;
  }
  if ((HW & 3) == 0) {
    const long p = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
    if (p >= HW) return;
    const T* xb = x + ((long)b * C + c0) * HW + p;
    T* yb = y + ((long)b * C + c0) * HW + p;
    if (n == 8) {
      if (!pre) {
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = ld4(xb + (long)u * HW);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) st4(yb + (long)u * HW, v[u] * gb[u]);
    } else {
      for (int u = 0; u < n; ++u) st4(yb + (long)u * HW, ld4(xb + (long)u * HW) * gb[u]);
    }
  } else {
    const long p = (long)blockIdx.x * 256 + threadIdx.x;
    if (p >= HW) return;
    for (int u = 0; u < n; ++u) {
      const long o = ((long)b * C + c0 + u) * HW + p;
      st1(y + o, ld1(x + o) * gb[u]);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// CBAM pass 2: per-pixel channel sum / max of o = ca[c] * x over channel group g -> mpart[b][g][0|1][HW].
// grid = (ceil(HW / (256*V)), G, images); V = 4 (vector pixels) when HW % 4 == 0.
// FUSED: the workgroup first computes the channel gate of its group from the plane partials (gate_mlp; blockIdx.x
// == 0 also stores it to ca for the apply pass), so channel gate + pixel statistics are one launch; dynamic LDS =
// (3*C + 128) floats.
// ------------------------------------------------------------------------------------------------
template <int V, class T, bool FUSED>
__global__ __launch_bounds__(256) void cbam_pixel_stats_kernel(const T* __restrict__ x, float* __restrict__ ca,
                                                               int C, int CG, long HW, float* __restrict__ mpart,
                                                               const float* __restrict__ psum,
                                                               const float* __restrict__ pmax, int parts,
                                                               float inv_hw, const float* __restrict__ w1,
                                                               const float* __restrict__ w2, int hid) {
  extern __shared__ float sh[];
  const int b = blockIdx.z, g = blockIdx.y, G = gridDim.y;
  const int c0 = g * CG;
  const int c1 = (c0 + CG < C) ? c0 + CG : C;
  const long p = ((long)blockIdx.x * 256 + threadIdx.x) * V;
  // the first 8 channels' loads go out before the gate MLP (they do not depend on it), so its latency chain
  // overlaps them instead of preceding them
  const bool pre = V == 4 && p < HW && c0 + 8 <= c1;
  f32x4 v0[8];
  if (pre) {
#pragma unroll
    for (int u = 0; u < 8; ++u) v0[u] = ld4(x + ((long)b * C + c0 + u) * HW + p);
  }
  const float* cab;
  if (FUSED) {
    float* gs = sh + 2 * C + 128;
    gate_mlp<true>(psum, pmax, parts, C, inv_hw, w1, nullptr, w2, nullptr, hid, b, sh, sh + C, sh + 2 * C, c0, c1 - c0,
                   gs);
    if (blockIdx.x == 0)
      for (int i = threadIdx.x; i < c1 - c0; i += 256) ca[(long)b * C + c0 + i] = gs[i];
    cab = gs - c0;
  } else {
    cab = ca + (long)b * C;
  }
  if (p >= HW) return;
  const T* xb = x + ((long)b * C) * HW + p;
  float* sp = mpart + ((long)(b * G + g) * 2) * HW + p;
  if (V == 4) {
    f32x4 s = {0.f, 0.f, 0.f, 0.f}, m = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    int c = c0;
    if (pre) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const f32x4 o = cab[c + u] * v0[u];
        s += o;
        m.x = fmaxf(m.x, o.x); m.y = fmaxf(m.y, o.y); m.z = fmaxf(m.z, o.z); m.w = fmaxf(m.w, o.w);
      }
      c += 8;
    }
    for (; c + 8 <= c1; c += 8) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = ld4(xb + (long)(c + u) * HW);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const f32x4 o = cab[c + u] * v[u];
        s += o;
        m.x = fmaxf(m.x, o.x); m.y = fmaxf(m.y, o.y); m.z = fmaxf(m.z, o.z); m.w = fmaxf(m.w, o.w);
      }
    }
    for (; c < c1; ++c) {
      const f32x4 o = cab[c] * ld4(xb + (long)c * HW);
      s += o;
      m.x = fmaxf(m.x, o.x); m.y = fmaxf(m.y, o.y); m.z = fmaxf(m.z, o.z); m.w = fmaxf(m.w, o.w);
    }
    *reinterpret_cast<f32x4*>(sp) = s;
    *reinterpret_cast<f32x4*>(sp + HW) = m;
  } else {
    float s = 0.f, m = -INFINITY;
    int c = c0;
    for (; c + 8 <= c1; c += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = ld1(xb + (long)(c + u) * HW);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float o = cab[c + u] * v[u];
        s += o;
        m = fmaxf(m, o);
      }
    }
    for (; c < c1; ++c) {
      const float o = cab[c] * ld1(xb + (long)c * HW);
      s += o;
      m = fmaxf(m, o);
    }
    sp[0] = s;
    sp[HW] = m;
  }
}

// mean / max over the channel groups of pixel (yy, xx), zero outside the image (conv2d's zero padding of the
// [mean; max] map, cbam_block.py:33-37)
__device__ __forceinline__ float2 cbam_map_at(const float* __restrict__ mp, int G, long HW, int H, int W, int yy,
                                              int xx, float invC) {
  float s = 0.f, m = 0.f;
  if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
    const float* q = mp + (long)yy * W + xx;
    m = -INFINITY;
    int g = 0;
    for (; g + 4 <= G; g += 4) {  // 8 independent loads in flight (the sums keep their g order)
      float a[4], c[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a[u] = q[(long)(2 * (g + u)) * HW];
        c[u] = q[(long)(2 * (g + u) + 1) * HW];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        s += a[u];
        m = fmaxf(m, c[u]);
      }
    }
    for (; g < G; ++g) {
      s += q[(long)(2 * g) * HW];
      m = fmaxf(m, q[(long)(2 * g + 1) * HW]);
    }
    s *= invC;
  }
  return make_float2(s, m);
}

// CBAM pass 2b (split path): sa = sigmoid(conv7x7([mean_c o ; max_c o]), zero pad 3, no bias) on 16-wide x 64-tall
// output tiles, the 22 x 70 halo of both maps (combined over the G channel groups) staged in LDS. Each thread
// computes 4 vertically adjacent outputs, so each staged value is read from LDS once per 4 outputs (140 reads for
// 392 FMAs; the weights are scalar loads; 16x16 tiles with one output per thread read 196 LDS values - weights
// included - per 98 FMAs, and needed two rounds of workgroups). Per output the products accumulate in the same (map, ky, kx) order as before.
// grid = (tiles_x, tiles_y, images).
constexpr int kSaTW = 16, kSaTH = 64;
__global__ __launch_bounds__(256) void cbam_sa_kernel(const float* __restrict__ mpart, int G, int C, int H, int W,
                                                      const float* __restrict__ wsa, float* __restrict__ sa) {
  constexpr int HX = kSaTW + 6, HY = kSaTH + 6, NPOS = HX * HY, PT = (NPOS + 255) / 256;
  __shared__ float mm[2][HY][HX + 1];
  const int b = blockIdx.z;
  const long HW = (long)H * W;
  const int tid = threadIdx.x;
  const int oy = blockIdx.y * kSaTH - 3, ox = blockIdx.x * kSaTW - 3;
  const float invC = 1.0f / (float)C;
  // the thread's halo positions: every partial-map load unconditional from a clamped position (loads under a
  // bounds branch were merged into phis that each waited for all loads in flight), all positions' loads of up to
  // 4 groups in flight together; out-of-image positions take the conv's zero padding afterwards. Sums keep their
  // g order.
  const float* mp = mpart + (long)b * G * 2 * HW;
  int q[PT];
  bool in[PT];
#pragma unroll
  for (int k = 0; k < PT; ++k) {
    const int i = min(tid + 256 * k, NPOS - 1), ty = i / HX, tx = i - (i / HX) * HX;
    const int yy = oy + ty, xx = ox + tx;
    in[k] = yy >= 0 && yy < H && xx >= 0 && xx < W;
    q[k] = min(max(yy, 0), H - 1) * W + min(max(xx, 0), W - 1);
  }
  float sm[PT], mx[PT];
#pragma unroll
  for (int k = 0; k < PT; ++k) {
    sm[k] = 0.f;
    mx[k] = -INFINITY;
  }
  for (int g0 = 0; g0 < G; g0 += 4) {
    float a[PT][4], c[PT][4];
#pragma unroll
    for (int k = 0; k < PT; ++k)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int gu = min(g0 + u, G - 1);
        a[k][u] = mp[(long)(2 * gu) * HW + q[k]];
        c[k][u] = mp[(long)(2 * gu + 1) * HW + q[k]];
      }
#pragma unroll
    for (int k = 0; k < PT; ++k)
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (g0 + u < G) {
          sm[k] += a[k][u];
          mx[k] = fmaxf(mx[k], c[k][u]);
        }
  }
#pragma unroll
  for (int k = 0; k < PT; ++k) {
    const int i = tid + 256 * k;
    if (i < NPOS) {
      const int ty = i / HX, tx = i - (i / HX) * HX;
      mm[0][ty][tx] = in[k] ? sm[k] * invC : 0.f;
      mm[1][ty][tx] = in[k] ? mx[k] : 0.f;
    }
  }
  __syncthreads();
  const int lx = tid & 15, ly = (tid >> 4) * 4;
  float z[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      float v[7];
#pragma unroll
      for (int kx = 0; kx < 7; ++kx) v[kx] = mm[ci][ly + r][lx + kx];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ky = r - j;
        if (ky >= 0 && ky < 7)
#pragma unroll
          for (int kx = 0; kx < 7; ++kx) z[j] += wsa[ci * 49 + ky * 7 + kx] * v[kx];  // uniform: scalar loads
      }
    }
  const int px = blockIdx.x * kSaTW + lx;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int py = blockIdx.y * kSaTH + ly + j;
    if (py < H && px < W) sa[(long)b * HW + (long)py * W + px] = sigmoidf_(z[j]);
  }
}

// CBAM pass 3 (split path): y = sa[p] * (ca[c] * x). grid = (ceil(HW / (256*V)), ceil(C / 8), images).
template <int V, class T>
__global__ __launch_bounds__(256) void cbam_apply_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                         const float* __restrict__ ca, const float* __restrict__ sa,
                                                         int C, long HW) {
  const int b = blockIdx.z;
  const long p = ((long)blockIdx.x * 256 + threadIdx.x) * V;
  if (p >= HW) return;
  const int c0 = blockIdx.y * 8;
  const int n = (C - c0 < 8) ? C - c0 : 8;
  const T* xb = x + ((long)b * C + c0) * HW + p;
  T* yb = y + ((long)b * C + c0) * HW + p;
  const float* cab = ca + (long)b * C + c0;
  if (V == 4) {
    const f32x4 s4 = *reinterpret_cast<const f32x4*>(sa + (long)b * HW + p);
    if (n == 8) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = ld4(xb + (long)u * HW);
#pragma unroll
      for (int u = 0; u < 8; ++u) st4(yb + (long)u * HW, s4 * (cab[u] * v[u]));
    } else {
      for (int u = 0; u < n; ++u) st4(yb + (long)u * HW, s4 * (cab[u] * ld4(xb + (long)u * HW)));
    }
  } else {
    const float s = sa[(long)b * HW + p];
    for (int u = 0; u < n; ++u) st1(yb + (long)u * HW, s * (cab[u] * ld1(xb + (long)u * HW)));
  }
}

template <class T>
__global__ __launch_bounds__(256) void ca_pool_kernel(const T* __restrict__ x, int H, int W, int RB,
                                                      float* __restrict__ yin) {
  extern __shared__ float band[];
  const long plane = blockIdx.x;
  const T* p = x + plane * (long)H * W;
  float* o = yin + plane * (long)(H + W);
  const int tid = threadIdx.x;
  float col[4] = {0.f, 0.f, 0.f, 0.f};
  const float invW = 1.0f / (float)W;
  for (int h0 = 0; h0 < H; h0 += RB) {
    const int rb = (H - h0 < RB) ? H - h0 : RB;
    const int n = rb * W;
    const T* src = p + (long)h0 * W;
    if ((W & 3) == 0) {
      for (int i = tid; i < (n >> 2); i += 256) reinterpret_cast<f32x4*>(band)[i] = ld4(src + 4 * i);
    } else {
      for (int i = tid; i < n; i += 256) band[i] = ld1(src + i);
    }
    __syncthreads();
    for (int r = tid >> 2; r < rb; r += 64) {
      float s = 0.f;
      for (int w = tid & 3; w < W; w += 4) s += band[r * W + w];
      s = quad_sum(s);
      if ((tid & 3) == 0) o[h0 + r] = s * invW;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int w = tid + 256 * u;
      if (w < W)
        for (int r = 0; r < rb; ++r) col[u] += band[r * W + w];
    }
    __syncthreads();
  }
  const float invH = 1.0f / (float)H;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int w = tid + 256 * u;
    if (w < W) o[H + w] = col[u] * invH;
  }
}

// CA pass 2: per position p of the concatenated (H+W) axis:
//   t[j]   = h_sigmoid(BN(sum_c W1[j][c] yin[c][p] + b1[j]))        (conv1 + bn1 + act; BN eval, eps given)
//   gate[c][p] = sigmoid(sum_j Wx[c][j] t[j] + bx[c]),  Wx = conv_h for p < H, conv_w otherwise.
// grid = (ceil((H+W)/16), images); the 16 positions of yin, W1 (row stride C+1) and conv_h/conv_w staged in LDS.
__global__ __launch_bounds__(256) void ca_gate_kernel(const float* __restrict__ yin, int C, int H, int W, int mip,
                                                      const float* __restrict__ w1, const float* __restrict__ b1,
                                                      const float* __restrict__ bn_w, const float* __restrict__ bn_b,
                                                      const float* __restrict__ bn_m, const float* __restrict__ bn_v,
                                                      float bn_eps, const float* __restrict__ wh,
                                                      const float* __restrict__ bh, const float* __restrict__ ww,
                                                      const float* __restrict__ bw, float* __restrict__ gate) {
  constexpr int P = 16;
  extern __shared__ float sh[];
  float* ys = sh;                              // [C][P]
  float* w1s = ys + C * P;                     // [mip][C+1]
  float* whs = w1s + mip * (C + 1);            // [C*mip]
  float* wws = whs + C * mip;                  // [C*mip]
  float* ts = wws + C * mip;                   // [P][mip+1]
  const int b = blockIdx.y;
  const int L = H + W;
  const int p0 = blockIdx.x * P;
  const int tid = threadIdx.x;
  const float* yb = yin + (long)b * C * L;
  // staging: every load unconditional from a clamped index, 8 in flight per thread before their LDS stores (a load
  // under a predicate merges into a phi whose copy waits for all loads in flight: each load was its own L2 / MALL
  // round trip)
  constexpr int U = 8;
  const int nys = C * P, nw = mip * C;
  for (int i0 = 0; i0 < nys; i0 += 256 * U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = min(i0 + tid + 256 * u, nys - 1), c = i / P, pp = i % P;
      v[u] = yb[(long)c * L + min(p0 + pp, L - 1)];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + tid + 256 * u;
      if (i < nys) ys[i] = (p0 + i % P < L) ? v[u] : 0.f;
    }
  }
  for (int i0 = 0; i0 < nw; i0 += 256 * U) {
    float v[U], a[U], c_[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = min(i0 + tid + 256 * u, nw - 1);
      v[u] = w1[i];
      a[u] = wh[i];
      c_[u] = ww[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + tid + 256 * u;
      if (i < nw) {
        w1s[(i / C) * (C + 1) + i % C] = v[u];
        whs[i] = a[u];
        wws[i] = c_[u];
      }
    }
  }
  __syncthreads();
  for (int o = tid; o < P * mip; o += 256) {
    const int pp = o / mip, j = o % mip;
    const float* wr = w1s + j * (C + 1);
    // four independent partial sums (one dependent chain of C FMAs through LDS reads was the kernel's critical path)
    float acc4[4] = {0.f, 0.f, 0.f, 0.f};
    int c = 0;
    for (; c + 4 <= C; c += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) acc4[u] = fmaf(wr[c + u], ys[(c + u) * P + pp], acc4[u]);
    }
    for (; c < C; ++c) acc4[0] = fmaf(wr[c], ys[c * P + pp], acc4[0]);
    const float acc = (acc4[0] + acc4[1]) + (acc4[2] + acc4[3]);
    float z = acc + b1[j];
    const float inv = 1.0f / sqrtf(bn_v[j] + bn_eps);
    z = (z - bn_m[j]) * inv * bn_w[j] + bn_b[j];
    z = fminf(fmaxf(z + 3.0f, 0.0f), 6.0f) / 6.0f;
    ts[pp * (mip + 1) + j] = z;
  }
  __syncthreads();
  float* gb = gate + (long)b * C * L;
  for (int o = tid; o < P * C; o += 256) {
    const int c = o / P, pp = o % P;
    const int p = p0 + pp;
    if (p >= L) continue;
    const float* wx = ((p < H) ? whs : wws) + c * mip;
    const float bx = (p < H) ? bh[c] : bw[c];
    const float* t = ts + pp * (mip + 1);
    float acc = 0.f;
    for (int j = 0; j < mip; ++j) acc += wx[j] * t[j];
    gb[(long)c * L + p] = sigmoidf_(acc + bx);
  }
}

static size_t ca_gate_lds_bytes(int C, int mip) {
  return sizeof(float) * ((size_t)C * 16 + (size_t)mip * (C + 1) + 2 * (size_t)C * mip + 16 * (size_t)(mip + 1));
}

// CA pass 3: y[b,c,h,w] = (x * a_w[b,c,w]) * a_h[b,c,h]; gate rows are [a_h (H) | a_w (W)].
// grid = (planes, ceil(HW / (256*V))); V = 4 when W % 4 == 0 (a vector never straddles two rows).
template <int V, class T>
__global__ __launch_bounds__(256) void ca_apply_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                       const float* __restrict__ gate, int H, int W) {
  const long plane = blockIdx.x;
  const long HW = (long)H * W;
  const long e = ((long)blockIdx.y * 256 + threadIdx.x) * V;
  if (e >= HW) return;
  const int h = (int)(e / W), w = (int)(e - (long)h * W);
  const float* g = gate + plane * (H + W);
  const float ah = g[h];
  if (V == 8 && sizeof(T) == 2) {  // bf16 storage: 16-byte accesses (8 elements of one row: W % 8 == 0)
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(x + plane * HW + e), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (f[j] * g[H + w + j]) * ah;
    *reinterpret_cast<uint4*>(y + plane * HW + e) = pack8(f);
  } else if (V == 4) {
    f32x4 v = ld4(x + plane * HW + e);
    v.x = (v.x * g[H + w]) * ah;
    v.y = (v.y * g[H + w + 1]) * ah;
    v.z = (v.z * g[H + w + 2]) * ah;
    v.w = (v.w * g[H + w + 3]) * ah;
    st4(y + plane * HW + e, v);
  } else {
    st1(y + plane * HW + e, (ld1(x + plane * HW + e) * g[H + w]) * ah);
  }
}

}  // namespace ys

using namespace ys;

// =================================================================================================
// C ABI
// =================================================================================================
YS_EXPORT size_t yolosod_se_workspace(int B, int C, int H, int W) {
  (void)H; (void)W;
  Sizer s;
  s.take<float>((size_t)B * C * part_plan((long)H * W).parts);  // partial sums
  s.take<float>((size_t)B * C);              // gates
  return s.off;
}

// plane segmentation of the per-plane statistics (parts per plane, elements per part) for an H*W plane, so a
// producer epilogue (yolosod_bias_act_stats) can emit the partials the *_forward_pre entry points consume
YS_EXPORT int yolosod_plane_parts(long HW, long* seg) {
  const PartPlan pp = part_plan(HW);
  if (seg) *seg = pp.seg;
  return pp.parts;
}

// y == nullptr: the gate only, into gate_out [B][C] (its consumer applies it: yolosod_conv3x3s2_silu)
template <class T>
static int se_forward_impl(const T* x, T* y, int B, int C, int H, int W, const float* fc1_w, const float* fc1_b,
                           const float* fc2_w, const float* fc2_b, int hidden, const float* psum_pre, void* workspace,
                           size_t workspace_bytes, void* stream, float* gate_out = nullptr) {
  YS_CHECK_ARG(x && (y || gate_out) && fc1_w && fc1_b && fc2_w && fc2_b, "se: null pointer");
  YS_CHECK_ARG(B >= 0 && C > 0 && C <= 16384 && H > 0 && W > 0, "se: bad shape");
  YS_CHECK_ARG(hidden > 0 && hidden <= 64, "se: hidden=%d unsupported (1..64)", hidden);
  if (B == 0) return 0;
  Carver cv(workspace, workspace_bytes);
  float* psum = cv.take<float>((size_t)B * C * part_plan((long)H * W).parts);
  float* gate = cv.take<float>((size_t)B * C);
  YS_CHECK_ARG(gate, "se: workspace too small (%zu)", workspace_bytes);
  hipStream_t st = (hipStream_t)stream;
  const long HW = (long)H * W;
  const PartPlan pp = part_plan(HW);
  const long xchunks = (HW % 4 == 0) ? (HW + 1023) / 1024 : (HW + 255) / 256;
  const size_t lds = sizeof(float) * (3 * (size_t)C + 128);
  const size_t lds_fused = sizeof(float) * (2 * (size_t)C + 136);
  // gate MLP fused into the apply pass for small planes; a separate gate launch for large ones, where the fused
  // form's per-workgroup MLP (12800 workgroups at 32x32x320x320) cost more than the launch: SE L1 0.158 -> 0.150 ms,
  // L23 0.038 fused vs 0.040 split (same box, profiles/r04_se/)
  constexpr long fused_max_hw = 65536;
  const bool fused = y && lds_fused <= 64 * 1024 && (HW < fused_max_hw || lds > 64 * 1024);
  YS_CHECK_ARG(lds <= 64 * 1024 || fused, "se: C=%d too large for the gate kernel", C);
  if (!y) gate = gate_out;
  // the fused apply issues its 8 loads per lane before the gate MLP (pre = 1)
  const float* ps = psum_pre ? psum_pre : psum;
  if (!psum_pre)
    hipLaunchKernelGGL((plane_part_stats_kernel<false, T>), dim3((unsigned)(B * C * pp.parts)), dim3(256), 0, st, x,
                       HW, pp.parts, pp.seg, psum, nullptr);
  const dim3 grid((unsigned)xchunks, (unsigned)((C + 7) / 8), (unsigned)B);
  if (fused) {
    hipLaunchKernelGGL((plane_scale_kernel<T, true>), grid, dim3(256), lds_fused, st, x, y, nullptr, C, HW,
                       mall_reverse(), 1, ps, pp.parts, 1.0f / (float)HW, fc1_w, fc1_b, fc2_w, fc2_b, hidden);
  } else {
    hipLaunchKernelGGL((channel_gate_kernel<false>), dim3(B), dim3(256), lds, st, ps, nullptr, pp.parts, C,
                       1.0f / (float)HW, fc1_w, fc1_b, fc2_w, fc2_b, hidden, gate);
    if (y)
      hipLaunchKernelGGL((plane_scale_kernel<T, false>), grid, dim3(256), 0, st, x, y, gate, C, HW, mall_reverse(), 0,
                         nullptr, 0, 0.f, nullptr, nullptr, nullptr, nullptr, 0);
  }
  YS_CHECK_LAUNCH("se");
  return 0;
}

YS_EXPORT int yolosod_se_forward(const float* x, float* y, int B, int C, int H, int W, const float* fc1_w,
                                 const float* fc1_b, const float* fc2_w, const float* fc2_b, int hidden,
                                 void* workspace, size_t workspace_bytes, void* stream) {
  return se_forward_impl(x, y, B, C, H, W, fc1_w, fc1_b, fc2_w, fc2_b, hidden, nullptr, workspace, workspace_bytes,
                         stream);
}

// As yolosod_se_forward, with x's per-plane partial sums already computed by its producer
// (psum[B*C*parts], yolosod_plane_parts segmentation; yolosod_bias_act_stats): no statistics pass over x.
YS_EXPORT int yolosod_se_forward_pre(const float* x, float* y, int B, int C, int H, int W, const float* fc1_w,
                                     const float* fc1_b, const float* fc2_w, const float* fc2_b, int hidden,
                                     const float* psum, void* workspace, size_t workspace_bytes, void* stream) {
  YS_CHECK_ARG(psum, "se_pre: null partials");
  return se_forward_impl(x, y, B, C, H, W, fc1_w, fc1_b, fc2_w, fc2_b, hidden, psum, workspace, workspace_bytes,
                         stream);
}

// bf16 storage variants (x, y: bf16 bit patterns; parameters and partials fp32)
// The SE gate only (sigmoid(fc2(relu(fc1(mean_hw(x))))), smallobj_modules.py:87-90) into gate [B][C], for a consumer
// that applies it itself (yolosod_conv3x3s2_silu); psum: x's per-plane partial sums from its producer, or NULL (a
// statistics pass over x).
YS_EXPORT int yolosod_se_gate(const float* x, int B, int C, int H, int W, const float* fc1_w, const float* fc1_b,
                              const float* fc2_w, const float* fc2_b, int hidden, const float* psum, float* gate,
                              void* workspace, size_t workspace_bytes, void* stream) {
  YS_CHECK_ARG(gate, "se_gate: null gate");
  return se_forward_impl<float>(x, nullptr, B, C, H, W, fc1_w, fc1_b, fc2_w, fc2_b, hidden, psum, workspace,
                                workspace_bytes, stream, gate);
}

YS_EXPORT int yolosod_se_forward_bf16(const bf16_t* x, bf16_t* y, int B, int C, int H, int W, const float* fc1_w,
                                      const float* fc1_b, const float* fc2_w, const float* fc2_b, int hidden,
                                      const float* psum, void* workspace, size_t workspace_bytes, void* stream) {
  return se_forward_impl(x, y, B, C, H, W, fc1_w, fc1_b, fc2_w, fc2_b, hidden, psum, workspace, workspace_bytes,
                         stream);
}

// channel groups of the CBAM per-pixel pass: 32 channels each (fixed, for batch-invariant sums); the partial
// maps cost 2/32 of x in extra traffic.
constexpr int kCbamGroup = 32;

YS_EXPORT size_t yolosod_cbam_workspace(int B, int C, int H, int W) {
  const long HW = (long)H * W;
  const int G = (C + kCbamGroup - 1) / kCbamGroup;
  Sizer s;
  s.take<float>((size_t)B * C * part_plan((long)H * W).parts);  // partial sums
  s.take<float>((size_t)B * C * part_plan((long)H * W).parts);  // partial maxes
  s.take<float>((size_t)B * C);              // ca
  s.take<float>((size_t)B * G * 2 * HW);     // per-group [sum;max] maps
  s.take<float>((size_t)B * HW);             // sa
  return s.off;
}

// y == nullptr: the gates only, into ca_out [B][C] and sa_out [B][H][W] (the consumer applies (x * ca) * sa)
template <class T>
static int cbam_forward_impl(const T* x, T* y, int B, int C, int H, int W, const float* fc0_w, const float* fc2_w,
                             int hidden, const float* sa_w, const float* psum_pre, const float* pmax_pre,
                             void* workspace, size_t workspace_bytes, void* stream, float* ca_out = nullptr,
                             float* sa_out = nullptr) {
  YS_CHECK_ARG(x && (y || (ca_out && sa_out)) && fc0_w && fc2_w && sa_w, "cbam: null pointer");
  YS_CHECK_ARG(B >= 0 && C > 0 && C <= 16384 && H > 0 && W > 0, "cbam: bad shape");
  YS_CHECK_ARG(hidden > 0 && hidden <= 64, "cbam: hidden=%d unsupported (1..64)", hidden);
  if (B == 0) return 0;
  const long HW = (long)H * W;
  const int V = (HW % 4 == 0) ? 4 : 1;
  const long pxb = (HW + 256 * V - 1) / (256 * V);
  const int G = (C + kCbamGroup - 1) / kCbamGroup;
  Carver cv(workspace, workspace_bytes);
  float* psum = cv.take<float>((size_t)B * C * part_plan((long)H * W).parts);
  float* pmax = cv.take<float>((size_t)B * C * part_plan((long)H * W).parts);
  float* ca = cv.take<float>((size_t)B * C);
  float* mpart = cv.take<float>((size_t)B * G * 2 * HW);
  float* sa = cv.take<float>((size_t)B * HW);
  YS_CHECK_ARG(sa, "cbam: workspace too small (%zu)", workspace_bytes);
  if (!y) {
    ca = ca_out;
    sa = sa_out;
  }
  hipStream_t st = (hipStream_t)stream;
  const PartPlan pp = part_plan(HW);
  const size_t lds = sizeof(float) * (3 * (size_t)C + 128);
  // fused launch: channel gate + pixel statistics
  const bool fused = V == 4 && lds <= 64 * 1024;
  YS_CHECK_ARG(lds <= 64 * 1024, "cbam: C=%d too large for the gate kernel", C);
  // (Folding the 7x7 spatial conv into the apply pass measured slower at both CBAM shapes - L4 0.134 -> 0.187 ms,
  // L18 0.043 -> 0.058 ms same-box: the per-run map staging and the conv, recomputed by every channel block, cost
  // more than the sa launch they replace - and so did a pixel-statistics pass with 8 channels per wave: level at
  // L18, 3 % slower at L4.)
  const float* ps = psum_pre ? psum_pre : psum;
  const float* pm = pmax_pre ? pmax_pre : pmax;
  if (!psum_pre)
    hipLaunchKernelGGL((plane_part_stats_kernel<true, T>), dim3((unsigned)(B * C * pp.parts)), dim3(256), 0, st, x, HW,
                       pp.parts, pp.seg, psum, pmax);
  dim3 gs((unsigned)pxb, G, B);
  if (fused) {  // channel gate computed inside the pixel-statistics workgroups
    hipLaunchKernelGGL((cbam_pixel_stats_kernel<4, T, true>), gs, dim3(256), lds, st, x, ca, C, kCbamGroup, HW, mpart,
                       ps, pm, pp.parts, 1.0f / (float)HW, fc0_w, fc2_w, hidden);
  } else {
    hipLaunchKernelGGL((channel_gate_kernel<true>), dim3(B), dim3(256), lds, st, ps, pm, pp.parts, C, 1.0f / (float)HW,
                       fc0_w, nullptr, fc2_w, nullptr, hidden, ca);
    if (V == 4)
      hipLaunchKernelGGL((cbam_pixel_stats_kernel<4, T, false>), gs, dim3(256), 0, st, x, ca, C, kCbamGroup, HW, mpart,
                         nullptr, nullptr, 0, 0.f, nullptr, nullptr, 0);
    else
      hipLaunchKernelGGL((cbam_pixel_stats_kernel<1, T, false>), gs, dim3(256), 0, st, x, ca, C, kCbamGroup, HW, mpart,
                         nullptr, nullptr, 0, 0.f, nullptr, nullptr, 0);
  }
  hipLaunchKernelGGL(cbam_sa_kernel, dim3((W + kSaTW - 1) / kSaTW, (H + kSaTH - 1) / kSaTH, B), dim3(256), 0, st, mpart, G, C, H, W, sa_w,
                     sa);
  if (y) {
    dim3 ga((unsigned)pxb, (C + 7) / 8, B);
    if (V == 4)
      hipLaunchKernelGGL((cbam_apply_kernel<4, T>), ga, dim3(256), 0, st, x, y, ca, sa, C, HW);
    else
      hipLaunchKernelGGL((cbam_apply_kernel<1, T>), ga, dim3(256), 0, st, x, y, ca, sa, C, HW);
  }
  YS_CHECK_LAUNCH("cbam");
  return 0;
}

YS_EXPORT int yolosod_cbam_forward(const float* x, float* y, int B, int C, int H, int W, const float* fc0_w,
                                   const float* fc2_w, int hidden, const float* sa_w, void* workspace,
                                   size_t workspace_bytes, void* stream) {
  return cbam_forward_impl(x, y, B, C, H, W, fc0_w, fc2_w, hidden, sa_w, (const float*)nullptr, nullptr, workspace,
                           workspace_bytes, stream);
}

// As yolosod_cbam_forward, with x's per-plane partial sums and maxes from its producer (yolosod_bias_act_stats).
YS_EXPORT int yolosod_cbam_forward_pre(const float* x, float* y, int B, int C, int H, int W, const float* fc0_w,
                                       const float* fc2_w, int hidden, const float* sa_w, const float* psum,
                                       const float* pmax, void* workspace, size_t workspace_bytes, void* stream) {
  YS_CHECK_ARG(psum && pmax, "cbam_pre: null partials");
  return cbam_forward_impl(x, y, B, C, H, W, fc0_w, fc2_w, hidden, sa_w, psum, pmax, workspace, workspace_bytes,
                           stream);
}

// The CBAM gates only (ca = sigmoid(fc(avg) + fc(max)), sa = sigmoid(conv7x7([mean_c; max_c](x * ca))),
// cbam_block.py:14-23,33-37) into ca [B][C] and sa [B][H][W], for a consumer that applies (x * ca) * sa itself
// (yolosod_conv3x3s2_silu); psum / pmax: x's per-plane partials from its producer, or both NULL.
YS_EXPORT int yolosod_cbam_gates(const float* x, int B, int C, int H, int W, const float* fc0_w, const float* fc2_w,
                                 int hidden, const float* sa_w, const float* psum, const float* pmax, float* ca,
                                 float* sa, void* workspace, size_t workspace_bytes, void* stream) {
  YS_CHECK_ARG((psum == nullptr) == (pmax == nullptr), "cbam_gates: give both partials or neither");
  YS_CHECK_ARG(ca && sa, "cbam_gates: null output");
  return cbam_forward_impl<float>(x, nullptr, B, C, H, W, fc0_w, fc2_w, hidden, sa_w, psum, pmax, workspace,
                                  workspace_bytes, stream, ca, sa);
}

// bf16 storage variant; psum / pmax may both be NULL (statistics pass over x) or both given (from the producer)
YS_EXPORT int yolosod_cbam_forward_bf16(const bf16_t* x, bf16_t* y, int B, int C, int H, int W, const float* fc0_w,
                                        const float* fc2_w, int hidden, const float* sa_w, const float* psum,
                                        const float* pmax, void* workspace, size_t workspace_bytes, void* stream) {
  YS_CHECK_ARG((psum == nullptr) == (pmax == nullptr), "cbam_bf16: give both partials or neither");
  return cbam_forward_impl(x, y, B, C, H, W, fc0_w, fc2_w, hidden, sa_w, psum, pmax, workspace, workspace_bytes,
                           stream);
}

YS_EXPORT size_t yolosod_ca_workspace(int B, int C, int H, int W) {
  Sizer s;
  s.take<float>((size_t)B * C * (H + W));  // pooled
  s.take<float>((size_t)B * C * (H + W));  // gates
  return s.off;
}

template <class T>
static int ca_forward_impl(const T* x, T* y, int B, int C, int H, int W, const float* conv1_w, const float* conv1_b,
                           int mip, const float* bn_w, const float* bn_b, const float* bn_mean, const float* bn_var,
                           float bn_eps, const float* convh_w, const float* convh_b, const float* convw_w,
                           const float* convw_b, const float* yin_pre, void* workspace, size_t workspace_bytes,
                           void* stream) {
  YS_CHECK_ARG(x && y && conv1_w && conv1_b && bn_w && bn_b && bn_mean && bn_var && convh_w && convh_b && convw_w &&
                   convw_b,
               "ca: null pointer");
  YS_CHECK_ARG(B >= 0 && C > 0 && H > 0 && W > 0 && W <= 1024, "ca: bad shape (W <= 1024 supported)");
  YS_CHECK_ARG(mip > 0 && mip <= 64, "ca: mip=%d unsupported (1..64)", mip);
  const size_t gate_lds = ca_gate_lds_bytes(C, mip);
  YS_CHECK_ARG(gate_lds <= 64 * 1024, "ca: C=%d mip=%d exceed the gate kernel's LDS budget", C, mip);
  if (B == 0) return 0;
  Carver cv(workspace, workspace_bytes);
  float* yin = cv.take<float>((size_t)B * C * (H + W));
  float* gate = cv.take<float>((size_t)B * C * (H + W));
  YS_CHECK_ARG(gate, "ca: workspace too small (%zu)", workspace_bytes);
  hipStream_t st = (hipStream_t)stream;
  const long HW = (long)H * W;
  int RB = 8192 / W;
  if (RB < 1) RB = 1;
  if (RB > H) RB = H;
  const size_t pool_lds = sizeof(float) * (size_t)RB * W;
  const int V = (W % 4 == 0) ? 4 : 1;
  // bf16: 8 elements (16 bytes) per thread in the apply pass when rows allow it (4 elements = 8-byte accesses ran at
  // ~4 TB/s at the m640 shape)
  const int VA = (sizeof(T) == 2 && W % 8 == 0) ? 8 : V;
  const unsigned apply_y = (unsigned)((HW + 256 * VA - 1) / (256 * VA));
  // (An apply pass with one workgroup per plane ran faster alone - 0.079 -> 0.057 ms - but 2x slower in the model
  // beside the Detect towers' side-stream convs: its 4096 long-lived workgroups lost the CUs; profiles/r04_channel_ab/)
  if (!yin_pre)
    hipLaunchKernelGGL((ca_pool_kernel<T>), dim3(B * C), dim3(256), pool_lds, st, x, H, W, RB, yin);
  hipLaunchKernelGGL(ca_gate_kernel, dim3((H + W + 15) / 16, B), dim3(256), gate_lds, st, yin_pre ? yin_pre : yin, C,
                     H, W, mip, conv1_w, conv1_b, bn_w, bn_b, bn_mean, bn_var, bn_eps, convh_w, convh_b, convw_w,
                     convw_b, gate);
  if (VA == 8)
    hipLaunchKernelGGL((ca_apply_kernel<8, T>), dim3(B * C, apply_y), dim3(256), 0, st, x, y, gate, H, W);
  else if (V == 4)
    hipLaunchKernelGGL((ca_apply_kernel<4, T>), dim3(B * C, apply_y), dim3(256), 0, st, x, y, gate, H, W);
  else
    hipLaunchKernelGGL((ca_apply_kernel<1, T>), dim3(B * C, apply_y), dim3(256), 0, st, x, y, gate, H, W);
  YS_CHECK_LAUNCH("ca");
  return 0;
}

YS_EXPORT int yolosod_ca_forward(const float* x, float* y, int B, int C, int H, int W, const float* conv1_w,
                                 const float* conv1_b, int mip, const float* bn_w, const float* bn_b,
                                 const float* bn_mean, const float* bn_var, float bn_eps, const float* convh_w,
                                 const float* convh_b, const float* convw_w, const float* convw_b, void* workspace,
                                 size_t workspace_bytes, void* stream) {
  return ca_forward_impl(x, y, B, C, H, W, conv1_w, conv1_b, mip, bn_w, bn_b, bn_mean, bn_var, bn_eps, convh_w,
                         convh_b, convw_w, convw_b, (const float*)nullptr, workspace, workspace_bytes, stream);
}

// CA_Block with the pooled row / column means already computed by x's producer (yolosod_bias_act_capool):
// gate + apply only.
YS_EXPORT int yolosod_ca_forward_pre(const float* x, float* y, int B, int C, int H, int W, const float* conv1_w,
                                     const float* conv1_b, int mip, const float* bn_w, const float* bn_b,
                                     const float* bn_mean, const float* bn_var, float bn_eps, const float* convh_w,
                                     const float* convh_b, const float* convw_w, const float* convw_b,
                                     const float* yin, void* workspace, size_t workspace_bytes, void* stream) {
  YS_CHECK_ARG(yin, "ca_pre: null pooled means");
  return ca_forward_impl(x, y, B, C, H, W, conv1_w, conv1_b, mip, bn_w, bn_b, bn_mean, bn_var, bn_eps, convh_w,
                         convh_b, convw_w, convw_b, yin, workspace, workspace_bytes, stream);
}

// bf16 storage variant; yin may be NULL (pooling pass over x) or the producer's pooled means
YS_EXPORT int yolosod_ca_forward_bf16(const bf16_t* x, bf16_t* y, int B, int C, int H, int W, const float* conv1_w,
                                      const float* conv1_b, int mip, const float* bn_w, const float* bn_b,
                                      const float* bn_mean, const float* bn_var, float bn_eps, const float* convh_w,
                                      const float* convh_b, const float* convw_w, const float* convw_b,
                                      const float* yin, void* workspace, size_t workspace_bytes, void* stream) {
  return ca_forward_impl(x, y, B, C, H, W, conv1_w, conv1_b, mip, bn_w, bn_b, bn_mean, bn_var, bn_eps, convh_w,
                         convh_b, convw_w, convw_b, yin, workspace, workspace_bytes, stream);
}
