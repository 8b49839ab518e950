// Detect-head post-processing on gfx950: DFL box decode + class sigmoid (standalone, or fused with the last 1x1
// convs of the head towers).
//
// Compile with -ffp-contract=off: the decode arithmetic (dist2bbox, xywh<->xyxy) and the IoU test must round
// exactly like the reference's fp32 CPU code so that kept-box indices after NMS are bit-exact.
//
// Reference semantics:
//   Detect._inference          ultralytics/nn/modules/head.py:100-131 (DFL block.py:79-82, make_anchors / dist2bbox
//                              utils/tal.py:333-357)
//   non_max_suppression        ultralytics/utils/ops.py:167-316 (xywh2xyxy :416-434) with torchvision==0.20.1
//                              ops.nms (CPU kernel: stable descending score sort, strict IoU > thr, area w/o +1).
//
// Class-wise NMS lives in nms.hip.
#include "common.h"
#include <math.h>
#include <stdlib.h>

namespace ys {

struct DecodeArgs {
  const float* maps[4];
  int hw[4];
  int w[4];
  int a_off[5];
  float stride[4];
  int nl, nc, reg_max, A;
  float* y;
};

__global__ __launch_bounds__(256) void detect_decode_kernel(DecodeArgs d) {
  const int b = blockIdx.y;
  const int a = blockIdx.x * 256 + threadIdx.x;
  if (a >= d.A) return;
  int l = 0;
#pragma unroll
  for (int i = 1; i < 4; ++i)
    if (i < d.nl && a >= d.a_off[i]) l = i;
  const int p = a - d.a_off[l];
  const int HW = d.hw[l];
  const int no = d.nc + 64;
  const float* m = d.maps[l] + (long)b * no * HW + p;
  const int iy = p / d.w[l], ix = p - (p / d.w[l]) * d.w[l];
  const float ax = (float)ix + 0.5f, ay = (float)iy + 0.5f;
  constexpr int RM = 16;  // Detect.reg_max (head.py:40)
  float dist[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    float v[RM];
    float mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < RM; ++k) {
      v[k] = m[(long)(s * RM + k) * HW];
      mx = fmaxf(mx, v[k]);
    }
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < RM; ++k) {
      v[k] = expf(v[k] - mx);
      sum += v[k];
    }
    const float inv = 1.0f / sum;
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < RM; ++k) acc += (float)k * (v[k] * inv);
    dist[s] = acc;
  }
  const float x1 = ax - dist[0], y1 = ay - dist[1];
  const float x2 = ax + dist[2], y2 = ay + dist[3];
  const float st = d.stride[l];
  float* yb = d.y + (long)b * (4 + d.nc) * d.A + a;
  yb[0] = ((x1 + x2) / 2.0f) * st;
  yb[(long)d.A] = ((y1 + y2) / 2.0f) * st;
  yb[2L * d.A] = (x2 - x1) * st;
  yb[3L * d.A] = (y2 - y1) * st;
  for (int c = 0; c < d.nc; ++c) yb[(long)(4 + c) * d.A] = sigmoidf_(m[(long)(64 + c) * HW]);
}

// ------------------------------------------------------------------------------------------------
// Fused head tail + decode: the last 1x1 convs of both towers (cv2[i][-1]: c2 -> 64 box
// logits, cv3[i][-1]: c3 -> nc class logits, head.py:45-48,70) run on MFMA straight into the DFL / dist2bbox /
// sigmoid decode, so the [B, 64+nc, H, W] raw maps never exist in HBM (detect_head_x2_kernel: fp16 two-term splits,
// the default; detect_head_lds_kernel: exact fp32 MFMA, the split-range fallback).
//   A = conv weights [out][k], B = tower features [k][pixel] (NCHW, loaded straight from HBM), D[out][pixel]:
//   lane (g = lane>>4, j = lane&15) holds outputs 4g..4g+3 of pixel j.
//   Box tile s (16 rows) is exactly side s's 16 DFL bins, so the softmax max / sum / expectation are 4 local
//   values plus two permlane swaps (xor16, xor32). Class tile: rows 0..15 (nc <= 16).
// Each wave owns NTS consecutive 16-pixel groups of one level of one image.
// ------------------------------------------------------------------------------------------------
struct HeadArgs {
  const void* fb[4];   // box tower features  [B][C2][HW] (fp32 or bf16, the kernel's FT)
  const void* fc[4];   // class tower features [B][C3][HW]
  const float* wb[4];  // [64][C2]
  const float* bb[4];  // [64]
  const float* wc[4];  // [nc][C3]
  const float* bc[4];  // [nc]
  int hw[4], w[4], a_off[4], blk_off[5];
  float stride[4];
  int nl, nc, A;
  float* y;
  unsigned* range_flag;  // split-range guard of the x2 kernel (common.h range_report)
};

// The head tail + decode on exact fp32 MFMA (the split-range fallback), the conv weights in LDS (A fragments are ds_read_b128 of 4
// tiles' rows at once from a [q][g][j][t] image, conflict-free for the b128 lane groups) - the ~100 VGPRs that
// held them now double-buffer the next 16-pixel group's feature loads, so the HBM latency of a group overlaps the
// MFMAs and DFL of the previous one, at 3 waves per SIMD.
template <int C2, int C3, int NTS, class FT = float>
__global__ __launch_bounds__(256, C3 > 64 ? 2 : 3) void detect_head_lds_kernel(HeadArgs d) {
  __shared__ __attribute__((aligned(16))) float wl[C2 * 64 + C3 * 16];
  float* wlb = wl;            // [C2/4 q][4 g][16 j][4 t] = W_box[16t + j][4q + g]
  float* wlc = wl + C2 * 64;  // [C3/16 qq][4 g][16 j][4 u] = W_cls[j][4(4qq + u) + g] (0 for j >= nc)
  const int b = blockIdx.y;
  int l = 0;
#pragma unroll
  for (int i = 1; i < 4; ++i)
    if (i < d.nl && (int)blockIdx.x >= d.blk_off[i]) l = i;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int g = lane >> 4, j = lane & 15;
  const int nc = d.nc;
  {
    const float* wb = d.wb[l];
    const float* wc = d.wc[l];
    // every load first, then the LDS stores (a load-store loop waits for each load in turn)
    static_assert((C2 * 64) % 256 == 0 && (C3 * 16) % 256 == 0, "weight image sizes");
    constexpr int NB = C2 * 64 / 256, NCL = C3 * 16 / 256;
    float vb[NB], vc[NCL];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int e = tid + 256 * i;
      const int t = e & 3, jj = (e >> 2) & 15, gg = (e >> 6) & 3, q = e >> 8;
      vb[i] = wb[(16 * t + jj) * C2 + 4 * q + gg];
    }
#pragma unroll
    for (int i = 0; i < NCL; ++i) {
      const int e = tid + 256 * i;
      const int u = e & 3, jj = (e >> 2) & 15, gg = (e >> 6) & 3, qq = e >> 8;
      vc[i] = (jj < nc) ? wc[(jj < nc ? jj : 0) * C3 + 4 * (4 * qq + u) + gg] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) wlb[tid + 256 * i] = vb[i];
#pragma unroll
    for (int i = 0; i < NCL; ++i) wlc[tid + 256 * i] = vc[i];
  }
  __syncthreads();
  const int HW = d.hw[l];
  const int px0 = (((int)blockIdx.x - d.blk_off[l]) * 4 + wv) * (NTS * 16);
  if (px0 >= HW) return;  // whole wave; no barrier below
  float bbr[4][4], bcr[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) bbr[t][r] = d.bb[l][16 * t + 4 * g + r];
#pragma unroll
  for (int r = 0; r < 4; ++r) bcr[r] = (4 * g + r < nc) ? d.bc[l][4 * g + r] : 0.f;
  const FT* fbb = static_cast<const FT*>(d.fb[l]) + (long)b * C2 * HW;
  const FT* fcb = static_cast<const FT*>(d.fc[l]) + (long)b * C3 * HW;
  const int W = d.w[l];
  const float st = d.stride[l];
  float* yb = d.y + (long)b * (4 + nc) * d.A + d.a_off[l];
  const float4* wb4 = reinterpret_cast<const float4*>(wlb) + g * 16 + j;
  const float4* wc4 = reinterpret_cast<const float4*>(wlc) + g * 16 + j;

  // feature loads are buffer loads on per-image descriptors: the lane's voffset is (channel g, pixel p), the
  // channel step 4q goes into the scalar soffset (no per-load 64-bit addresses to keep live), and pixels past the
  // level's end get an out-of-range voffset, which the hardware returns as 0
  auto rsrc = [&](const FT* base, int bytes) {
    const unsigned long long a = (unsigned long long)base;
    return __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(a >> 32)) << 32) |
                (unsigned)__builtin_amdgcn_readfirstlane((unsigned)a)),
        (short)0, __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
  };
  constexpr int ES = (int)sizeof(FT);
  const __amdgpu_buffer_rsrc_t rb = rsrc(fbb, C2 * HW * ES), rc = rsrc(fcb, C3 * HW * ES);
  // one feature element: fp32 as is, bf16 widened (exact)
  auto ldf = [&](__amdgpu_buffer_rsrc_t r, unsigned vo, int so) -> float {
    if constexpr (sizeof(FT) == 2)
      return __uint_as_float((unsigned)__builtin_amdgcn_raw_buffer_load_b16(r, vo, so, 0) << 16);
    else
      return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0));
  };
  float xb[2][C2 / 4], xc[2][C3 / 4];
  auto load_group = [&](int ts, float (&fb)[C2 / 4], float (&fcv)[C3 / 4]) {
    const int p = px0 + ts * 16 + j;
    const unsigned vo = (p < HW) ? (unsigned)((g * HW + p) * ES) : 0x80000000u;
#pragma unroll
    for (int q = 0; q < C2 / 4; ++q) fb[q] = ldf(rb, vo, q * 4 * ES * HW);
#pragma unroll
    for (int q = 0; q < C3 / 4; ++q) fcv[q] = ldf(rc, vo, q * 4 * ES * HW);
  };
  auto compute_group = [&](int ts, const float (&cb)[C2 / 4], const float (&cc)[C3 / 4]) {
    const int p0 = px0 + ts * 16;
    if (p0 >= HW) return;  // wave-uniform
    const int p = p0 + j;
    const bool ok = p < HW;
    f32x4 acc[5];
#pragma unroll
    for (int t = 0; t < 5; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < C2 / 4; ++q) {
      const float4 w4 = wb4[q * 64];
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(w4.x, cb[q], acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w4.y, cb[q], acc[1], 0, 0, 0);
      acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(w4.z, cb[q], acc[2], 0, 0, 0);
      acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(w4.w, cb[q], acc[3], 0, 0, 0);
    }
#pragma unroll
    for (int qq = 0; qq < C3 / 16; ++qq) {
      const float4 c4 = wc4[qq * 64];
      acc[4] = __builtin_amdgcn_mfma_f32_16x16x4f32(c4.x, cc[4 * qq], acc[4], 0, 0, 0);
      acc[4] = __builtin_amdgcn_mfma_f32_16x16x4f32(c4.y, cc[4 * qq + 1], acc[4], 0, 0, 0);
      acc[4] = __builtin_amdgcn_mfma_f32_16x16x4f32(c4.z, cc[4 * qq + 2], acc[4], 0, 0, 0);
      acc[4] = __builtin_amdgcn_mfma_f32_16x16x4f32(c4.w, cc[4 * qq + 3], acc[4], 0, 0, 0);
    }
    // DFL (block.py:79-82)
    float dist[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[s][r] + bbr[s][r];
      float mx = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
      mx = xor32_max(xor16_max(mx));
      float sum = 0.f, e = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = __expf(v[r] - mx);
        sum += v[r];
        e += (float)(4 * g + r) * v[r];
      }
      sum = xor32_sum(xor16_sum(sum));
      e = xor32_sum(xor16_sum(e));
      dist[s] = e * __builtin_amdgcn_rcpf(sum);
    }
    if (!ok) return;
    const int iy = p / W, ix = p - iy * W;
    const float ax = (float)ix + 0.5f, ay = (float)iy + 0.5f;
    const float x1 = ax - dist[0], y1 = ay - dist[1];
    const float x2 = ax + dist[2], y2 = ay + dist[3];
    const float out = g == 0 ? ((x1 + x2) / 2.0f) * st
                    : g == 1 ? ((y1 + y2) / 2.0f) * st
                    : g == 2 ? (x2 - x1) * st
                             : (y2 - y1) * st;
    yb[(long)g * d.A + p] = out;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = 4 * g + r;
      if (c < nc) yb[(long)(4 + c) * d.A + p] = sigmoidf_(acc[4][r] + bcr[r]);
    }
  };
  // ping-pong over group pairs (rolled: an unrolled group loop lets the scheduler hoist several groups' loads)
  static_assert(NTS % 2 == 0, "group pairs");
  load_group(0, xb[0], xc[0]);
#pragma unroll 1
  for (int ts = 0; ts < NTS; ts += 2) {
    if (px0 + (ts + 1) * 16 < HW) load_group(ts + 1, xb[1], xc[1]);
    compute_group(ts, xb[0], xc[0]);
    if (ts + 2 < NTS && px0 + (ts + 2) * 16 < HW) load_group(ts + 2, xb[0], xc[0]);
    compute_group(ts + 1, xb[1], xc[1]);
  }
}

// The same head tail + decode with the 1x1 convs as fp16 two-term splits on the fp16 matrix cores (common.h:
// three exact products per fp32 product, fp32 accumulation): 30 v_mfma_f32_16x16x32_f16 (16 cycles, beside the other
// waves' VALU) instead of 80 v_mfma_f32_16x16x4_f32 (32 cycles, which block the SIMD's VALU) per 16-pixel group, so
// the DFL / decode VALU work is no longer serialised behind the matrix work. Weights: LDS planes [t][s][g][row][i]
// of 64 W (exact scaling; rows of the box conv 16t + row, channel g + 32s + 4i - the k slots of the features a lane
// loads), split once per workgroup; the features are split in registers per group.
template <int C2, int C3, int NTS, class FT = float>
__global__ __launch_bounds__(256, C3 > 64 ? 2 : 3) void detect_head_x2_kernel(HeadArgs d) {
  static_assert(C2 == 64 && C3 % 32 == 0, "k steps of 32 channels");
  constexpr int NBW = C2 * 64, NCW = C3 * 16;  // image elements (box: 4 t x 2 s x 4 g x 16 rows x 8; cls: C3/32 s x ...)
  __shared__ __attribute__((aligned(16))) h16_t wl[2][NBW + NCW];
  constexpr float WS = 64.0f;
  const int b = blockIdx.y;
  int l = 0;
#pragma unroll
  for (int i = 1; i < 4; ++i)
    if (i < d.nl && (int)blockIdx.x >= d.blk_off[i]) l = i;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int g = lane >> 4, j = lane & 15;
  const int nc = d.nc;
  float rng = 0.f;  // largest magnitude split (64 W, features): split-range guard
  {
    const float* wb = d.wb[l];
    const float* wc = d.wc[l];
    static_assert(NBW % 512 == 0 && NCW % 512 == 0, "weight image sizes");
    constexpr int NB = NBW / 512, NCL = NCW / 512;  // pairs per thread
    f32x2 vb[NB], vc[NCL];
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int e = 2 * (tid + 256 * u);  // element pair (i, i + 1)
      const int i = e & 7, row = (e >> 3) & 15, gg = (e >> 7) & 3, s = (e >> 9) & 1, t = e >> 10;
      const float* src = wb + (16 * t + row) * C2 + gg + 32 * s + 4 * i;
      vb[u] = f32x2{src[0], src[4]} * WS;
    }
#pragma unroll
    for (int u = 0; u < NCL; ++u) {
      const int e = 2 * (tid + 256 * u);
      const int i = e & 7, row = (e >> 3) & 15, gg = (e >> 7) & 3, s = e >> 9;
      const float* src = wc + (row < nc ? row : 0) * C3 + gg + 32 * s + 4 * i;
      vc[u] = row < nc ? f32x2{src[0], src[4]} * WS : f32x2{0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      uint32_t h, lo;
      split2(vb[u], h, lo);
      rng = range_acc2(rng, vb[u]);
      reinterpret_cast<uint32_t*>(wl[0])[tid + 256 * u] = h;
      reinterpret_cast<uint32_t*>(wl[1])[tid + 256 * u] = lo;
    }
#pragma unroll
    for (int u = 0; u < NCL; ++u) {
      uint32_t h, lo;
      split2(vc[u], h, lo);
      rng = range_acc2(rng, vc[u]);
      reinterpret_cast<uint32_t*>(wl[0] + NBW)[tid + 256 * u] = h;
      reinterpret_cast<uint32_t*>(wl[1] + NBW)[tid + 256 * u] = lo;
    }
  }
  __syncthreads();
  const int HW = d.hw[l];
  const int px0 = (((int)blockIdx.x - d.blk_off[l]) * 4 + wv) * (NTS * 16);
  if (px0 >= HW) return;  // whole wave; no barrier below
  float bbr[4][4], bcr[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) bbr[t][r] = d.bb[l][16 * t + 4 * g + r];
#pragma unroll
  for (int r = 0; r < 4; ++r) bcr[r] = (4 * g + r < nc) ? d.bc[l][4 * g + r] : 0.f;
  const FT* fbb = static_cast<const FT*>(d.fb[l]) + (long)b * C2 * HW;
  const FT* fcb = static_cast<const FT*>(d.fc[l]) + (long)b * C3 * HW;
  const int W = d.w[l];
  const float st = d.stride[l];
  float* yb = d.y + (long)b * (4 + nc) * d.A + d.a_off[l];
  // A-operand rows of this lane: (t, s) block base + (g * 16 + j) * 8 halves
  const h16_t* wbh = wl[0] + (g * 16 + j) * 8;
  const h16_t* wbl = wl[1] + (g * 16 + j) * 8;

  auto rsrc = [&](const FT* base, int bytes) {
    const unsigned long long a = (unsigned long long)base;
    return __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(a >> 32)) << 32) |
                (unsigned)__builtin_amdgcn_readfirstlane((unsigned)a)),
        (short)0, __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
  };
  constexpr int ES = (int)sizeof(FT);
  const __amdgpu_buffer_rsrc_t rb = rsrc(fbb, C2 * HW * ES), rc = rsrc(fcb, C3 * HW * ES);
  auto ldf = [&](__amdgpu_buffer_rsrc_t r, unsigned vo, int so) -> float {
    if constexpr (sizeof(FT) == 2)
      return __uint_as_float((unsigned)__builtin_amdgcn_raw_buffer_load_b16(r, vo, so, 0) << 16);
    else
      return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0));
  };
  // lane (g, j) loads channels g + 4q of pixel j: q = 8s + i is k slot i of lane group g in k step s
  float xb[2][C2 / 4], xc[2][C3 / 4];
  auto load_group = [&](int ts, float (&fb)[C2 / 4], float (&fcv)[C3 / 4]) {
    const int p = px0 + ts * 16 + j;
    const unsigned vo = (p < HW) ? (unsigned)((g * HW + p) * ES) : 0x80000000u;
#pragma unroll
    for (int q = 0; q < C2 / 4; ++q) fb[q] = ldf(rb, vo, q * 4 * ES * HW);
#pragma unroll
    for (int q = 0; q < C3 / 4; ++q) fcv[q] = ldf(rc, vo, q * 4 * ES * HW);
  };
  auto compute_group = [&](int ts, const float (&cb)[C2 / 4], const float (&cc)[C3 / 4]) {
    const int p0 = px0 + ts * 16;
    if (p0 >= HW) return;  // wave-uniform
    const int p = p0 + j;
    const bool ok = p < HW;
    f32x4 acc[5];
#pragma unroll
    for (int t = 0; t < 5; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < C2 / 32; ++s) {
      f16x8_t fh, fl;
      const f32x4 va{cb[8 * s], cb[8 * s + 1], cb[8 * s + 2], cb[8 * s + 3]};
      const f32x4 vb2{cb[8 * s + 4], cb[8 * s + 5], cb[8 * s + 6], cb[8 * s + 7]};
      split8x(va, vb2, fh, fl);  // loaded features: the 3-VALU split (common.h split2x)
      rng = range_acc(range_acc(rng, va), vb2);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int o = (t * 2 + s) * 512;
        acc[t] = mfma_f16x3(*reinterpret_cast<const f16x8_t*>(wbh + o), *reinterpret_cast<const f16x8_t*>(wbl + o),
                            fh, fl, acc[t]);
      }
    }
#pragma unroll
    for (int s = 0; s < C3 / 32; ++s) {
      f16x8_t fh, fl;
      const f32x4 va{cc[8 * s], cc[8 * s + 1], cc[8 * s + 2], cc[8 * s + 3]};
      const f32x4 vb2{cc[8 * s + 4], cc[8 * s + 5], cc[8 * s + 6], cc[8 * s + 7]};
      split8x(va, vb2, fh, fl);  // loaded features: the 3-VALU split (common.h split2x)
      rng = range_acc(range_acc(rng, va), vb2);
      const int o = NBW + s * 512;
      acc[4] = mfma_f16x3(*reinterpret_cast<const f16x8_t*>(wbh + o), *reinterpret_cast<const f16x8_t*>(wbl + o), fh,
                          fl, acc[4]);
    }
    // DFL (block.py:79-82)
    float dist[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[s][r] * (1.0f / WS) + bbr[s][r];
      float mx = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
      mx = xor32_max(xor16_max(mx));
      float sum = 0.f, e = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = __expf(v[r] - mx);
        sum += v[r];
        e += (float)(4 * g + r) * v[r];
      }
      sum = xor32_sum(xor16_sum(sum));
      e = xor32_sum(xor16_sum(e));
      dist[s] = e * __builtin_amdgcn_rcpf(sum);
    }
    if (!ok) return;
    const int iy = p / W, ix = p - iy * W;
    const float ax = (float)ix + 0.5f, ay = (float)iy + 0.5f;
    const float x1 = ax - dist[0], y1 = ay - dist[1];
    const float x2 = ax + dist[2], y2 = ay + dist[3];
    const float out = g == 0 ? ((x1 + x2) / 2.0f) * st
                    : g == 1 ? ((y1 + y2) / 2.0f) * st
                    : g == 2 ? (x2 - x1) * st
                             : (y2 - y1) * st;
    yb[(long)g * d.A + p] = out;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = 4 * g + r;
      // class score: sigmoid on the hardware exp2 / rcp (1-2 ulp; the libm expf + IEEE division were ~15 % of the
      // kernel's VALU, and the split products already carry a few ulp)
      if (c < nc) yb[(long)(4 + c) * d.A + p] = sigmoid_fast_(acc[4][r] * (1.0f / WS) + bcr[r]);
    }
  };
  static_assert(NTS % 2 == 0, "group pairs");
  // Both 16-pixel groups of a 32-pixel run - the two 64-byte halves of each channel row's 128-byte line - are loaded
  // together, then computed. Loading group ts + 1 one compute phase ahead of its use (the previous form) fetched the
  // two halves of a line ~1-2 us apart; with ~6 MB of rows in flight per XCD the line was often evicted from the
  // 4 MB L2 in between and fetched twice (PMC: 868 MB read per call against 557 MB of features). 0.164 -> 0.156 ms
  // same box; the other waves of the CU hide the load latency. A group past HW reads out of the buffer range (zeros,
  // no memory traffic), so no load sits under a branch.
#pragma unroll 1
  for (int ts = 0; ts < NTS; ts += 2) {
    load_group(ts, xb[0], xc[0]);
    load_group(ts + 1, xb[1], xc[1]);
    compute_group(ts, xb[0], xc[0]);
    compute_group(ts + 1, xb[1], xc[1]);
  }
  range_report(d.range_flag, rng);
}

}  // namespace ys

using namespace ys;

YS_EXPORT int yolosod_detect_decode(int nl, const float* const* maps, const int* heights, const int* widths,
                                    const float* strides, int B, int nc, int reg_max, float* y, void* stream) {
  YS_CHECK_ARG(nl >= 1 && nl <= 4, "detect_decode: nl=%d unsupported (1..4)", nl);
  YS_CHECK_ARG(maps && heights && widths && strides && y, "detect_decode: null pointer");
  YS_CHECK_ARG(reg_max == 16, "detect_decode: reg_max=%d unsupported (16)", reg_max);
  YS_CHECK_ARG(B >= 0 && nc >= 0, "detect_decode: bad shape");
  DecodeArgs d{};
  d.nl = nl;
  d.nc = nc;
  d.reg_max = reg_max;
  int off = 0;
  for (int i = 0; i < nl; ++i) {
    YS_CHECK_ARG(maps[i], "detect_decode: null map %d", i);
    d.maps[i] = maps[i];
    d.hw[i] = heights[i] * widths[i];
    d.w[i] = widths[i];
    d.stride[i] = strides[i];
    d.a_off[i] = off;
    off += d.hw[i];
  }
  d.a_off[nl] = off;
  d.A = off;
  d.y = y;
  if (B == 0 || off == 0) return 0;
  hipLaunchKernelGGL(detect_decode_kernel, dim3((off + 255) / 256, B), dim3(256), 0, (hipStream_t)stream, d);
  YS_CHECK_LAUNCH("detect_decode");
  return 0;
}

static int g_head_x2 = -1;  // head 1x1 convs: fp16-split matrix products (1, default) or exact fp32 MFMA (0)
static bool head_x2_env() {
  if (g_head_x2 < 0) {
    const char* e = getenv("YOLOSOD_HEAD_X2");
    g_head_x2 = (e && e[0] == '0') ? 0 : 1;
  }
  return g_head_x2 != 0;
}
// Test hook: route the Detect head through detect_head_x2_kernel (1) or detect_head_lds_kernel (0).
YS_EXPORT int yolosod_debug_set_head_x2(int on) {
  const int prev = head_x2_env() ? 1 : 0;
  g_head_x2 = on ? 1 : 0;
  return prev;
}

// levels [l0, l1) of the nl-level anchor layout (the anchor offsets and A of all nl levels; the other levels' slices
// of y are not written and their feature pointers not read)
static int detect_head_impl(int nl, const void* const* box_feat, const void* const* cls_feat, int c2, int c3,
                            const float* const* box_w, const float* const* box_b, const float* const* cls_w,
                            const float* const* cls_b, const int* heights, const int* widths, const float* strides,
                            int B, int nc, int reg_max, float* y, bool bf16, void* stream, int l0 = 0, int l1 = -1) {
  if (l1 < 0) l1 = nl;
  YS_CHECK_ARG(nl >= 1 && nl <= 4, "detect_head: nl=%d unsupported (1..4)", nl);
  YS_CHECK_ARG(0 <= l0 && l0 < l1 && l1 <= nl, "detect_head: level range [%d, %d) outside [0, %d)", l0, l1, nl);
  YS_CHECK_ARG(box_feat && cls_feat && box_w && box_b && cls_w && cls_b && heights && widths && strides && y,
               "detect_head: null pointer");
  YS_CHECK_ARG(reg_max == 16, "detect_head: reg_max=%d unsupported (16)", reg_max);
  YS_CHECK_ARG(nc >= 1 && nc <= 16, "detect_head: nc=%d unsupported (1..16)", nc);
  YS_CHECK_ARG(c2 == 64 && (c3 == 64 || c3 == 128), "detect_head: (c2=%d, c3=%d) unsupported ((64, 64|128))", c2, c3);
  HeadArgs d{};
  d.nl = l1 - l0;
  d.nc = nc;
  d.range_flag = range_flag_dev();
  constexpr int NTS = 8;  // 16-pixel groups per wave -> 512 pixels per workgroup
  int off = 0, blk = 0;
  for (int i = 0; i < nl; ++i) {
    const int hw = heights[i] * widths[i];
    if (i >= l0 && i < l1) {
      const int k = i - l0;
      YS_CHECK_ARG(box_feat[i] && cls_feat[i] && box_w[i] && box_b[i] && cls_w[i] && cls_b[i],
                   "detect_head: null pointer at level %d", i);
      d.fb[k] = box_feat[i];
      d.fc[k] = cls_feat[i];
      d.wb[k] = box_w[i];
      d.bb[k] = box_b[i];
      d.wc[k] = cls_w[i];
      d.bc[k] = cls_b[i];
      d.hw[k] = hw;
      d.w[k] = widths[i];
      d.stride[k] = strides[i];
      d.a_off[k] = off;
      d.blk_off[k] = blk;
      blk += (hw + 4 * NTS * 16 - 1) / (4 * NTS * 16);
    }
    off += hw;
  }
  d.blk_off[l1 - l0] = blk;
  d.A = off;
  d.y = y;
  if (B == 0 || off == 0) return 0;
  const dim3 grid(blk, B);
  hipStream_t st = (hipStream_t)stream;
  head_x2_env();
  if (bf16) {
    if (g_head_x2) {
      if (c3 == 64) hipLaunchKernelGGL((detect_head_x2_kernel<64, 64, NTS, bf16_t>), grid, dim3(256), 0, st, d);
      else hipLaunchKernelGGL((detect_head_x2_kernel<64, 128, NTS, bf16_t>), grid, dim3(256), 0, st, d);
    } else {
      if (c3 == 64) hipLaunchKernelGGL((detect_head_lds_kernel<64, 64, NTS, bf16_t>), grid, dim3(256), 0, st, d);
      else hipLaunchKernelGGL((detect_head_lds_kernel<64, 128, NTS, bf16_t>), grid, dim3(256), 0, st, d);
    }
    YS_CHECK_LAUNCH("detect_head_bf16");
    return 0;
  }
  // default: fp16-split matrix products (detect_head_x2_kernel); YOLOSOD_HEAD_X2=0 (the split-range fallback):
  // exact fp32 MFMA with the weights in LDS
  if (g_head_x2) {
    if (c3 == 64) hipLaunchKernelGGL((detect_head_x2_kernel<64, 64, NTS>), grid, dim3(256), 0, st, d);
    else hipLaunchKernelGGL((detect_head_x2_kernel<64, 128, NTS>), grid, dim3(256), 0, st, d);
  } else {
    if (c3 == 64) hipLaunchKernelGGL((detect_head_lds_kernel<64, 64, NTS>), grid, dim3(256), 0, st, d);
    else hipLaunchKernelGGL((detect_head_lds_kernel<64, 128, NTS>), grid, dim3(256), 0, st, d);
  }
  YS_CHECK_LAUNCH("detect_head");
  return 0;
}

YS_EXPORT int yolosod_detect_head(int nl, const float* const* box_feat, const float* const* cls_feat, int c2, int c3,
                                  const float* const* box_w, const float* const* box_b, const float* const* cls_w,
                                  const float* const* cls_b, const int* heights, const int* widths,
                                  const float* strides, int B, int nc, int reg_max, float* y, void* stream) {
  return detect_head_impl(nl, (const void* const*)box_feat, (const void* const*)cls_feat, c2, c3, box_w, box_b, cls_w,
                          cls_b, heights, widths, strides, B, nc, reg_max, y, false, stream);
}

// levels [l0, l1) only, into y laid out for all nl levels (the executor launches the levels whose towers are done
// while the last level's towers still run); fp32 or bf16 (bf16 != 0) tower features
YS_EXPORT int yolosod_detect_head_levels(int nl, int l0, int l1, const void* const* box_feat, const void* const* cls_feat,
                                         int c2, int c3, const float* const* box_w, const float* const* box_b,
                                         const float* const* cls_w, const float* const* cls_b, const int* heights,
                                         const int* widths, const float* strides, int B, int nc, int reg_max, float* y,
                                         int bf16, void* stream) {
  return detect_head_impl(nl, box_feat, cls_feat, c2, c3, box_w, box_b, cls_w, cls_b, heights, widths, strides, B, nc,
                          reg_max, y, bf16 != 0, stream, l0, l1);
}

// bf16 tower features (bf16 model config); weights, biases and the decode stay fp32, y is fp32
YS_EXPORT int yolosod_detect_head_bf16(int nl, const bf16_t* const* box_feat, const bf16_t* const* cls_feat, int c2,
                                       int c3, const float* const* box_w, const float* const* box_b,
                                       const float* const* cls_w, const float* const* cls_b, const int* heights,
                                       const int* widths, const float* strides, int B, int nc, int reg_max, float* y,
                                       void* stream) {
  return detect_head_impl(nl, (const void* const*)box_feat, (const void* const*)cls_feat, c2, c3, box_w, box_b, cls_w,
                          cls_b, heights, widths, strides, B, nc, reg_max, y, true, stream);
}
