// SPPF's pooling pyramid in one pass (ultralytics/nn/modules/block.py SPPF.forward: y = [cv1(x)], three chained
// MaxPool2d(5, stride 1, pad 2), torch.cat(y, 1) -> cv2). The executor lets cv1 write its output into channels [0, C)
// of the concat buffer z [B][4C][H][W]; this kernel fills channels [C, 2C), [2C, 3C), [3C, 4C) with the one-, two- and
// three-fold pools. A stride-1 max pool of radius 2 applied k times is the max over the (4k + 1)-square window clipped
// to the image (max_pool2d pads with -inf, so the padding never wins), so the three outputs are windows of radius 2,
// 4, 6 of the same plane: a max over the same elements as the chained pools, hence the same values. Replaces three
// max_pool2d launches (each a full read + write of the plane at ~0.3 TB/s) and the torch.cat copy.
#include "common.h"
#include <math.h>

namespace ys {

constexpr int SPPF_MAX_HW = 64 * 64;  // a plane and its three row-maximum planes in LDS (64 KB at the maximum)

// NaN-propagating max, as max_pool2d's (a NaN anywhere in a window makes that output NaN; fmaxf would drop it)
__device__ __forceinline__ float nan_max(float m, float v) { return (v > m || v != v) ? v : m; }

// one 256-thread workgroup per (channel, image) plane: the plane is read once into LDS; row maxima of radius 2 / 4 / 6
// (each extends the previous one), then column maxima of the same radius over them
__global__ __launch_bounds__(256) void sppf_pool_kernel(float* __restrict__ z, long zbs, int C, int H, int W) {
  extern __shared__ float sm[];
  const int c = blockIdx.x, b = blockIdx.y, HW = H * W, tid = threadIdx.x;
  float* pl = sm;
  float* rm = sm + HW;  // [3][HW]
  const float* src = z + (long)b * zbs + (long)c * HW;
  for (int i = tid; i < HW; i += 256) pl[i] = src[i];
  __syncthreads();
  for (int i = tid; i < HW; i += 256) {
    const int y = i / W, x = i - y * W;
    const float* row = pl + y * W;
    float m = -INFINITY;
#pragma unroll
    for (int d = -2; d <= 2; ++d)
      if (x + d >= 0 && x + d < W) m = nan_max(m, row[x + d]);
    rm[i] = m;
#pragma unroll
    for (int d = 3; d <= 4; ++d) {
      if (x - d >= 0) m = nan_max(m, row[x - d]);
      if (x + d < W) m = nan_max(m, row[x + d]);
    }
    rm[HW + i] = m;
#pragma unroll
    for (int d = 5; d <= 6; ++d) {
      if (x - d >= 0) m = nan_max(m, row[x - d]);
      if (x + d < W) m = nan_max(m, row[x + d]);
    }
    rm[2 * HW + i] = m;
  }
  __syncthreads();
  float* dst = z + (long)b * zbs + (long)c * HW;
  for (int i = tid; i < HW; i += 256) {
    const int y = i / W, x = i - y * W;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int r = 2 * (k + 1);
      const float* col = rm + k * HW + x;
      float m = -INFINITY;
      const int y0 = y - r < 0 ? 0 : y - r, y1 = y + r >= H ? H - 1 : y + r;
      for (int yy = y0; yy <= y1; ++yy) m = nan_max(m, col[yy * W]);
      dst[(long)(k + 1) * C * HW + i] = m;
    }
  }
}

}  // namespace ys

using namespace ys;

// z [B][4C][H][W] (image b at z + b z_bstride, images contiguous): channels [C, 4C) <- the 5 / 9 / 13 max pools
// (stride 1, the window clipped to the image) of channels [0, C). H W <= 4096.
YS_EXPORT int yolosod_sppf_pool(float* z, long z_bstride, int B, int C, int H, int W, void* stream) {
  YS_CHECK_ARG(z, "sppf_pool: null pointer");
  YS_CHECK_ARG(B >= 0 && C > 0 && H > 0 && W > 0 && H * W <= SPPF_MAX_HW, "sppf_pool: bad shape (H W <= %d)",
               SPPF_MAX_HW);
  YS_CHECK_ARG(z_bstride >= 4L * C * H * W, "sppf_pool: batch stride %ld < 4 C H W", z_bstride);
  YS_CHECK_ARG(C <= 65535 && B <= 65535, "sppf_pool: grid too large");
  if (B == 0) return 0;
  const size_t lds = (size_t)4 * H * W * sizeof(float);
  hipLaunchKernelGGL(sppf_pool_kernel, dim3((unsigned)C, (unsigned)B), dim3(256), lds, (hipStream_t)stream, z,
                     z_bstride, C, H, W);
  YS_CHECK_LAUNCH("sppf_pool");
  return 0;
}
