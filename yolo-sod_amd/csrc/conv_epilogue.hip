// Conv epilogue for the PyTorch-ROCm backbone convolutions: out = act(y + bias[c]) (+ res), one HBM pass.
//
// PyTorch runs a fused Conv (nn/modules/conv.py:37-55 after fuse(), tasks.py:227-255) as MIOpen conv, then a
// separate bias-add pass and a separate SiLU pass (MIOpen's fusion API has no SiLU); Bottleneck adds its shortcut
// in a third pass and C2f/Concat copy everything once more into torch.cat. This kernel does bias + activation
// (+ shortcut) in one read/write and can write straight into a channel slice of a preallocated concat buffer
// (out batch stride != C*HW), so those passes and copies disappear. Same arithmetic as the reference:
// (conv + b) rounded once, SiLU = x / (1 + exp(-x)).
#include "common.h"

namespace ys {

template <int ACT, bool RES>
__global__ __launch_bounds__(256) void bias_act_kernel(const float* __restrict__ y, float* __restrict__ out,
                                                       const float* __restrict__ bias, const float* __restrict__ res,
                                                       int C, long HW4, long y_bs4, long o_bs4, long r_bs4,
                                                       long total4) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total4; i += (long)gridDim.x * 256) {
    const long b = i / ((long)C * HW4);
    const long rem = i - b * (long)C * HW4;
    const int c = (int)(rem / HW4);
    const float bc = bias[c];
    float4 v = reinterpret_cast<const float4*>(y)[b * y_bs4 + rem];
    v.x += bc; v.y += bc; v.z += bc; v.w += bc;
    if (ACT == 1) {
      v.x = siluf_(v.x); v.y = siluf_(v.y); v.z = siluf_(v.z); v.w = siluf_(v.w);
    }
    if (RES) {
      const float4 r = reinterpret_cast<const float4*>(res)[b * r_bs4 + rem];
      v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
    }
    reinterpret_cast<float4*>(out)[b * o_bs4 + rem] = v;
  }
}

}  // namespace ys

using namespace ys;

// out[b*out_bstride + c*HW + p] = act(y[b*y_bstride + c*HW + p] + bias[c]) + res[b*res_bstride + c*HW + p]
// act: 0 identity, 1 SiLU. res may be NULL. In place (out == y) allowed. HW and all strides multiples of 4.
YS_EXPORT int yolosod_bias_act(const float* y, long y_bstride, float* out, long out_bstride, const float* bias,
                               const float* res, long res_bstride, int B, int C, long HW, int act, void* stream) {
  YS_CHECK_ARG(y && out && bias, "bias_act: null pointer");
  YS_CHECK_ARG(act == 0 || act == 1, "bias_act: act=%d unsupported", act);
  YS_CHECK_ARG(HW % 4 == 0 && y_bstride % 4 == 0 && out_bstride % 4 == 0 && (!res || res_bstride % 4 == 0),
               "bias_act: HW and batch strides must be multiples of 4");
  YS_CHECK_ARG((((uintptr_t)y | (uintptr_t)out | (uintptr_t)(res ? res : y)) & 15) == 0,
               "bias_act: pointers must be 16-byte aligned");
  const long total4 = (long)B * C * (HW / 4);
  if (total4 == 0) return 0;
  long blocks = (total4 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipStream_t st = (hipStream_t)stream;
  const long hw4 = HW / 4, yb = y_bstride / 4, ob = out_bstride / 4, rb = res_bstride / 4;
  if (act == 1) {
    if (res) hipLaunchKernelGGL((bias_act_kernel<1, true>), dim3(blocks), dim3(256), 0, st, y, out, bias, res, C, hw4, yb, ob, rb, total4);
    else hipLaunchKernelGGL((bias_act_kernel<1, false>), dim3(blocks), dim3(256), 0, st, y, out, bias, res, C, hw4, yb, ob, rb, total4);
  } else {
    if (res) hipLaunchKernelGGL((bias_act_kernel<0, true>), dim3(blocks), dim3(256), 0, st, y, out, bias, res, C, hw4, yb, ob, rb, total4);
    else hipLaunchKernelGGL((bias_act_kernel<0, false>), dim3(blocks), dim3(256), 0, st, y, out, bias, res, C, hw4, yb, ob, rb, total4);
  }
  YS_CHECK_LAUNCH("bias_act");
  return 0;
}
