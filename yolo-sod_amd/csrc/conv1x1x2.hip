// 1x1 convolution (stride 1, groups 1) + folded BN bias + SiLU on the fp16 matrix cores at fp32 accuracy, for the
// PAN neck's wide 1x1 convs (C2f cv1 / cv2 and the lateral convs of the paper YAML: Cout 128..512, Cin 128..1024;
// ultralytics/nn/modules/conv.py:37-55 with the BN folded by fuse(), block.py:249-253 for C2f's split / concat).
// Per image a GEMM y[Cout][HW] = W[Cout][Cin] x[Cin][HW], epilogue fused: bias, SiLU, the output written into a
// channel slice of a concat buffer, optionally its channels [c2lo, Cout) stored a second time packed (C2f's first
// Bottleneck input). Replaces MIOpen's fp32 GEMM (v_mfma_f32_16x16x4_f32, 157 TF/s) + the separate bias / SiLU pass.
//
// Method as conv3x3.hip: two-term fp16 splits, three v_mfma_f32_16x16x32_f16 per product block, weights x 64 split
// once per parameter version into fragment-major planes (k step s of 32 input channels, 16-channel output block cb,
// plane p: the 64 lanes' fragments are 1 KB contiguous). One 256-thread workgroup per (image, 64-pixel tile, 128
// output channels): per stage of 128 input channels the x tile [128][64] is loaded (4 channels of one pixel per item,
// consecutive threads on consecutive pixels), split and stored as two fp16 planes [pixel][channel] in LDS; wave w
// computes output channel blocks 2 w, 2 w + 1 for the 4 pixel blocks, pixels as the MFMA A operand (a lane holds 4
// consecutive pixels of one channel: 16-byte stores). The next stage's loads are spread over the current stage's
// k steps behind each step's weight prefetch (vmcnt counts in issue order); sched barriers keep them there.
#include "common.h"

namespace ys {
namespace c1 {

constexpr float WSC = 64.0f;
constexpr int KS = 128;        // input channels per stage
constexpr int PS = KS + 8;     // plane row stride (halves): 272-byte pixel rows
constexpr int NT = 256;

struct Args {
  const float* x;      // image b at x + b xbs: [Cin][HW]
  long xbs;
  const h16_t* wp;     // prepared planes
  const float* bias;   // [Cout]
  float* y;            // image b at y + b ybs: [Cout][HW]
  long ybs;
  float* y2;           // optional: channels [c2lo, Cout) again at y2 + b y2bs: [Cout - c2lo][HW]
  long y2bs;
  int c2lo, cin, cout, HW, ntile;
  unsigned* range_flag;
  const unsigned* prep_flag;
  const float* x2;     // optional second input (a virtual concat): channels [k1, Cin) at x2 + b x2bs ([Cin - k1][HW])
  long x2bs;
  int k1;              // channels taken from x (Cin when x2 is NULL; else a multiple of KS)
};

// NP pixels per tile (64 or 128: the weights are read from L2 once per tile, 128 halves that traffic)
// CPW: 16-channel output blocks per wave (2: workgroups of 128 output channels; 1: of 64, for Cout 64)
template <bool DUAL, int NP, int CPW = 2>
__global__ __launch_bounds__(NT, 2) void conv1x1_x2_kernel(Args p) {
  constexpr int PL = NP * PS;           // plane (halves)
  constexpr int NITEM = (KS / 4) * NP;  // (channel quad, pixel) items per stage
  constexpr int NIT = NITEM / NT;
  constexpr int NPB = NP / 16;          // pixel blocks
  static_assert(NITEM % NT == 0, "items");
  __shared__ __attribute__((aligned(16))) h16_t Pl[2 * PL];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, g = lane >> 4;
  const int ngrp = p.cout / (64 * CPW);
  const int grp = blockIdx.x % ngrp, tile = (blockIdx.x / ngrp) % p.ntile, b = blockIdx.x / (ngrp * p.ntile);
  const int HW = p.HW, p0 = tile * NP, nst = (p.cin + KS - 1) / KS, nks = nst * (KS / 32);  // weights padded to KS
  float rng = 0.f;

  auto rsrc = [&](const void* base, unsigned bytes) {
    const unsigned long long a = (unsigned long long)base;
    return __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(a >> 32)) << 32) |
                (unsigned)__builtin_amdgcn_readfirstlane((unsigned)a)),
        (short)0, __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
  };
  // the part of a virtual concat a stage reads (stages from k1 / KS on: x2) as a buffer resource built from scalars
  // per stage (a select between two resource values is lowered to VGPRs, and every load then runs a waterfall loop)
  const float* xb1 = p.x + (long)b * p.xbs;
  const float* xb2 = p.x2 ? p.x2 + (long)b * p.x2bs : xb1;
  const unsigned nb1 = (unsigned)((long)p.k1 * HW * 4), nb2 = (unsigned)((long)(p.cin - p.k1) * HW * 4);
  const __amdgpu_buffer_rsrc_t rw = rsrc(p.wp, (unsigned)((long)nks * (p.cout >> 4) * 2 * 1024));

  // staging item e = tid + NT i: channel quad e / NP (channels 4 quad .. + 3 of the stage), pixel e % NP (clamped
  // to the image: pixels past HW load the last pixel, their outputs are not stored)
  unsigned voff[NIT];
#pragma unroll
  for (int i = 0; i < NIT; ++i) {
    const int e = tid + NT * i, quad = e / NP, px = e - quad * NP;
    voff[i] = (unsigned)((4 * quad * HW + min(p0 + px, HW - 1)) * 4);
  }
  f32x4 sv[NIT];
  // the stage / channel offset is in the per-lane offset, so the buffer range check covers it: channels past Cin
  // (the last stage of a Cin that is not a multiple of KS) read 0, as do the padded weights they meet
  auto load_part = [&](int st, int k0, int k1, bool live) __attribute__((always_inline)) {
    const bool second = KS * st >= p.k1;  // stage-uniform
    const unsigned sx = (unsigned)((second ? KS * st - p.k1 : KS * st) * HW * 4);
    // !live: an empty range (the last stage's "next stage" loads return 0 at once)
    const __amdgpu_buffer_rsrc_t r = rsrc(second ? xb2 : xb1, live ? (second ? nb2 : nb1) : 0u);
#pragma unroll
    for (int k = 0; k < 4 * NIT; ++k)
      if (k >= k0 && k < k1)
        sv[k >> 2][k & 3] = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(r, voff[k >> 2] + sx + (unsigned)((k & 3) * HW * 4), 0, 0));
  };
  // weight fragments of k step s (global), channel blocks cb0 + u, planes 0 / 1
  const int cb0 = grp * 4 * CPW + CPW * wid;
  auto wfrag = [&](int s, int u, int pl) __attribute__((always_inline)) {
    const int st = __builtin_amdgcn_readfirstlane((s * (p.cout >> 4) * 2) * 1024);
    return __builtin_bit_cast(f16x8_t, __builtin_amdgcn_raw_buffer_load_b128(
                                           rw, (unsigned)((((cb0 + u) * 2 + pl) * 64 + lane) * 16), st, 0));
  };
  f32x4 acc[CPW][NPB];
#pragma unroll
  for (int u = 0; u < CPW; ++u)
#pragma unroll
    for (int k = 0; k < NPB; ++k) acc[u][k] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bo[CPW];  // loaded before the loop: an epilogue load would wait behind every load in flight
#pragma unroll
  for (int u = 0; u < CPW; ++u) bo[u] = p.bias[16 * (cb0 + u) + l15];

  load_part(0, 0, 4 * NIT, true);
  for (int st = 0; st < nst; ++st) {
    __syncthreads();  // every wave is done with the previous stage's planes
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int e = tid + NT * i, quad = e / NP, px = e - quad * NP;
      uint2 hh, ll;
      split4x(sv[i], hh, ll);
      rng = range_acc(rng, sv[i]);
      h16_t* d = Pl + px * PS + 4 * quad;
      *reinterpret_cast<uint2*>(d) = hh;
      *reinterpret_cast<uint2*>(d + PL) = ll;
    }
    __syncthreads();
    const bool nlive = st + 1 < nst;
    const int stn = nlive ? st + 1 : st;
    f16x8_t wa[CPW][2], wn[CPW][2];
#pragma unroll
    for (int u = 0; u < CPW; ++u) {
      wa[u][0] = wfrag(4 * st, u, 0);
      wa[u][1] = wfrag(4 * st, u, 1);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < KS / 32; ++kk) {
      const int sn = kk + 1 < KS / 32 ? 4 * st + kk + 1 : 4 * st + kk;  // one k step ahead (unconditional)
#pragma unroll
      for (int u = 0; u < CPW; ++u) {
        wn[u][0] = wfrag(sn, u, 0);
        wn[u][1] = wfrag(sn, u, 1);
      }
      load_part(stn, NIT * kk, NIT * kk + NIT, nlive);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < NPB; ++k) {
        const h16_t* src = Pl + (16 * k + l15) * PS + 32 * kk + 8 * g;
        const f16x8_t xh = *reinterpret_cast<const f16x8_t*>(src);
        const f16x8_t xl = *reinterpret_cast<const f16x8_t*>(src + PL);
#pragma unroll
        for (int u = 0; u < CPW; ++u) {
          f32x4 c = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh, wa[u][1], acc[u][k], 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(xl, wa[u][0], c, 0, 0, 0);
          acc[u][k] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh, wa[u][0], c, 0, 0, 0);
        }
      }
#pragma unroll
      for (int u = 0; u < CPW; ++u) {
        wa[u][0] = wn[u][0];
        wa[u][1] = wn[u][1];
      }
    }
  }
  // epilogue: lane (g, l15) of (u, pixel block k) holds channel 16 (cb0 + u) + l15, pixels 16 k + 4 g .. + 3
  float* yb = p.y + (long)b * p.ybs;
#pragma unroll
  for (int u = 0; u < CPW; ++u) {
    const int o = 16 * (cb0 + u) + l15;
#pragma unroll
    for (int k = 0; k < NPB; ++k) {
      const int px = p0 + 16 * k + 4 * g;
      f32x4 v;
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = silu_fast_(acc[u][k][j] * (1.0f / WSC) + bo[u]);
      if (px < HW) {  // HW % 4 == 0: 4 pixels all in or all out
        __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(yb + (long)o * HW + px));
        if (DUAL && o >= p.c2lo)
          __builtin_nontemporal_store(
              v, reinterpret_cast<f32x4*>(p.y2 + (long)b * p.y2bs + (long)(o - p.c2lo) * HW + px));
      }
    }
  }
  range_report(p.range_flag, rng);
  if (p.prep_flag && p.range_flag && blockIdx.x == 0 && threadIdx.x == 0 && *p.prep_flag) *p.range_flag = 1u;
}

// W [Cout][Cin] -> fragment-major planes of 64 W: one thread per (output channel, input channel)
__global__ __launch_bounds__(256) void conv1x1_prep_kernel(const float* __restrict__ w, int cin, int cin_pad,
                                                           int cout, h16_t* __restrict__ wp, unsigned* range_flag,
                                                           unsigned* prep_flag) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)cout * cin_pad) return;
  const int k = (int)(i % cin_pad), n = (int)(i / cin_pad);
  const float v = k < cin ? w[(long)n * cin + k] * WSC : 0.f;  // zero weights for the padded channels
  const _Float16 hh = (_Float16)v;
  const _Float16 ll = (_Float16)(v - (float)hh);
  const int s = k >> 5, kk = k & 31, cbk = n >> 4, ncb = cout >> 4;
  const int ln = ((kk >> 3) << 4) + (n & 15);
  const long base = ((long)(s * ncb + cbk) * 2) * 512 + ln * 8 + (kk & 7);
  wp[base] = __builtin_bit_cast(h16_t, hh);
  wp[base + 512] = __builtin_bit_cast(h16_t, ll);
  const float m = fabsf(v);
  range_report(range_flag, m);
  range_report(prep_flag, m);
}

}  // namespace c1
}  // namespace ys

using namespace ys;

static int c1_pad(int cin) { return (cin + c1::KS - 1) / c1::KS * c1::KS; }

// Cout 64 or a multiple of 128 (<= 1024), Cin a multiple of 32 (<= 4096; the weights are padded to a multiple of 128)
YS_EXPORT size_t yolosod_conv1x1x2_prep_bytes(int cin, int cout) {
  if (cin <= 0 || cin % 32 || cin > 4096 || cout <= 0 || (cout != 64 && cout % 128) || cout > 1024) return 0;
  Sizer s;
  s.take<h16_t>((size_t)2 * cout * c1_pad(cin));
  s.take<unsigned>(1);
  return s.off;
}

static bool c1_carve(void* buf, size_t bytes, int cin, int cout, h16_t** wp, unsigned** flag) {
  Carver cv(buf, bytes);
  *wp = cv.take<h16_t>((size_t)2 * cout * c1_pad(cin));
  *flag = cv.take<unsigned>(1);
  return *flag != nullptr;
}

// Weight preparation (re-run whenever the weights change): w [cout][cin] fp32 (BN folded) -> prep block.
YS_EXPORT int yolosod_conv1x1x2_prepare(const float* w, int cin, int cout, void* prep, size_t prep_bytes,
                                        void* stream) {
  YS_CHECK_ARG(w && prep, "conv1x1x2_prepare: null pointer");
  YS_CHECK_ARG(yolosod_conv1x1x2_prep_bytes(cin, cout) > 0, "conv1x1x2_prepare: (cin=%d, cout=%d) unsupported", cin,
               cout);
  h16_t* wp;
  unsigned* flag;
  YS_CHECK_ARG(c1_carve(prep, prep_bytes, cin, cout, &wp, &flag), "conv1x1x2_prepare: block too small (%zu)",
               prep_bytes);
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(flag, 0, sizeof(unsigned), st) != hipSuccess) {
    set_error("conv1x1x2_prepare: flag reset failed");
    return -1;
  }
  const long n = (long)cout * c1_pad(cin);
  hipLaunchKernelGGL(c1::conv1x1_prep_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, w, cin, c1_pad(cin),
                     cout, wp, range_flag_dev(), flag);
  YS_CHECK_LAUNCH("conv1x1x2_prep");
  return 0;
}

// y = SiLU(W [x; x2] + bias): x image b at x + b x_bstride ([k1][HW]), x2 (or NULL) image b at x2 + b x2_bstride
// ([cin - k1][HW]: the second part of a virtual concat, k1 a multiple of 128), y image b at y + b y_bstride
// ([cout][HW]); y2 (or NULL): channels [c2lo, cout) stored again at y2 + b y2_bstride. HW % 4 == 0; 16-byte aligned
// images.
YS_EXPORT int yolosod_conv1x1x2_silu_cat(const float* x, long x_bstride, const float* x2, long x2_bstride, int k1,
                                         float* y, long y_bstride, float* y2, long y2_bstride, int c2lo, int B, int cin,
                                         int cout, int HW, const float* bias, const void* prep, size_t prep_bytes,
                                         void* stream) {
  YS_CHECK_ARG(x && y && bias && prep, "conv1x1x2: null pointer");
  if (!x2) k1 = cin;
  YS_CHECK_ARG(k1 > 0 && k1 <= cin && (!x2 || (k1 % c1::KS == 0 && k1 < cin && x2_bstride >= (long)(cin - k1) * HW)),
               "conv1x1x2: concat split k1=%d (Cin %d) must be a multiple of %d", k1, cin, c1::KS);
  YS_CHECK_ARG(B >= 0 && HW > 0 && HW % 4 == 0 && yolosod_conv1x1x2_prep_bytes(cin, cout) > 0, "conv1x1x2: bad shape");
  YS_CHECK_ARG(x_bstride >= (long)k1 * HW && y_bstride >= (long)cout * HW, "conv1x1x2: batch strides too small");
  YS_CHECK_ARG((long)c1_pad(cin) * HW * 4 < (1L << 32), "conv1x1x2: image too large for 32-bit buffer offsets");
  YS_CHECK_ARG((((uintptr_t)y | (uintptr_t)(y2 ? y2 : y)) & 15) == 0 && y_bstride % 4 == 0 && y2_bstride % 4 == 0,
               "conv1x1x2: outputs must be 16-byte aligned");
  YS_CHECK_ARG(!y2 || (c2lo >= 0 && c2lo < cout && y2_bstride >= (long)(cout - c2lo) * HW), "conv1x1x2: c2lo=%d",
               c2lo);
  if (B == 0) return 0;
  h16_t* wp;
  unsigned* flag;
  YS_CHECK_ARG(c1_carve(const_cast<void*>(prep), prep_bytes, cin, cout, &wp, &flag),
               "conv1x1x2: prepared block too small");
  constexpr int NPx = 64;  // pixels per tile (128-pixel tiles measured slower on four of five neck shapes)
  const int ntile = (HW + NPx - 1) / NPx;
  c1::Args a{x, x_bstride, wp, bias, y, y_bstride, y2, y2_bstride, c2lo, cin, cout, HW, ntile, range_flag_dev(), flag,
             x2, x2_bstride, k1};
  const long nwg = (long)B * ntile * (cout == 64 ? 1 : cout / 128);
  YS_CHECK_ARG(nwg < (1L << 31), "conv1x1x2: too many tiles");
  hipStream_t st = (hipStream_t)stream;
  if (cout == 64) {  // one 64-channel group: a 16-channel block per wave
    if (y2) hipLaunchKernelGGL((c1::conv1x1_x2_kernel<true, 64, 1>), dim3((unsigned)nwg), dim3(c1::NT), 0, st, a);
    else hipLaunchKernelGGL((c1::conv1x1_x2_kernel<false, 64, 1>), dim3((unsigned)nwg), dim3(c1::NT), 0, st, a);
  } else {
    if (y2) hipLaunchKernelGGL((c1::conv1x1_x2_kernel<true, NPx>), dim3((unsigned)nwg), dim3(c1::NT), 0, st, a);
    else hipLaunchKernelGGL((c1::conv1x1_x2_kernel<false, NPx>), dim3((unsigned)nwg), dim3(c1::NT), 0, st, a);
  }
  YS_CHECK_LAUNCH("conv1x1x2");
  return 0;
}

// y = SiLU(W x + bias) for one input tensor (yolosod_conv1x1x2_silu_cat without a second part)
YS_EXPORT int yolosod_conv1x1x2_silu(const float* x, long x_bstride, float* y, long y_bstride, float* y2,
                                     long y2_bstride, int c2lo, int B, int cin, int cout, int HW, const float* bias,
                                     const void* prep, size_t prep_bytes, void* stream) {
  return yolosod_conv1x1x2_silu_cat(x, x_bstride, nullptr, 0, cin, y, y_bstride, y2, y2_bstride, c2lo, B, cin, cout, HW,
                                    bias, prep, prep_bytes, stream);
}
