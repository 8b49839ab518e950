// Conv epilogue for the PyTorch-ROCm backbone convolutions: out = act(y + bias[c]) (+ res), one HBM pass.
//
// PyTorch runs a fused Conv (nn/modules/conv.py:37-55 after fuse(), tasks.py:227-255) as MIOpen conv, then a
// separate bias-add pass and a separate SiLU pass (MIOpen's fusion API has no SiLU); Bottleneck adds its shortcut
// in a third pass and C2f/Concat copy everything once more into torch.cat. This kernel does bias + activation
// (+ shortcut) in one read/write and can write straight into a channel slice of a preallocated concat buffer
// (out batch stride != C*HW), so those passes and copies disappear. Same arithmetic as the reference:
// (conv + b) rounded once, SiLU = x / (1 + exp(-x)).
#include "common.h"
#include <math.h>

namespace ys {

// SiLU of an epilogue value: bf16 storage uses the hardware exp2 / rcp form (error ~2^-22 relative, far below the
// bf16 rounding of the store; the libm expf + IEEE division made the bf16 passes VALU-bound), fp32 storage the
// libm form (x / (1 + exp(-x)), the reference's arithmetic)
template <class T>
__device__ __forceinline__ float silu_st(float v) {
#ifdef YS_FAST_SILU_F32  // A/B builds only: the fast form for fp32 storage too
  return silu_fast_(v);
#else
  if constexpr (sizeof(T) == 2) return silu_fast_(v);
  else return siluf_(v);
#endif
}

template <int ACT, bool RES, bool DUAL = false, class T = float>
__global__ __launch_bounds__(256) void bias_act_kernel(const T* __restrict__ y, T* __restrict__ out,
                                                       const float* __restrict__ bias, const T* __restrict__ res,
                                                       int C, long HW4, long y_bs4, long o_bs4, long r_bs4,
                                                       long total4, int rev, T* __restrict__ out2 = nullptr,
                                                       int c2lo = 0, long o2_bs4 = 0) {
  for (long i0 = (long)blockIdx.x * 256 + threadIdx.x; i0 < total4; i0 += (long)gridDim.x * 256) {
    const long i = rev ? total4 - 1 - i0 : i0;
    const long b = i / ((long)C * HW4);
    const long rem = i - b * (long)C * HW4;
    const int c = (int)(rem / HW4);
    const float bc = bias[c];
    f32x4 v = ld4(y + 4 * (b * y_bs4 + rem));
    v += bc;
    if (ACT == 1) {
      v.x = silu_st<T>(v.x); v.y = silu_st<T>(v.y); v.z = silu_st<T>(v.z); v.w = silu_st<T>(v.w);
    }
    if (RES) v += ld4(res + 4 * (b * r_bs4 + rem));
    st4(out + 4 * (b * o_bs4 + rem), v);
    // second, packed copy of channels [c2lo, C): the next conv's input without a separate .contiguous() pass
    if (DUAL && c >= c2lo) st4(out2 + 4 * (b * o2_bs4 + rem - (long)c2lo * HW4), v);
  }
}

// bf16 storage, 8 elements (16 bytes) per access: the same grid-stride walk in 8-element units (HW % 8 == 0, batch
// strides % 8 == 0, 16-byte aligned). With 4 elements per access (8 bytes) the bf16 epilogues ran at 2-3.3 TB/s.
// The bf16 config's semantics: fp32 arithmetic, one rounding on store.
template <int ACT, bool RES, bool DUAL>
__global__ __launch_bounds__(256) void bias_act8_bf16_kernel(const bf16_t* __restrict__ y, bf16_t* __restrict__ out,
                                                             const float* __restrict__ bias,
                                                             const bf16_t* __restrict__ res, int C, long HW8,
                                                             long y_bs8, long o_bs8, long r_bs8, long total8, int rev,
                                                             bf16_t* __restrict__ out2, int c2lo, long o2_bs8) {
  for (long i0 = (long)blockIdx.x * 256 + threadIdx.x; i0 < total8; i0 += (long)gridDim.x * 256) {
    const long i = rev ? total8 - 1 - i0 : i0;
    const long b = i / ((long)C * HW8);
    const long rem = i - b * (long)C * HW8;
    const int c = (int)(rem / HW8);
    const float bc = bias[c];
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(y + 8 * (b * y_bs8 + rem)), f);
    float r[8];
    if (RES) unpack8(*reinterpret_cast<const uint4*>(res + 8 * (b * r_bs8 + rem)), r);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = f[j] + bc;
      if (ACT == 1) v = silu_st<bf16_t>(v);
      if (RES) v += r[j];
      f[j] = v;
    }
    const uint4 o = pack8(f);
    *reinterpret_cast<uint4*>(out + 8 * (b * o_bs8 + rem)) = o;
    if (DUAL && c >= c2lo) *reinterpret_cast<uint4*>(out2 + 8 * (b * o2_bs8 + rem - (long)c2lo * HW8)) = o;
  }
}

// Same epilogue, plus the per-plane partial statistics of `out` that a following SE / CBAM channel gate needs
// (smallobj_modules.py:87 mean, cbam_block.py:14-17 mean + max): workgroup (plane, k) handles the plane segment
// [k*seg, (k+1)*seg) - the segmentation of channel_attention.hip's part_plan - and writes psum/pmax[plane*parts + k].
// The gate then needs no extra pass over the producer's output.
// V8 (bf16 storage, segment and plane multiples of 8, 16-byte aligned): 8 elements per 16-byte access.
template <int ACT, bool RES, bool MAX, class T = float, bool V8 = false>
__global__ __launch_bounds__(256) void bias_act_stats_kernel(const T* __restrict__ y, T* __restrict__ out,
                                                             const float* __restrict__ bias,
                                                             const T* __restrict__ res, int C, long HW,
                                                             long y_bs, long o_bs, long r_bs, int parts, long seg,
                                                             float* __restrict__ psum, float* __restrict__ pmax,
                                                             int rev) {
  const long bx = rev ? (long)gridDim.x - 1 - blockIdx.x : (long)blockIdx.x;
  const long plane = bx / parts;
  const int k = (int)(bx % parts);
  const long b = plane / C;
  const int c = (int)(plane - b * C);
  const long s0 = k * seg;
  const long s1 = (s0 + seg < HW) ? s0 + seg : HW;
  const float bc = bias[c];
  const T* y4 = y + b * y_bs + (long)c * HW + s0;
  const T* r4 = RES ? res + b * r_bs + (long)c * HW + s0 : nullptr;
  T* o4 = out + b * o_bs + (long)c * HW + s0;
  const long n4 = (s1 - s0) >> 2;
  const int tid = threadIdx.x;
  float s = 0.f, m = -INFINITY;
  if constexpr (V8 && sizeof(T) == 2) {
    const long n8 = (s1 - s0) >> 3;
    for (long i0 = tid; i0 < n8; i0 += 4 * 256) {
      uint4 v[4], r[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long i = i0 + u * 256;
        if (i < n8) {
          v[u] = *reinterpret_cast<const uint4*>(y4 + 8 * i);
          if (RES) r[u] = *reinterpret_cast<const uint4*>(r4 + 8 * i);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long i = i0 + u * 256;
        if (i >= n8) continue;
        float f[8], rr[8];
        unpack8(v[u], f);
        if (RES) unpack8(r[u], rr);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float o = f[j] + bc;
          if (ACT == 1) o = silu_st<T>(o);
          if (RES) o += rr[j];
          f[j] = o;
        }
        const uint4 ob = pack8(f);
        *reinterpret_cast<uint4*>(o4 + 8 * i) = ob;
        unpack8(ob, f);  // statistics of the stored (rounded) values
        s += ((f[0] + f[1]) + (f[2] + f[3])) + ((f[4] + f[5]) + (f[6] + f[7]));
        if (MAX)
          m = fmaxf(m, fmaxf(fmaxf(fmaxf(f[0], f[1]), fmaxf(f[2], f[3])), fmaxf(fmaxf(f[4], f[5]), fmaxf(f[6], f[7]))));
      }
    }
  } else
  for (long i0 = tid; i0 < n4; i0 += 4 * 256) {
    f32x4 v[4], r[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long i = i0 + u * 256;
      if (i < n4) {
        v[u] = ld4(y4 + 4 * i);
        if (RES) r[u] = ld4(r4 + 4 * i);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long i = i0 + u * 256;
      if (i >= n4) continue;
      f32x4 o = v[u] + bc;
      if (ACT == 1) {
        o.x = silu_st<T>(o.x); o.y = silu_st<T>(o.y); o.z = silu_st<T>(o.z); o.w = silu_st<T>(o.w);
      }
      if (RES) o += r[u];
      st4(o4 + 4 * i, o);
      // statistics of the stored values (bf16 storage: of the rounded values, as a consumer re-reading out sees)
      if (sizeof(T) == 2) o = round_bf16(o);
      s += (o.x + o.y) + (o.z + o.w);
      if (MAX) m = fmaxf(m, fmaxf(fmaxf(o.x, o.y), fmaxf(o.z, o.w)));
    }
  }
  __shared__ float ss[4], sm[4];
  s = wave_sum(s);
  if (MAX) m = wave_max(m);
  const int w = tid >> 6;
  if ((tid & 63) == 0) {
    ss[w] = s;
    sm[w] = m;
  }
  __syncthreads();
  if (tid == 0) {
    psum[bx] = (ss[0] + ss[1]) + (ss[2] + ss[3]);
    if (MAX) pmax[bx] = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
  }
}

// Same epilogue for a conv whose output feeds a CA_Block (ca_block.py:43-44): the pass also produces the plane's row
// means (over W) and column means (over H) in yin[b][c][0..H+W), the input of CA's gate, so CA never runs its
// pooling pass over the feature map. One workgroup per plane; the activated plane streams through LDS in bands of
// <= 8192 floats, every thread's (at most 8) 16-byte loads of a band issued before the first is used (with one load
// in flight per thread the kernel ran at 2.2x the plain epilogue's time on a cold HBM input). Rows are reduced by
// lane quads over float4s; columns as float4 quads by NG = 256 / (W/4) row groups, whose partials meet in LDS at the
// end.
template <int ACT, bool RES, class T = float>
__global__ __launch_bounds__(256) void bias_act_capool_kernel(const T* __restrict__ y, T* __restrict__ out,
                                                              const float* __restrict__ bias,
                                                              const T* __restrict__ res, int C, int H, int W,
                                                              int RB, long y_bs, long o_bs, long r_bs,
                                                              float* __restrict__ yin) {
  extern __shared__ __attribute__((aligned(16))) float band[];  // [RB * W] band + [NG * W] column partials
  const long plane = blockIdx.x;
  const long b = plane / C;
  const int c = (int)(plane - b * C);
  const long HW = (long)H * W;
  const T* yp = y + b * y_bs + (long)c * HW;
  T* op = out + b * o_bs + (long)c * HW;
  const T* rp = RES ? res + b * r_bs + (long)c * HW : nullptr;
  float* o = yin + plane * (long)(H + W);
  const float bc = bias[c];
  const int tid = threadIdx.x;
  const int W4 = W >> 2, NG = 256 / W4;
  const int cq = tid % W4, rg = tid / W4;
  f32x4* band4 = reinterpret_cast<f32x4*>(band);
  f32x4 col = f32x4{0.f, 0.f, 0.f, 0.f};
  const float invW = 1.0f / (float)W;
  for (int h0 = 0; h0 < H; h0 += RB) {
    const int rb = (H - h0 < RB) ? H - h0 : RB;
    const int n4 = rb * W4;  // <= 2048 = 8 per thread
    const long base = (long)h0 * W;
    // loads unconditional (index clamped into the band), all values computed, then the predicated stores: loads
    // under per-u predicates left the waitcnt pass exec-masked regions it merged conservatively, so each u's block
    // began with vmcnt(0) - which on gfx950 also waits for the previous block's global store to complete
    f32x4 v[8], r[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = tid + 256 * u < n4 ? tid + 256 * u : n4 - 1;
      v[u] = ld4(yp + base + 4 * i);
      if (RES) r[u] = ld4(rp + base + 4 * i);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      f32x4 t = v[u] + bc;
      if (ACT == 1) {
        t.x = silu_st<T>(t.x); t.y = silu_st<T>(t.y); t.z = silu_st<T>(t.z); t.w = silu_st<T>(t.w);
      }
      if (RES) t += r[u];
      v[u] = t;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = tid + 256 * u;
      if (i < n4) {
        f32x4 t = v[u];
        st4(op + base + 4 * i, t);
        if (sizeof(T) == 2) t = round_bf16(t);  // pool the stored (rounded) values
        band4[i] = t;
      }
    }
    __syncthreads();
    for (int rr = tid >> 2; rr < rb; rr += 64) {
      f32x4 s4 = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int q = tid & 3; q < W4; q += 4) s4 += band4[rr * W4 + q];
      const float sm = quad_sum((s4.x + s4.y) + (s4.z + s4.w));
      if ((tid & 3) == 0) o[h0 + rr] = sm * invW;
    }
    if (rg < NG)
      for (int rr = rg; rr < rb; rr += NG) col += band4[rr * W4 + cq];
    __syncthreads();
  }
  float* cpart = band + (long)RB * W;
  if (rg < NG) reinterpret_cast<f32x4*>(cpart)[rg * W4 + cq] = col;
  __syncthreads();
  const float invH = 1.0f / (float)H;
  for (int w = tid; w < W; w += 256) {
    float s = 0.f;
    for (int g = 0; g < NG; ++g) s += cpart[g * W + w];
    o[H + w] = s * invH;
  }
}


// Thin 1x1 convolution (stride 1, groups 1) with the epilogue fused: out = act(W x + b) (+ res), optional packed
// second store of channels [c2lo, M). For the backbone's large-HW, small-channel 1x1 convs (Cout 64 / 128,
// Cin <= 256) the MIOpen path (a GEMM library kernel at low arithmetic intensity + this file's epilogue pass) runs
// far below HBM speed. Here one workgroup owns a 64-pixel column of one image at a time: the x tile [K][64] is staged
// in LDS with float4 loads, the weights sit in registers for the workgroup's whole run of tiles (k-permuted so each
// lane group holds a contiguous k quarter as float4s), and v_mfma_f32_16x16x4_f32 (exact fp32) produces all M
// outputs of the 64 pixels; wave w owns output rows [w*M/4, (w+1)*M/4).
// STATS: also the per-(plane, tile) sum and max of out in tsum/tmax[(b*M + row)*ntile + tile] (a following SE /
// CBAM gate's statistics, reduced per plane by thin_stats_reduce_kernel).
template <int M, int K, bool RES, bool DUAL, bool STATS = false>
__global__ __launch_bounds__(256, 2) void conv1x1_thin_kernel(const float* __restrict__ x, long x_bs,
                                                              const float* __restrict__ w,
                                                              const float* __restrict__ bias, float* __restrict__ out,
                                                              long o_bs, const float* __restrict__ res, long r_bs,
                                                              float* __restrict__ out2, long o2_bs, int c2lo, int HW,
                                                              int ntile, int rev, float* __restrict__ tsum = nullptr,
                                                              float* __restrict__ tmax = nullptr,
                                                              const float* __restrict__ x2 = nullptr, long x2_bs = 0,
                                                              int k1 = K) {
  constexpr int RB = M / 64;   // 16-row blocks per wave
  constexpr int KQ = K / 4;    // k quarter per lane group
  constexpr int XS = 68;       // LDS row stride (floats)
  __shared__ __attribute__((aligned(16))) float xs[K * XS];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l15 = lane & 15, g = lane >> 4;
  const int b = rev ? gridDim.y - 1 - blockIdx.y : blockIdx.y;  // last images first: see mall_reverse()
  const float* xb = x + (long)b * x_bs;
  // a virtual concat: channels [k1, K) come from x2 (image b at x2 + b x2_bs)
  const float* xb2 = x2 ? x2 + (long)b * x2_bs - (long)k1 * HW : xb;
  float4 a[RB][KQ / 4];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const float* wr = w + (long)(wid * (M / 4) + rb * 16 + l15) * K + g * KQ;
#pragma unroll
    for (int t = 0; t < KQ / 4; ++t) a[rb][t] = *reinterpret_cast<const float4*>(wr + 4 * t);
  }
  float bv[RB][4];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[rb][r] = bias[wid * (M / 4) + rb * 16 + 4 * g + r];
  for (int tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
    const int p0 = tile * 64;
    __syncthreads();  // the previous tile's readers are done with xs
#pragma unroll 4
    for (int e = tid; e < K * 16; e += 256) {
      const int row = e >> 4, c4 = e & 15;
      *reinterpret_cast<float4*>(xs + row * XS + 4 * c4) =
          *reinterpret_cast<const float4*>((row < k1 ? xb : xb2) + (long)row * HW + p0 + 4 * c4);
    }
    __syncthreads();
    f32x4 acc[RB][4];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int pb = 0; pb < 4; ++pb) acc[rb][pb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t4 = 0; t4 < KQ / 4; ++t4)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float* xr = xs + (g * KQ + 4 * t4 + c) * XS + l15;
        float bx[4];
#pragma unroll
        for (int pb = 0; pb < 4; ++pb) bx[pb] = xr[16 * pb];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
          const float av = c == 0 ? a[rb][t4].x : c == 1 ? a[rb][t4].y : c == 2 ? a[rb][t4].z : a[rb][t4].w;
#pragma unroll
          for (int pb = 0; pb < 4; ++pb) acc[rb][pb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bx[pb], acc[rb][pb], 0, 0, 0);
        }
      }
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wid * (M / 4) + rb * 16 + 4 * g + r;
        float ts = 0.f, tm = -INFINITY;
#pragma unroll
        for (int pb = 0; pb < 4; ++pb) {
          const int p = p0 + pb * 16 + l15;
          float v = siluf_(acc[rb][pb][r] + bv[rb][r]);
          if (RES) v += res[(long)b * r_bs + (long)row * HW + p];
          out[(long)b * o_bs + (long)row * HW + p] = v;
          if (DUAL && row >= c2lo) out2[(long)b * o2_bs + (long)(row - c2lo) * HW + p] = v;
          if (STATS) {
            ts += v;
            tm = fmaxf(tm, v);
          }
        }
        if (STATS) {
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) {  // the 16 lanes of this lane group hold the row's 64 pixels
            ts += __shfl_xor(ts, o, 64);
            tm = fmaxf(tm, __shfl_xor(tm, o, 64));
          }
          if (l15 == 0) {
            const long ti = ((long)b * M + row) * ntile + tile;
            tsum[ti] = ts;
            tmax[ti] = tm;
          }
        }
      }
  }
}

// Per-plane totals of the thin kernel's tile partials, in the (psum, pmax)[plane*parts + k] layout the SE / CBAM
// *_forward_pre gates read: k = 0 holds the plane's sum / max, k > 0 hold 0 / -inf (the gate sums / maxes over k).
// One wave per plane, fixed order: deterministic and independent of the batch size.
__global__ __launch_bounds__(256) void thin_stats_reduce_kernel(const float* __restrict__ tsum,
                                                                const float* __restrict__ tmax, long planes, int ntile,
                                                                int parts, float* __restrict__ psum,
                                                                float* __restrict__ pmax) {
  const long plane = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (plane >= planes) return;
  float s = 0.f, m = -INFINITY;
  for (int t = lane; t < ntile; t += 64) {
    s += tsum[plane * ntile + t];
    m = fmaxf(m, tmax[plane * ntile + t]);
  }
  s = wave_sum(s);
  m = wave_max(m);
  for (int k = lane; k < parts; k += 64) {
    psum[plane * parts + k] = k == 0 ? s : 0.f;
    if (pmax) pmax[plane * parts + k] = k == 0 ? m : -INFINITY;
  }
}

// Nearest 2x upsample (nn.Upsample(scale_factor=2, mode='nearest'), conv.py / tasks.py neck rows) straight into a
// channel slice of the Concat buffer (batch stride ob). A thread takes 4 consecutive pixels of one input row (one 16 /
// 8-byte load) and writes them doubled to output rows 2i and 2i + 1 (two 32 / 16-byte row chunks, 16-byte stores):
// the strided 6-D copy PyTorch runs for it streams at ~3.3 TB/s. Pure data movement: E is the element's bit pattern
// (uint32_t for fp32, uint16_t for bf16). Requires w % 4 == 0 and 16-byte aligned x / out / strides (host checks).
template <class E>
__global__ __launch_bounds__(256) void upsample2x_kernel(const E* __restrict__ x, E* __restrict__ out, long ob, int C,
                                                         int h, int w, long quads) {
  const int wq = w >> 2;
  for (long q = (long)blockIdx.x * 256 + threadIdx.x; q < quads; q += (long)gridDim.x * 256) {
    const long row = q / wq;  // (b, c, i)
    const int j = (int)(q - row * wq) * 4;
    const long plane = row / h;
    const int i = (int)(row - plane * h);
    const int b = (int)(plane / C), c = (int)(plane - (long)b * C);
    E* o = out + (long)b * ob + ((long)c * 2 * h + 2 * i) * (2L * w) + 2 * j;
    if (sizeof(E) == 4) {
      const uint4 v = *reinterpret_cast<const uint4*>(x + row * w + j);
      const uint4 lo = make_uint4(v.x, v.x, v.y, v.y), hi = make_uint4(v.z, v.z, v.w, v.w);
      uint4* o0 = reinterpret_cast<uint4*>(o);
      uint4* o1 = reinterpret_cast<uint4*>(o + 2L * w);
      o0[0] = lo; o0[1] = hi; o1[0] = lo; o1[1] = hi;
    } else {
      const uint2 v = *reinterpret_cast<const uint2*>(x + row * w + j);
      const uint32_t e0 = v.x & 0xffffu, e1 = v.x >> 16, e2 = v.y & 0xffffu, e3 = v.y >> 16;
      const uint4 d = make_uint4(e0 | (e0 << 16), e1 | (e1 << 16), e2 | (e2 << 16), e3 | (e3 << 16));
      *reinterpret_cast<uint4*>(o) = d;
      *reinterpret_cast<uint4*>(o + 2L * w) = d;
    }
  }
}

}  // namespace ys

using namespace ys;

// x [B, C, h, w] contiguous -> out [B, C, 2h, 2w] with batch stride out_bstride (elements); elem_bytes 4 (fp32) or 2
// (bf16). Returns 0, or a negative code when the shape / alignment is not handled (the caller keeps its copy).
YS_EXPORT int yolosod_upsample2x(const void* x, void* out, long out_bstride, int B, int C, int h, int w, int elem_bytes,
                                 void* stream) {
  YS_CHECK_ARG(x && out, "upsample2x: null pointer");
  YS_CHECK_ARG(B >= 0 && C > 0 && h > 0 && w > 0 && (elem_bytes == 4 || elem_bytes == 2), "upsample2x: bad shape");
  YS_CHECK_ARG(w % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)out & 15) == 0 &&
                   (out_bstride * elem_bytes) % 16 == 0 && (4L * h * w * elem_bytes) % 16 == 0 &&
                   out_bstride >= 4L * C * h * w,
               "upsample2x: w %% 4, 16-byte alignment and a batch stride >= C*4*h*w required");
  if (B == 0) return 0;
  const long quads = (long)B * C * h * (w / 4);
  const unsigned grid = (unsigned)((quads + 255) / 256 < 8192 ? (quads + 255) / 256 : 8192);
  hipStream_t st = (hipStream_t)stream;
  if (elem_bytes == 4)
    hipLaunchKernelGGL(upsample2x_kernel<uint32_t>, dim3(grid), dim3(256), 0, st, (const uint32_t*)x, (uint32_t*)out,
                       out_bstride, C, h, w, quads);
  else
    hipLaunchKernelGGL(upsample2x_kernel<uint16_t>, dim3(grid), dim3(256), 0, st, (const uint16_t*)x, (uint16_t*)out,
                       out_bstride, C, h, w, quads);
  YS_CHECK_LAUNCH("upsample2x");
  return 0;
}

template <class T>
static int bias_act_stats_impl(const T* y, long y_bstride, T* out, long out_bstride, const float* bias, const T* res,
                               long res_bstride, int B, int C, long HW, int act, int parts, long seg, float* psum,
                               float* pmax, void* stream) {
  YS_CHECK_ARG(y && out && bias && psum, "bias_act_stats: null pointer");
  YS_CHECK_ARG(act == 0 || act == 1, "bias_act_stats: act=%d unsupported", act);
  YS_CHECK_ARG(HW % 4 == 0 && seg % 4 == 0 && y_bstride % 4 == 0 && out_bstride % 4 == 0 &&
                   (!res || res_bstride % 4 == 0),
               "bias_act_stats: HW, seg and batch strides must be multiples of 4");
  YS_CHECK_ARG(parts >= 1 && seg >= 1 && (long)parts * seg >= HW && (long)(parts - 1) * seg < HW,
               "bias_act_stats: plane plan (%d x %ld) does not cover HW=%ld", parts, seg, HW);
  YS_CHECK_ARG((((uintptr_t)y | (uintptr_t)out | (uintptr_t)(res ? res : y)) & (4 * sizeof(T) - 1)) == 0,
               "bias_act_stats: pointers must be aligned to 4 elements");
  const long blocks = (long)B * C * parts;
  if (blocks == 0) return 0;
  YS_CHECK_ARG(blocks < (1L << 31), "bias_act_stats: too many planes");
  hipStream_t st = (hipStream_t)stream;
  // bf16: 8 elements per 16-byte access when the plane plan and the strides allow it
  const bool v8 = sizeof(T) == 2 && HW % 8 == 0 && seg % 8 == 0 && y_bstride % 8 == 0 && out_bstride % 8 == 0 &&
                  (!res || res_bstride % 8 == 0) && (((uintptr_t)y | (uintptr_t)out | (uintptr_t)(res ? res : y)) & 15) == 0;
#define YS_BAS(A_, R_, M_)                                                                                         \
  do {                                                                                                             \
    if (v8)                                                                                                        \
      hipLaunchKernelGGL((bias_act_stats_kernel<A_, R_, M_, T, true>), dim3((unsigned)blocks), dim3(256), 0, st, y, \
                         out, bias, res, C, HW, y_bstride, out_bstride, res_bstride, parts, seg, psum, pmax,       \
                         mall_reverse());                                                                          \
    else                                                                                                           \
      hipLaunchKernelGGL((bias_act_stats_kernel<A_, R_, M_, T>), dim3((unsigned)blocks), dim3(256), 0, st, y, out,  \
                         bias, res, C, HW, y_bstride, out_bstride, res_bstride, parts, seg, psum, pmax,            \
                         mall_reverse());                                                                          \
  } while (0)
  const bool mx = pmax != nullptr;
  if (act == 1) {
    if (res) { if (mx) YS_BAS(1, true, true); else YS_BAS(1, true, false); }
    else { if (mx) YS_BAS(1, false, true); else YS_BAS(1, false, false); }
  } else {
    if (res) { if (mx) YS_BAS(0, true, true); else YS_BAS(0, true, false); }
    else { if (mx) YS_BAS(0, false, true); else YS_BAS(0, false, false); }
  }
#undef YS_BAS
  YS_CHECK_LAUNCH("bias_act_stats");
  return 0;
}

// out = act(y + bias[c]) (+ res), optionally also channels [c2lo, C) packed into out2 (out2 == NULL: no copy)
template <class T>
static int bias_act_impl(const T* y, long y_bstride, T* out, long out_bstride, const float* bias, const T* res,
                         long res_bstride, T* out2, long out2_bstride, int c2lo, int B, int C, long HW, int act,
                         void* stream) {
  YS_CHECK_ARG(y && out && bias, "bias_act: null pointer");
  YS_CHECK_ARG(act == 0 || act == 1, "bias_act: act=%d unsupported", act);
  YS_CHECK_ARG(!out2 || (c2lo >= 0 && c2lo < C), "bias_act_dual: c2lo=%d outside [0, C=%d)", c2lo, C);
  YS_CHECK_ARG(HW % 4 == 0 && y_bstride % 4 == 0 && out_bstride % 4 == 0 && (!res || res_bstride % 4 == 0) &&
                   (!out2 || out2_bstride % 4 == 0),
               "bias_act: HW and batch strides must be multiples of 4");
  YS_CHECK_ARG((((uintptr_t)y | (uintptr_t)out | (uintptr_t)(res ? res : y) | (uintptr_t)(out2 ? out2 : y)) &
                (4 * sizeof(T) - 1)) == 0,
               "bias_act: pointers must be aligned to 4 elements");
  const long total4 = (long)B * C * (HW / 4);
  if (total4 == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if constexpr (sizeof(T) == 2) {
    if (HW % 8 == 0 && y_bstride % 8 == 0 && out_bstride % 8 == 0 && (!res || res_bstride % 8 == 0) &&
        (!out2 || out2_bstride % 8 == 0) &&
        (((uintptr_t)y | (uintptr_t)out | (uintptr_t)(res ? res : y) | (uintptr_t)(out2 ? out2 : y)) & 15) == 0) {
      const long total8 = total4 / 2;
      long b8 = (total8 + 255) / 256;
      if (b8 > 8192) b8 = 8192;
      const long hw8 = HW / 8, yb8 = y_bstride / 8, ob8 = out_bstride / 8, rb8 = res_bstride / 8, o28 = out2_bstride / 8;
#define YS_BA8(A_, R_, D_)                                                                                              \
  hipLaunchKernelGGL((bias_act8_bf16_kernel<A_, R_, D_>), dim3(b8), dim3(256), 0, st, y, out, bias, res, C, hw8, yb8, ob8, \
                     rb8, total8, mall_reverse(), out2, c2lo, o28)
      if (out2) {
        if (act == 1) { if (res) YS_BA8(1, true, true); else YS_BA8(1, false, true); }
        else { if (res) YS_BA8(0, true, true); else YS_BA8(0, false, true); }
      } else {
        if (act == 1) { if (res) YS_BA8(1, true, false); else YS_BA8(1, false, false); }
        else { if (res) YS_BA8(0, true, false); else YS_BA8(0, false, false); }
      }
#undef YS_BA8
      YS_CHECK_LAUNCH("bias_act8_bf16");
      return 0;
    }
  }
  long blocks = (total4 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  const long hw4 = HW / 4, yb = y_bstride / 4, ob = out_bstride / 4, rb = res_bstride / 4, o2 = out2_bstride / 4;
#define YS_BA(A_, R_, D_)                                                                                          \
  hipLaunchKernelGGL((bias_act_kernel<A_, R_, D_, T>), dim3(blocks), dim3(256), 0, st, y, out, bias, res, C, hw4, yb, \
                     ob, rb, total4, mall_reverse(), out2, c2lo, o2)
  if (out2) {
    if (act == 1) { if (res) YS_BA(1, true, true); else YS_BA(1, false, true); }
    else { if (res) YS_BA(0, true, true); else YS_BA(0, false, true); }
  } else {
    if (act == 1) { if (res) YS_BA(1, true, false); else YS_BA(1, false, false); }
    else { if (res) YS_BA(0, true, false); else YS_BA(0, false, false); }
  }
#undef YS_BA
  YS_CHECK_LAUNCH("bias_act");
  return 0;
}

template <class T>
static int bias_act_capool_impl(const T* y, long y_bstride, T* out, long out_bstride, const float* bias, const T* res,
                                long res_bstride, int B, int C, int H, int W, int act, float* yin, void* stream) {
  YS_CHECK_ARG(y && out && bias && yin, "bias_act_capool: null pointer");
  YS_CHECK_ARG(act == 0 || act == 1, "bias_act_capool: act=%d unsupported", act);
  YS_CHECK_ARG(B >= 0 && C > 0 && H > 0 && W > 0 && W % 4 == 0 && W <= 1024,
               "bias_act_capool: W=%d must be a multiple of 4 and <= 1024", W);
  YS_CHECK_ARG(y_bstride % 4 == 0 && out_bstride % 4 == 0 && (!res || res_bstride % 4 == 0),
               "bias_act_capool: batch strides must be multiples of 4");
  YS_CHECK_ARG((((uintptr_t)y | (uintptr_t)out | (uintptr_t)(res ? res : y)) & (4 * sizeof(T) - 1)) == 0,
               "bias_act_capool: pointers must be aligned to 4 elements");
  const long planes = (long)B * C;
  if (planes == 0) return 0;
  YS_CHECK_ARG(planes < (1L << 31), "bias_act_capool: too many planes");
  int RB = 8192 / W;
  if (RB < 1) RB = 1;
  if (RB > H) RB = H;
  const size_t lds = sizeof(float) * ((size_t)RB * W + (size_t)(256 / (W / 4)) * W);
  hipStream_t st = (hipStream_t)stream;
#define YS_BAC(A_, R_)                                                                                               \
  hipLaunchKernelGGL((bias_act_capool_kernel<A_, R_, T>), dim3((unsigned)planes), dim3(256), lds, st, y, out, bias, \
                     res, C, H, W, RB, y_bstride, out_bstride, res_bstride, yin)
  if (act == 1) { if (res) YS_BAC(1, true); else YS_BAC(1, false); }
  else { if (res) YS_BAC(0, true); else YS_BAC(0, false); }
#undef YS_BAC
  YS_CHECK_LAUNCH("bias_act_capool");
  return 0;
}

// yolosod_bias_act + per-plane partial sums (and maxes when pmax != NULL) of `out` in psum/pmax[B*C*parts], with
// the plane segmentation (parts, seg) that yolosod_se_forward_pre / yolosod_cbam_forward_pre expect
// (yolosod_plane_parts). Requires HW % 4 == 0 and seg % 4 == 0.
YS_EXPORT int yolosod_bias_act_stats(const float* y, long y_bstride, float* out, long out_bstride, const float* bias,
                                     const float* res, long res_bstride, int B, int C, long HW, int act, int parts,
                                     long seg, float* psum, float* pmax, void* stream) {
  return bias_act_stats_impl(y, y_bstride, out, out_bstride, bias, res, res_bstride, B, C, HW, act, parts, seg, psum,
                             pmax, stream);
}

// out[b*out_bstride + c*HW + p] = act(y[b*y_bstride + c*HW + p] + bias[c]) + res[b*res_bstride + c*HW + p]
// act: 0 identity, 1 SiLU. res may be NULL. In place (out == y) allowed. HW and all strides multiples of 4.
YS_EXPORT int yolosod_bias_act(const float* y, long y_bstride, float* out, long out_bstride, const float* bias,
                               const float* res, long res_bstride, int B, int C, long HW, int act, void* stream) {
  return bias_act_impl(y, y_bstride, out, out_bstride, bias, res, res_bstride, (float*)nullptr, 0L, 0, B, C, HW, act,
                       stream);
}

// yolosod_bias_act that also writes channels [c2lo, C) of the result to out2 ([B, C - c2lo, HW], batch stride
// out2_bstride). C2f feeds its Bottleneck chain from channel slices of the concat buffer; MIOpen needs packed
// inputs, so without this every Bottleneck input was re-read and re-written by a copy kernel.
YS_EXPORT int yolosod_bias_act_dual(const float* y, long y_bstride, float* out, long out_bstride, const float* bias,
                                    const float* res, long res_bstride, float* out2, long out2_bstride, int c2lo,
                                    int B, int C, long HW, int act, void* stream) {
  YS_CHECK_ARG(out2, "bias_act_dual: null pointer");
  return bias_act_impl(y, y_bstride, out, out_bstride, bias, res, res_bstride, out2, out2_bstride, c2lo, B, C, HW, act,
                       stream);
}

// yolosod_bias_act + the CA_Block pooling of `out` (row means over W, then column means over H, per plane) into
// yin[B*C*(H+W)], the layout yolosod_ca_forward_pre takes. Requires W % 4 == 0, W <= 1024 and 4-aligned strides.
YS_EXPORT int yolosod_bias_act_capool(const float* y, long y_bstride, float* out, long out_bstride, const float* bias,
                                      const float* res, long res_bstride, int B, int C, int H, int W, int act,
                                      float* yin, void* stream) {
  return bias_act_capool_impl(y, y_bstride, out, out_bstride, bias, res, res_bstride, B, C, H, W, act, yin, stream);
}

// bf16 storage variants of the three epilogues (y / out / res / out2: bf16 bit patterns; bias, statistics fp32).
// mode 0: plain (out2 optional, NULL = none); statistics in the *_stats / *_capool entry points. The statistics are
// of the stored (bf16-rounded) values.
YS_EXPORT int yolosod_bias_act_bf16(const bf16_t* y, long y_bstride, bf16_t* out, long out_bstride, const float* bias,
                                    const bf16_t* res, long res_bstride, bf16_t* out2, long out2_bstride, int c2lo,
                                    int B, int C, long HW, int act, void* stream) {
  return bias_act_impl(y, y_bstride, out, out_bstride, bias, res, res_bstride, out2, out2_bstride, c2lo, B, C, HW, act,
                       stream);
}
YS_EXPORT int yolosod_bias_act_stats_bf16(const bf16_t* y, long y_bstride, bf16_t* out, long out_bstride,
                                          const float* bias, const bf16_t* res, long res_bstride, int B, int C,
                                          long HW, int act, int parts, long seg, float* psum, float* pmax,
                                          void* stream) {
  return bias_act_stats_impl(y, y_bstride, out, out_bstride, bias, res, res_bstride, B, C, HW, act, parts, seg, psum,
                             pmax, stream);
}
YS_EXPORT int yolosod_bias_act_capool_bf16(const bf16_t* y, long y_bstride, bf16_t* out, long out_bstride,
                                           const float* bias, const bf16_t* res, long res_bstride, int B, int C, int H,
                                           int W, int act, float* yin, void* stream) {
  return bias_act_capool_impl(y, y_bstride, out, out_bstride, bias, res, res_bstride, B, C, H, W, act, yin, stream);
}

// Thin fused 1x1 conv (+ bias + SiLU (+ res)) for Cout in {64, 128}, Cin in {64, 96, 128, 192, 256}, HW % 64 == 0,
// 16-byte aligned pointers and 4-aligned batch strides; x / out / res / out2 may be channel slices (batch strides).
// out2 (optional): packed copy of channels [c2lo, Cout). Returns a non-zero code (no launch) for other shapes.
YS_EXPORT int yolosod_conv1x1_thin(const float* x, long x_bs, const float* w, const float* bias, float* out, long out_bs,
                                   const float* res, long res_bs, float* out2, long out2_bs, int c2lo, int B, int Cin,
                                   int Cout, long HW, void* stream) {
  YS_CHECK_ARG(x && w && bias && out, "conv1x1_thin: null pointer");
  YS_CHECK_ARG(HW % 64 == 0 && HW < (1L << 30), "conv1x1_thin: HW=%ld must be a multiple of 64", HW);
  YS_CHECK_ARG(Cout == 64 || Cout == 128, "conv1x1_thin: Cout=%d unsupported", Cout);
  YS_CHECK_ARG(x_bs % 4 == 0 && out_bs % 4 == 0 && (!res || res_bs % 4 == 0) && (!out2 || out2_bs % 4 == 0),
               "conv1x1_thin: batch strides must be multiples of 4");
  YS_CHECK_ARG((((uintptr_t)x | (uintptr_t)w | (uintptr_t)out) & 15) == 0, "conv1x1_thin: pointers must be 16-byte aligned");
  YS_CHECK_ARG(!out2 || (c2lo >= 0 && c2lo < Cout), "conv1x1_thin: c2lo=%d", c2lo);
  if (B == 0) return 0;
  const int ntile = (int)(HW / 64);
  const int gx = ntile < 4 ? ntile : (ntile + 3) / 4;  // ~4 tiles per workgroup: weights loaded once per run
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)gx, (unsigned)B);
  bool ok = false;
#define YS_THIN(M_, K_)                                                                                            \
  if (Cout == M_ && Cin == K_) {                                                                                   \
    ok = true;                                                                                                     \
    if (res && out2) hipLaunchKernelGGL((conv1x1_thin_kernel<M_, K_, true, true>), grid, dim3(256), 0, st, x, x_bs, w, bias, out, out_bs, res, res_bs, out2, out2_bs, c2lo, (int)HW, ntile, mall_reverse()); \
    else if (res) hipLaunchKernelGGL((conv1x1_thin_kernel<M_, K_, true, false>), grid, dim3(256), 0, st, x, x_bs, w, bias, out, out_bs, res, res_bs, out2, out2_bs, c2lo, (int)HW, ntile, mall_reverse()); \
    else if (out2) hipLaunchKernelGGL((conv1x1_thin_kernel<M_, K_, false, true>), grid, dim3(256), 0, st, x, x_bs, w, bias, out, out_bs, res, res_bs, out2, out2_bs, c2lo, (int)HW, ntile, mall_reverse()); \
    else hipLaunchKernelGGL((conv1x1_thin_kernel<M_, K_, false, false>), grid, dim3(256), 0, st, x, x_bs, w, bias, out, out_bs, res, res_bs, out2, out2_bs, c2lo, (int)HW, ntile, mall_reverse()); \
  }
  YS_THIN(64, 64) YS_THIN(64, 96) YS_THIN(64, 128) YS_THIN(64, 192) YS_THIN(64, 256)
  YS_THIN(128, 64) YS_THIN(128, 96) YS_THIN(128, 128) YS_THIN(128, 192) YS_THIN(128, 256)
#undef YS_THIN
  YS_CHECK_ARG(ok, "conv1x1_thin: Cin=%d unsupported", Cin);
  YS_CHECK_LAUNCH("conv1x1_thin");
  return 0;
}

// yolosod_conv1x1_thin over a virtual concat [x; x2] (channels [0, k1) from x, [k1, Cin) from x2), no residual /
// statistics: the C2f cv1 after a neck Concat reads both parts in place instead of a materialised concat.
YS_EXPORT int yolosod_conv1x1_thin_cat(const float* x, long x_bs, const float* x2, long x2_bs, int k1, const float* w,
                                       const float* bias, float* out, long out_bs, float* out2, long out2_bs, int c2lo,
                                       int B, int Cin, int Cout, long HW, void* stream) {
  YS_CHECK_ARG(x && x2 && w && bias && out, "conv1x1_thin_cat: null pointer");
  YS_CHECK_ARG(k1 > 0 && k1 < Cin, "conv1x1_thin_cat: k1=%d (Cin %d)", k1, Cin);
  YS_CHECK_ARG(HW % 64 == 0 && HW < (1L << 30), "conv1x1_thin_cat: HW=%ld must be a multiple of 64", HW);
  YS_CHECK_ARG(Cout == 64 || Cout == 128, "conv1x1_thin_cat: Cout=%d unsupported", Cout);
  YS_CHECK_ARG(x_bs % 4 == 0 && x2_bs % 4 == 0 && out_bs % 4 == 0 && (!out2 || out2_bs % 4 == 0),
               "conv1x1_thin_cat: batch strides must be multiples of 4");
  YS_CHECK_ARG((((uintptr_t)x | (uintptr_t)x2 | (uintptr_t)w | (uintptr_t)out) & 15) == 0,
               "conv1x1_thin_cat: pointers must be 16-byte aligned");
  YS_CHECK_ARG(!out2 || (c2lo >= 0 && c2lo < Cout), "conv1x1_thin_cat: c2lo=%d", c2lo);
  if (B == 0) return 0;
  const int ntile = (int)(HW / 64);
  const int gx = ntile < 4 ? ntile : (ntile + 3) / 4;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)gx, (unsigned)B);
  bool ok = false;
#define YS_THINC(M_, K_)                                                                                          \
  if (Cout == M_ && Cin == K_) {                                                                                  \
    ok = true;                                                                                                    \
    if (out2) hipLaunchKernelGGL((conv1x1_thin_kernel<M_, K_, false, true>), grid, dim3(256), 0, st, x, x_bs, w,    \
                                 bias, out, out_bs, nullptr, 0L, out2, out2_bs, c2lo, (int)HW, ntile, mall_reverse(), \
                                 nullptr, nullptr, x2, x2_bs, k1);                                                 \
    else hipLaunchKernelGGL((conv1x1_thin_kernel<M_, K_, false, false>), grid, dim3(256), 0, st, x, x_bs, w, bias,  \
                            out, out_bs, nullptr, 0L, nullptr, 0L, 0, (int)HW, ntile, mall_reverse(), nullptr, nullptr, \
                            x2, x2_bs, k1);                                                                        \
  }
  YS_THINC(64, 64) YS_THINC(64, 96) YS_THINC(64, 128) YS_THINC(64, 192) YS_THINC(64, 256)
  YS_THINC(128, 64) YS_THINC(128, 96) YS_THINC(128, 128) YS_THINC(128, 192) YS_THINC(128, 256)
#undef YS_THINC
  YS_CHECK_ARG(ok, "conv1x1_thin_cat: Cin=%d unsupported", Cin);
  YS_CHECK_LAUNCH("conv1x1_thin_cat");
  return 0;
}

// yolosod_conv1x1_thin (no residual / second store) that also emits the output's per-plane statistics for a
// following SE / CBAM gate in the psum / pmax[B*Cout*parts] layout of yolosod_se_forward_pre /
// yolosod_cbam_forward_pre (parts = yolosod_plane_parts(HW)); pmax may be NULL. tile_ws: 2*B*Cout*(HW/64) floats.
YS_EXPORT int yolosod_conv1x1_thin_stats(const float* x, long x_bs, const float* w, const float* bias, float* out,
                                         long out_bs, int B, int Cin, int Cout, long HW, int parts, float* psum,
                                         float* pmax, float* tile_ws, void* stream) {
  YS_CHECK_ARG(x && w && bias && out && psum && tile_ws, "conv1x1_thin_stats: null pointer");
  YS_CHECK_ARG(HW % 64 == 0 && HW < (1L << 30), "conv1x1_thin_stats: HW=%ld must be a multiple of 64", HW);
  YS_CHECK_ARG(Cout == 64 || Cout == 128, "conv1x1_thin_stats: Cout=%d unsupported", Cout);
  YS_CHECK_ARG(parts >= 1, "conv1x1_thin_stats: parts=%d", parts);
  YS_CHECK_ARG(x_bs % 4 == 0 && out_bs % 4 == 0, "conv1x1_thin_stats: batch strides must be multiples of 4");
  YS_CHECK_ARG((((uintptr_t)x | (uintptr_t)w | (uintptr_t)out) & 15) == 0,
               "conv1x1_thin_stats: pointers must be 16-byte aligned");
  if (B == 0) return 0;
  const int ntile = (int)(HW / 64);
  const int gx = ntile < 4 ? ntile : (ntile + 3) / 4;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)gx, (unsigned)B);
  float* tsum = tile_ws;
  float* tmax = tile_ws + (long)B * Cout * ntile;
  bool ok = false;
#define YS_THINS(M_, K_)                                                                                          \
  if (Cout == M_ && Cin == K_) {                                                                                  \
    ok = true;                                                                                                    \
    hipLaunchKernelGGL((conv1x1_thin_kernel<M_, K_, false, false, true>), grid, dim3(256), 0, st, x, x_bs, w, bias, \
                       out, out_bs, nullptr, 0L, nullptr, 0L, 0, (int)HW, ntile, mall_reverse(), tsum, tmax);                   \
  }
  YS_THINS(64, 64) YS_THINS(64, 96) YS_THINS(64, 128) YS_THINS(64, 192) YS_THINS(64, 256)
  YS_THINS(128, 64) YS_THINS(128, 96) YS_THINS(128, 128) YS_THINS(128, 192) YS_THINS(128, 256)
#undef YS_THINS
  YS_CHECK_ARG(ok, "conv1x1_thin_stats: Cin=%d unsupported", Cin);
  const long planes = (long)B * Cout;
  hipLaunchKernelGGL(thin_stats_reduce_kernel, dim3((unsigned)((planes + 3) / 4)), dim3(256), 0, st, tsum, tmax, planes,
                     ntile, parts, psum, pmax);
  YS_CHECK_LAUNCH("conv1x1_thin_stats");
  return 0;
}
