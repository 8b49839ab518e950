// 3x3 convolution (stride 1, pad 1, 64 output channels) + folded BN bias + SiLU as an implicit GEMM on the fp16
// matrix cores at fp32 accuracy: the Detect head's conv towers (ultralytics/nn/modules/head.py:
// 43-57: cv2[i] = Conv(c, c2, 3), Conv(c2, c2, 3); cv3[i] = Conv(c, c3, 3), Conv(c3, c3, 3) with c2 = c3 = 64 for the
// paper model). Each Conv is conv2d (no bias) -> BN (folded into weight / bias by fuse(), torch_utils.py:238-265) ->
// SiLU (conv.py:37-55).
//
// Method (the two-term split of swin_x3.hip): v = h + l with h = fp16(v), l = fp16(v - h); a product is
// ah.bh + ah.bl + al.bh on v_mfma_f32_16x16x32_f16 with fp32 accumulation. Weights are split once per parameter
// version by conv3x3_prep_kernel (x 64, exact, so their low terms stay normal fp16) into fragment-major planes:
// for tap t, 32-channel input chunk q, 16-channel output block rb and plane p, the 64 lanes' fragments (lane (g, l15):
// output channel 16 rb + l15, input channels 32 q + 8 g .. + 7) are 1 KB contiguous.
//
// One 256-thread workgroup per (image, 8 x 32 output tile), all 64 output channels, two workgroups per CU: per input
// chunk, the tile's 10 x 34 input halo (zero padding outside the image) is loaded, split and stored once as two fp16
// planes [pixel][32] in LDS; the nine taps read their pixel fragments (8 channels of one halo pixel per lane) at
// tap-shifted pixel offsets of the same planes, so every input value is split once per workgroup and reused by
// 9 taps x 64 outputs. Wave w computes output rows 4 (w >> 1) .. + 3 (eight 16-pixel blocks) for the output channel
// blocks 2 (w & 1), 2 (w & 1) + 1: 16 accumulator tiles from 4 weight fragments (L2, one tap ahead) and 16 pixel
// fragments (LDS) per tap. The pixels are the MFMA's A operand, so a lane's accumulators are 4 consecutive pixels of
// one channel (16-byte stores). The next chunk's halo loads are spread over the current chunk's taps.
#include "common.h"

namespace ys {
namespace c3 {

constexpr float WSC = 64.0f;
constexpr int TH = 8, TW = 32;              // output tile
constexpr int HH = TH + 2, HW_ = TW + 2;    // halo tile
constexpr int NPXH = HH * HW_;              // 340 halo pixels
constexpr int PS = 48;                       // plane row stride (halves): 96-byte pixel rows, conflict-free ds_read_b128
constexpr int PL = NPXH * PS;               // plane (halves)
constexpr int NQUAD = NPXH * 8;             // staged items per chunk: (4-channel quad, halo pixel)
constexpr int NT = 256;
constexpr int NIT = (NQUAD + NT - 1) / NT;  // 11

struct Args {
  const float* x;      // [B][Cin][H][W]
  const h16_t* wp;     // prepared planes (fragment-major, x 64)
  const float* bias;   // [Cout]
  float* y;            // image b's output [Cout][H][W] at y + b ybs (a channel slice of a concat buffer when
  long ybs;            // ybs > Cout H W)
  const float* res;    // RES: residual added after the activation (Bottleneck shortcut), image b at res + b rbs
  long rbs;
  int cin, H, W, tiles_x, tiles_y;
  int ncb_all;         // 16-channel blocks of the prepared weights (Cout / 16)
  unsigned* range_flag;
  const unsigned* prep_flag;
  int ntiles;          // persistent kernel: B tiles_y tiles_x
  long xbs;            // image b of x at x + b xbs (>= cin H W: x may be a channel slice of a concat buffer)
};

// ABL (timing ablations, wrong results; yolosod_debug_set_conv3x3_abl): 1 no halo loads, 2 every weight fragment from
// one address, 4 no MFMA (a VALU stand-in keeps the LDS reads), 8 no output stores. V4: W % 4 == 0 (16-byte stores).
// CBW: 16-channel blocks per wave (2: output groups of 64 channels; 1: of 32, the neck's C2f at P2), the workgroup's
// group = blockIdx % groups (the groups of a tile run side by side and share its input in L2). RES: + residual.
template <int ABL, bool V4, int CBW = 2, bool RES = false>
__global__ __launch_bounds__(256, 2) void conv3x3_x2_kernel(Args p) {
  __shared__ __attribute__((aligned(16))) h16_t Pl[2 * PL];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, g = lane >> 4;
  const int ngrp = p.ncb_all / (2 * CBW);
  const int grp = blockIdx.x % ngrp;
  const int t_lin = blockIdx.x / ngrp;
  const int tx = t_lin % p.tiles_x, ty = (t_lin / p.tiles_x) % p.tiles_y, b = t_lin / (p.tiles_x * p.tiles_y);
  const int H = p.H, W = p.W, HWi = H * W;
  const int x0 = tx * TW - 1, y0 = ty * TH - 1;  // halo origin
  const int nq = p.cin >> 5;
  const float* xb = p.x + (long)b * p.xbs;
  float rng = 0.f;

  // staging item e: quad = e / NPXH (channels 4 quad .. + 3 of the chunk), halo pixel e % NPXH; consecutive threads
  // take consecutive pixels (coalesced rows). Out-of-image pixels load a clamped in-image address (unconditional
  // loads) and store zeros. Buffer loads: 32-bit per-lane offsets, the channel / chunk offsets in the scalar offset.
  auto rsrc = [&](const void* base, unsigned bytes) {
    const unsigned long long a = (unsigned long long)base;
    return __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(a >> 32)) << 32) |
                (unsigned)__builtin_amdgcn_readfirstlane((unsigned)a)),
        (short)0, __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rx = rsrc(xb, (unsigned)((long)p.cin * HWi * 4));
  // the last chunk's "next chunk" loads go through an empty resource: out of range, they return 0 without a memory
  // access (the loads stay unconditional) and no residual / epilogue wait queues behind a needless reload
  const __amdgpu_buffer_rsrc_t rx0 = rsrc(xb, 0u);
  const __amdgpu_buffer_rsrc_t rw = rsrc(p.wp, (unsigned)(9L * nq * p.ncb_all * 2 * 1024));
  unsigned voff[NIT];
  bool okp[NIT];
#pragma unroll
  for (int i = 0; i < NIT; ++i) {
    const int e = min(tid + NT * i, NQUAD - 1);
    const int quad = e / NPXH, px = e - quad * NPXH;
    const int hy = px / HW_, hx = px - hy * HW_;
    const int yy = y0 + hy, xx = x0 + hx;
    okp[i] = yy >= 0 && yy < H && xx >= 0 && xx < W;
    voff[i] = (unsigned)(((4 * quad) * HWi + min(max(yy, 0), H - 1) * W + min(max(xx, 0), W - 1)) * 4);
  }
  f32x4 sv[NIT];
  // loads k = 4 i + c in [k0, k1) of chunk q's staging (item i, channel c of its quad)
  auto load_part = [&](int q, int k0, int k1, bool live) __attribute__((always_inline)) {
    const int sx = __builtin_amdgcn_readfirstlane(32 * q * HWi * 4);
    const __amdgpu_buffer_rsrc_t r = live ? rx : rx0;
#pragma unroll
    for (int k = 0; k < 4 * NIT; ++k)
      if (k >= k0 && k < k1) {
        if constexpr ((ABL & 1) != 0)
          sv[k >> 2][k & 3] = 0.5f + (float)q;
        else
          sv[k >> 2][k & 3] = __builtin_bit_cast(
              float, __builtin_amdgcn_raw_buffer_load_b32(r, voff[k >> 2], sx + (k & 3) * HWi * 4, 0));
      }
  };
  auto store_chunk = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int e = tid + NT * i;
      if (e < NQUAD) {
        const int quad = e / NPXH, px = e - quad * NPXH;
        const f32x4 v = okp[i] ? sv[i] : f32x4{0.f, 0.f, 0.f, 0.f};
        uint2 hh, ll;
        split4x(v, hh, ll);
        rng = range_acc(rng, v);
        h16_t* d = Pl + px * PS + 4 * quad;
        *reinterpret_cast<uint2*>(d) = hh;
        *reinterpret_cast<uint2*>(d + PL) = ll;
      }
    }
  };
  // this wave: output channels 32 rp .. + 31 (weight row blocks 2 rp + r), pixel rows 4 ph .. 4 ph + 3 (pixel blocks
  // cb: row 4 ph + (cb >> 1), columns (cb & 1) 16 .. + 15). The pixels are the MFMA's A operand (lane (g, l15) of a
  // fragment: pixel l15 of the block, channels 8 g .. + 7 of the chunk) and the weights its B operand, so the lane
  // holds 4 consecutive pixels (4 g .. + 3) of one output channel (l15): 16-byte output stores
  const int rp = wid & 1, ph = wid >> 1;
  int bpx[8];
#pragma unroll
  for (int cb = 0; cb < 8; ++cb) bpx[cb] = (4 * ph + (cb >> 1)) * HW_ + (cb & 1) * 16 + l15;
  // weight fragments of (tap t, chunk q): channel blocks cbw0 + r (r < CBW), planes 0 / 1; tap t's fragments of chunk
  // q start at byte ((t nq + q) ncb_all 2) KB, [channel block][plane][lane][16 bytes] (B-operand lane layout = A's)
  const int cbw0 = grp * 2 * CBW + CBW * rp;
  auto wfrag = [&](int t, int q, int r, int pl) __attribute__((always_inline)) {
    const int st = (ABL & 2) ? 0 : __builtin_amdgcn_readfirstlane(((t * nq + q) * p.ncb_all * 2) * 1024);
    return __builtin_bit_cast(f16x8_t, __builtin_amdgcn_raw_buffer_load_b128(
                                           rw, (unsigned)((((cbw0 + r) * 2 + pl) * 64 + lane) * 16), st, 0));
  };
  f32x4 acc[CBW][8];
#pragma unroll
  for (int r = 0; r < CBW; ++r)
#pragma unroll
    for (int cb = 0; cb < 8; ++cb) acc[r][cb] = f32x4{0.f, 0.f, 0.f, 0.f};

  load_part(0, 0, 4 * NIT, true);
  for (int q = 0; q < nq; ++q) {
    __syncthreads();  // every wave is done with the previous chunk's planes
    store_chunk();
    __syncthreads();
    // The next chunk's staging loads are spread over the nine taps, each part issued behind the next tap's weight
    // fragments, and sched barriers keep every prefetch where it is: vmcnt counts in issue order, so a wait for a
    // tap's weights also waits for every halo load issued before them (all 44 at once: the HBM latency at tap 0 of
    // every chunk), and without the barriers the scheduler sinks the loads to their first use (next chunk's staging,
    // next tap) to save registers. Unconditional: the last chunk reloads itself (loads under a branch merge into phis
    // whose copies wait for every load in flight).
    const int qn = q + 1 < nq ? q + 1 : q;
    const bool nlive = q + 1 < nq;
    f16x8_t wa[CBW][2], wn[CBW][2];
#pragma unroll
    for (int r = 0; r < CBW; ++r) {
      wa[r][0] = wfrag(0, q, r, 0);
      wa[r][1] = wfrag(0, q, r, 1);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int tn = t + 1 < 9 ? t + 1 : t;  // one tap ahead (unconditional)
#pragma unroll
      for (int r = 0; r < CBW; ++r) {
        wn[r][0] = wfrag(tn, q, r, 0);
        wn[r][1] = wfrag(tn, q, r, 1);
      }
      load_part(qn, 5 * t, t == 8 ? 4 * NIT : 5 * t + 5, nlive);
      __builtin_amdgcn_sched_barrier(0);
      const int toff = (t / 3) * HW_ + (t % 3);
#pragma unroll
      for (int cb = 0; cb < 8; ++cb) {
        const h16_t* src = Pl + (bpx[cb] + toff) * PS + 8 * g;
        const f16x8_t xh = *reinterpret_cast<const f16x8_t*>(src);
        const f16x8_t xlo = *reinterpret_cast<const f16x8_t*>(src + PL);
#pragma unroll
        for (int r = 0; r < CBW; ++r) {
          if constexpr ((ABL & 4) != 0) {
            acc[r][cb][0] += (float)xh[0] * (float)wa[r][0][0] + (float)xlo[1] * (float)wa[r][1][1];
          } else {  // the three split products, small terms first
            f32x4 c = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh, wa[r][1], acc[r][cb], 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_f16(xlo, wa[r][0], c, 0, 0, 0);
            acc[r][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh, wa[r][0], c, 0, 0, 0);
          }
        }
      }
#pragma unroll
      for (int r = 0; r < CBW; ++r) {
        wa[r][0] = wn[r][0];
        wa[r][1] = wn[r][1];
      }
    }
  }
  // epilogue: lane (g, l15) of (r, cb) holds output channel 16 (2 rp + r) + l15, pixels (row 4 ph + (cb >> 1),
  // columns (cb & 1) 16 + 4 g .. + 3) of the tile. SiLU on the hardware exp2 / rcp (~2^-22 relative, below the split
  // products' own few-ulp error)
  float* yb = p.y + (long)b * p.ybs;
  float bv[CBW];
#pragma unroll
  for (int r = 0; r < CBW; ++r) bv[r] = p.bias[16 * (cbw0 + r) + l15];
#pragma unroll
  for (int cb = 0; cb < 8; ++cb) {
    const int oy = ty * TH + 4 * ph + (cb >> 1), ox = tx * TW + (cb & 1) * 16 + 4 * g;
    if constexpr ((ABL & 8) != 0)
      if (acc[0][cb][0] != -1.2345e30f) continue;
#pragma unroll
    for (int r = 0; r < CBW; ++r) {
      const long po = (long)(16 * (cbw0 + r) + l15) * HWi + oy * W + ox;
      float* d = yb + po;
      f32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = silu_fast_(acc[r][cb][j] * (1.0f / WSC) + bv[r]);
      if constexpr (RES) {  // act(conv + b) + x (Bottleneck shortcut, block.py:343); V4 shapes only
#pragma clang fp contract(off)  // a separately rounded add, as x + cv2(...): no fma with SiLU's last multiply
        static_assert(!RES || V4, "residual: W % 4 == 0");
        if (oy < H && ox < W) o = o + *reinterpret_cast<const f32x4*>(p.res + (long)b * p.rbs + po);
      }
      if constexpr (V4) {  // W % 4 == 0: the 4 pixels are all in or all out of the image
        // non-temporal: the tile is not read again before it has left the caches (at P2 the kernel is 13 % faster)
        if (oy < H && ox < W) __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(d));
      } else if (oy < H) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (ox + j < W) d[j] = o[j];
      }
    }
  }
  range_report(p.range_flag, rng);
  if (p.prep_flag && p.range_flag && blockIdx.x == 0 && threadIdx.x == 0 && *p.prep_flag) *p.range_flag = 1u;
}

// Persistent form (W % 4 == 0): the same tile, MFMA and store scheme, but each workgroup walks a contiguous range of
// work items (tile, output group) of its XCD (neighbouring tiles share halo rows in that XCD's L2), one iteration per
// (item, input chunk), and the next iteration's halo loads (the next tile's first chunk included) are spread over the
// current iteration's taps, so no tile starts with an exposed HBM wait. Per-image buffer resources with unclamped
// offsets (rows above the image are negative offsets: out of range, 0); other out-of-image pixels masked by okb.
template <int CBW, bool RES>
__global__ __launch_bounds__(256, 2) void conv3x3_p_kernel(Args p) {
  __shared__ __attribute__((aligned(16))) h16_t Pl[2 * PL];
  __shared__ float bsh[512];  // every output channel's bias: an epilogue load would wait behind the prefetches
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, g = lane >> 4;
  const int H = p.H, W = p.W, HWi = H * W, nq = p.cin >> 5;
  float rng = 0.f;
  for (int o = tid; o < 16 * p.ncb_all; o += 256) bsh[o] = p.bias[o];  // ordered before use by the loop's barriers

  const int ngrp = p.ncb_all / (2 * CBW);
  const int nj = gridDim.x >> 3, j = blockIdx.x >> 3, xcd = blockIdx.x & 7;
  const int nitems = p.ntiles * ngrp;
  const int per = (nitems + 7) >> 3;
  const int t_beg = xcd * per + j, t_end = min((xcd + 1) * per, nitems);
  if (t_beg >= t_end) return;
  const int n_it = ((t_end - t_beg + nj - 1) / nj) * nq;

  auto rsrc = [&](const void* base, unsigned bytes) {
    const unsigned long long a = (unsigned long long)base;
    return __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(a >> 32)) << 32) |
                (unsigned)__builtin_amdgcn_readfirstlane((unsigned)a)),
        (short)0, __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rw = rsrc(p.wp, (unsigned)(9L * nq * p.ncb_all * 2 * 1024));
  int pk[NIT], el0[NIT];
#pragma unroll
  for (int i = 0; i < NIT; ++i) {
    const int e = min(tid + NT * i, NQUAD - 1);
    const int quad = e / NPXH, px = e - quad * NPXH;
    const int hy = px / HW_, hx = px - hy * HW_;
    pk[i] = (quad << 16) | (hy << 8) | hx;
    el0[i] = 4 * quad * HWi + hy * W + hx;
  }
  struct It {
    int b, ty, tx, q, grp;
  };
  auto it_of = [&](int it) __attribute__((always_inline)) {
    const int tg = t_beg + (it / nq) * nj;
    const int t = tg / ngrp;
    It r;
    r.grp = tg - t * ngrp;
    r.q = it - (it / nq) * nq;
    r.tx = t % p.tiles_x;
    r.ty = (t / p.tiles_x) % p.tiles_y;
    r.b = t / (p.tiles_x * p.tiles_y);
    return r;
  };
  f32x4 sv[NIT];
  unsigned okb_ld = 0;
  auto load_part = [&](const It& r, int k0, int k1) __attribute__((always_inline)) {
    const int iy0 = TH * r.ty - 1, ix0 = TW * r.tx - 1;
    const __amdgpu_buffer_rsrc_t ri =
        rsrc(p.x + (long)r.b * p.xbs + (long)32 * r.q * HWi, (unsigned)((p.cin - 32 * r.q) * HWi * 4));
    const int toff = iy0 * W + ix0;
    if (k0 == 0) {
      const bool interior = iy0 >= 0 && ix0 >= 0 && iy0 + HH <= H && ix0 + HW_ <= W;
      unsigned okb = 0xffffffffu;
      if (!interior) {
        okb = 0;
#pragma unroll
        for (int i = 0; i < NIT; ++i) {
          const int hy = (pk[i] >> 8) & 255, hx = pk[i] & 255;
          okb |= ((unsigned)(iy0 + hy) < (unsigned)H && (unsigned)(ix0 + hx) < (unsigned)W) ? (1u << i) : 0u;
        }
      }
      okb_ld = okb;
    }
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      if (4 * i + 3 < k0 || 4 * i >= k1) continue;
      const unsigned vo = (unsigned)((el0[i] + toff) * 4);
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (4 * i + c >= k0 && 4 * i + c < k1)
          sv[i][c] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ri, vo + c * HWi * 4, 0, 0));
    }
  };
  const int rp = wid & 1, ph = wid >> 1;
  int bpx[8];
#pragma unroll
  for (int cb = 0; cb < 8; ++cb) bpx[cb] = (4 * ph + (cb >> 1)) * HW_ + (cb & 1) * 16 + l15;
  auto wfrag = [&](int t, int q, int cbw, int pl) __attribute__((always_inline)) {
    const int st = __builtin_amdgcn_readfirstlane(((t * nq + q) * p.ncb_all * 2) * 1024);
    return __builtin_bit_cast(f16x8_t, __builtin_amdgcn_raw_buffer_load_b128(
                                           rw, (unsigned)(((cbw * 2 + pl) * 64 + lane) * 16), st, 0));
  };
  f32x4 acc[CBW][8];
#pragma unroll
  for (int r = 0; r < CBW; ++r)
#pragma unroll
    for (int cb = 0; cb < 8; ++cb) acc[r][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int NLD = 4 * NIT;             // loads per (tile, chunk): 44
  constexpr int PER_TAP = (NLD + 8) / 9;   // spread over the nine taps

  It cur = it_of(0);
  load_part(cur, 0, NLD);
  for (int it = 0; it < n_it; ++it) {
    const It r = cur;
    const unsigned okb = okb_ld;
    __syncthreads();  // every wave is done with the previous iteration's planes
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int e = tid + NT * i;
      if (e < NQUAD) {
        const int quad = pk[i] >> 16, px = e - quad * NPXH;
        const f32x4 v = ((okb >> i) & 1u) ? sv[i] : f32x4{0.f, 0.f, 0.f, 0.f};
        uint2 hh, ll;
        split4x(v, hh, ll);
        rng = range_acc(rng, v);
        h16_t* d = Pl + px * PS + 4 * quad;
        *reinterpret_cast<uint2*>(d) = hh;
        *reinterpret_cast<uint2*>(d + PL) = ll;
      }
    }
    __syncthreads();
    // the last iteration reloads itself (unconditional loads; L2-hot)
    if (it + 1 < n_it) cur = it_of(it + 1);
    const int cbw0 = r.grp * 2 * CBW + CBW * rp;
    f16x8_t wa[CBW][2], wn[CBW][2];
#pragma unroll
    for (int u = 0; u < CBW; ++u) {
      wa[u][0] = wfrag(0, r.q, cbw0 + u, 0);
      wa[u][1] = wfrag(0, r.q, cbw0 + u, 1);
    }
    // pixel fragments one (tap, pixel block) step ahead of their MFMAs (across taps too), and group barriers that
    // keep each step's two LDS reads ahead of the previous step's MFMAs: without them the reads sit right before
    // their use and every block waits an LDS round trip
    auto rd = [&](int t, int cb, f16x8_t& h, f16x8_t& l) __attribute__((always_inline)) {
      const h16_t* src = Pl + (bpx[cb] + (t / 3) * HW_ + (t % 3)) * PS + 8 * g;
      h = *reinterpret_cast<const f16x8_t*>(src);
      l = *reinterpret_cast<const f16x8_t*>(src + PL);
    };
    f16x8_t nh, nl;
    rd(0, 0, nh, nl);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int tn = t + 1 < 9 ? t + 1 : t;
#pragma unroll
      for (int u = 0; u < CBW; ++u) {
        wn[u][0] = wfrag(tn, r.q, cbw0 + u, 0);
        wn[u][1] = wfrag(tn, r.q, cbw0 + u, 1);
      }
      load_part(cur, PER_TAP * t, min(PER_TAP * t + PER_TAP, NLD));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int cb = 0; cb < 8; ++cb) {
        const f16x8_t xh = nh, xlo = nl;
        if (cb < 7) rd(t, cb + 1, nh, nl);
        else if (t < 8) rd(t + 1, 0, nh, nl);
#pragma unroll
        for (int u = 0; u < CBW; ++u) {
          f32x4 c = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh, wa[u][1], acc[u][cb], 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(xlo, wa[u][0], c, 0, 0, 0);
          acc[u][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh, wa[u][0], c, 0, 0, 0);
        }
      }
#pragma unroll
      for (int cb = 0; cb < 8; ++cb) {
        if (cb < 7 || t < 8) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS read
        __builtin_amdgcn_sched_group_barrier(0x008, 3 * CBW, 0);                 // MFMA
      }
#pragma unroll
      for (int u = 0; u < CBW; ++u) {
        wa[u][0] = wn[u][0];
        wa[u][1] = wn[u][1];
      }
    }
    if (r.q == nq - 1) {
      float* yb = p.y + (long)r.b * p.ybs;
      float bv[CBW];
#pragma unroll
      for (int u = 0; u < CBW; ++u) bv[u] = bsh[16 * (cbw0 + u) + l15];
#pragma unroll
      for (int cb = 0; cb < 8; ++cb) {
        const int oy = r.ty * TH + 4 * ph + (cb >> 1), ox = r.tx * TW + (cb & 1) * 16 + 4 * g;
#pragma unroll
        for (int u = 0; u < CBW; ++u) {
          const long po = (long)(16 * (cbw0 + u) + l15) * HWi + oy * W + ox;
          f32x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = silu_fast_(acc[u][cb][e] * (1.0f / WSC) + bv[u]);
          if constexpr (RES) {
#pragma clang fp contract(off)  // a separately rounded add, as x + cv2(...): no fma with SiLU's last multiply
            if (oy < H && ox < W) o = o + *reinterpret_cast<const f32x4*>(p.res + (long)r.b * p.rbs + po);
          }
          if (oy < H && ox < W) __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(yb + po));
          acc[u][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    }
  }
  range_report(p.range_flag, rng);
  if (p.prep_flag && p.range_flag && blockIdx.x == 0 && threadIdx.x == 0 && *p.prep_flag) *p.range_flag = 1u;
}

// W [64][Cin][3][3] -> fragment-major planes of 64 W (see the file comment); one thread per (output channel, input
// channel, tap). The block's own range word records whether 64 W left fp16's range (re-reported by every launch).
__global__ __launch_bounds__(256) void conv3x3_prep_kernel(const float* __restrict__ w, int cin, int cout,
                                                           h16_t* __restrict__ wp, unsigned* range_flag,
                                                           unsigned* prep_flag) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long n_all = (long)cout * cin * 9;
  if (i >= n_all) return;
  const int t = (int)(i % 9), k = (int)((i / 9) % cin), n = (int)(i / (9L * cin));
  const float v = w[i] * WSC;
  const _Float16 hh = (_Float16)v;
  const _Float16 ll = (_Float16)(v - (float)hh);
  const int nq = cin >> 5, q = k >> 5, kk = k & 31, rb = n >> 4, ncb = cout >> 4;
  const int ln = ((kk >> 3) << 4) + (n & 15);
  const long base = ((long)((t * nq + q) * ncb + rb) * 2) * 512 + ln * 8 + (kk & 7);
  wp[base] = __builtin_bit_cast(h16_t, hh);
  wp[base + 512] = __builtin_bit_cast(h16_t, ll);
  const float m = fabsf(v);
  range_report(range_flag, m);
  range_report(prep_flag, m);
}

}  // namespace c3
}  // namespace ys

using namespace ys;

static int g_c3_abl = 0;
YS_EXPORT int yolosod_debug_set_conv3x3_abl(int abl) {
  const int old = g_c3_abl;
  g_c3_abl = abl;
  return old;
}

static int c3_cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, c = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0)
      c = 256;
    n = c;
  }
  return n;
}

static bool c3_cout_ok(int cout) { return cout == 32 || (cout % 64 == 0 && cout <= 512); }

// 3x3 / stride 1 / pad 1 conv with Cout 32 or a multiple of 64 (<= 512): Cin a multiple of 32 (<= 2048)
YS_EXPORT size_t yolosod_conv3x3_prep_bytes_ex(int cin, int cout) {
  if (cin <= 0 || cin % 32 || cin > 2048 || !c3_cout_ok(cout)) return 0;
  Sizer s;
  s.take<h16_t>((size_t)2 * cout * cin * 9);
  s.take<unsigned>(1);
  return s.off;
}
YS_EXPORT size_t yolosod_conv3x3_prep_bytes(int cin) { return yolosod_conv3x3_prep_bytes_ex(cin, 64); }

static bool conv3x3_carve(void* buf, size_t bytes, int cin, int cout, h16_t** wp, unsigned** flag) {
  Carver cv(buf, bytes);
  *wp = cv.take<h16_t>((size_t)2 * cout * cin * 9);
  *flag = cv.take<unsigned>(1);
  return *flag != nullptr;
}

// Weight preparation (re-run whenever the weights change): w [cout][cin][3][3] fp32 (BN folded) -> prep block.
YS_EXPORT int yolosod_conv3x3_prepare_ex(const float* w, int cin, int cout, void* prep, size_t prep_bytes,
                                         void* stream) {
  YS_CHECK_ARG(w && prep, "conv3x3_prepare: null pointer");
  YS_CHECK_ARG(yolosod_conv3x3_prep_bytes_ex(cin, cout) > 0, "conv3x3_prepare: (cin=%d, cout=%d) unsupported", cin,
               cout);
  h16_t* wp;
  unsigned* flag;
  YS_CHECK_ARG(conv3x3_carve(prep, prep_bytes, cin, cout, &wp, &flag), "conv3x3_prepare: block too small (%zu)",
               prep_bytes);
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(flag, 0, sizeof(unsigned), st) != hipSuccess) {
    set_error("conv3x3_prepare: flag reset failed");
    return -1;
  }
  const long n = (long)cout * cin * 9;
  hipLaunchKernelGGL(c3::conv3x3_prep_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, w, cin, cout, wp,
                     range_flag_dev(), flag);
  YS_CHECK_LAUNCH("conv3x3_prep");
  return 0;
}
YS_EXPORT int yolosod_conv3x3_prepare(const float* w, int cin, void* prep, size_t prep_bytes, void* stream) {
  return yolosod_conv3x3_prepare_ex(w, cin, 64, prep, prep_bytes, stream);
}

// y = SiLU(conv3x3(x, W) + bias) (+ res): x image b at x + b x_bstride ([cin][H][W]) -> image b's output [cout][H][W] at y + b y_bstride
// (y_bstride >= cout H W: a channel slice of a concat buffer); res (or NULL): image b at res + b res_bstride, added
// after the activation (Bottleneck shortcut). y must not alias x.
YS_EXPORT int yolosod_conv3x3_silu_xs(const float* x, long x_bstride, float* y, long y_bstride, const float* res,
                                      long res_bstride, int B, int cin, int cout, int H, int W, const float* bias,
                                      const void* prep, size_t prep_bytes, void* stream) {
  YS_CHECK_ARG(x && y && bias && prep, "conv3x3: null pointer");
  YS_CHECK_ARG(x_bstride >= (long)cin * H * W, "conv3x3: input batch stride %ld < %ld", x_bstride, (long)cin * H * W);
  YS_CHECK_ARG(B >= 0 && H > 0 && W > 0 && yolosod_conv3x3_prep_bytes_ex(cin, cout) > 0, "conv3x3: bad shape");
  YS_CHECK_ARG((long)cin * H * W < (1L << 31) && (long)cout * H * W < (1L << 31), "conv3x3: plane too large");
  YS_CHECK_ARG(y_bstride >= (long)cout * H * W, "conv3x3: output batch stride %ld < %ld", y_bstride,
               (long)cout * H * W);
  const bool v4 = W % 4 == 0;
  YS_CHECK_ARG(!v4 || (((uintptr_t)y & 15) == 0 && y_bstride % 4 == 0), "conv3x3: output not 16-byte aligned");
  YS_CHECK_ARG(!res || (v4 && ((uintptr_t)res & 15) == 0 && res_bstride % 4 == 0 && res_bstride >= (long)cout * H * W),
               "conv3x3: the residual needs W %% 4 == 0 and 16-byte aligned images");
  if (B == 0) return 0;
  h16_t* wp;
  unsigned* flag;
  YS_CHECK_ARG(conv3x3_carve(const_cast<void*>(prep), prep_bytes, cin, cout, &wp, &flag),
               "conv3x3: prepared block too small");
  c3::Args a{x, wp, bias, y, y_bstride, res, res_bstride, cin, H, W, (W + c3::TW - 1) / c3::TW,
             (H + c3::TH - 1) / c3::TH, cout / 16, range_flag_dev(), flag, 0, x_bstride};
  const int ngrp = cout == 32 ? 1 : cout / 64;
  const long nwg = (long)B * a.tiles_x * a.tiles_y * ngrp;
  YS_CHECK_ARG(nwg < (1L << 31), "conv3x3: too many tiles");
  hipStream_t st = (hipStream_t)stream;
  // the persistent kernel for W % 4 == 0 (two workgroups per CU); the one-tile-per-workgroup kernel otherwise
  if (v4 && g_c3_abl == 0) {
    a.ntiles = (int)((long)B * a.tiles_x * a.tiles_y);
    long grid = 2L * c3_cu_count();
    grid = grid < ((nwg + 7) / 8) * 8 ? grid : ((nwg + 7) / 8) * 8;
    grid = (grid + 7) / 8 * 8;
    auto pk = cout == 32 ? (res ? c3::conv3x3_p_kernel<1, true> : c3::conv3x3_p_kernel<1, false>)
                         : (res ? c3::conv3x3_p_kernel<2, true> : c3::conv3x3_p_kernel<2, false>);
    hipLaunchKernelGGL(pk, dim3((unsigned)grid), dim3(256), 0, st, a);
    YS_CHECK_LAUNCH("conv3x3");
    return 0;
  }
  auto kern = v4 ? c3::conv3x3_x2_kernel<0, true> : c3::conv3x3_x2_kernel<0, false>;
  if (cout == 32) {
    kern = res ? c3::conv3x3_x2_kernel<0, true, 1, true>
               : (v4 ? c3::conv3x3_x2_kernel<0, true, 1, false> : c3::conv3x3_x2_kernel<0, false, 1, false>);
  } else if (res) {
    kern = c3::conv3x3_x2_kernel<0, true, 2, true>;
  } else if (cout == 64 && v4) {
    switch (g_c3_abl) {  // timing ablations (W % 4 == 0 shapes, Cout 64)
      case 1: kern = c3::conv3x3_x2_kernel<1, true>; break;
      case 2: kern = c3::conv3x3_x2_kernel<2, true>; break;
      case 4: kern = c3::conv3x3_x2_kernel<4, true>; break;
      case 8: kern = c3::conv3x3_x2_kernel<8, true>; break;
      case 12: kern = c3::conv3x3_x2_kernel<12, true>; break;
      case 15: kern = c3::conv3x3_x2_kernel<15, true>; break;
      default: break;
    }
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(256), 0, st, a);
  YS_CHECK_LAUNCH("conv3x3");
  return 0;
}

// As yolosod_conv3x3_silu_xs with a contiguous x [B][cin][H][W].
YS_EXPORT int yolosod_conv3x3_silu_ex(const float* x, float* y, long y_bstride, const float* res, long res_bstride,
                                      int B, int cin, int cout, int H, int W, const float* bias, const void* prep,
                                      size_t prep_bytes, void* stream) {
  return yolosod_conv3x3_silu_xs(x, (long)cin * H * W, y, y_bstride, res, res_bstride, B, cin, cout, H, W, bias, prep,
                                 prep_bytes, stream);
}

// 3x3 / stride 1 / pad 1 conv with 64 outputs, contiguous y [B][64][H][W].
YS_EXPORT int yolosod_conv3x3_silu(const float* x, float* y, int B, int cin, int H, int W, const float* bias,
                                   const void* prep, size_t prep_bytes, void* stream) {
  return yolosod_conv3x3_silu_ex(x, y, 64L * H * W, nullptr, 0, B, cin, 64, H, W, bias, prep, prep_bytes, stream);
}
