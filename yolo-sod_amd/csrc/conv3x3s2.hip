// 3x3 / stride 2 / pad 1 convolution + folded BN bias + SiLU on the fp16 matrix cores at fp32 accuracy, with the
// channel / spatial gate of the MAFN operator that produces its input applied while the input is staged: the consumer
// of SE_Block L1 (Conv(64, 3, 2) at P1 -> P2) and of CBAM_Block L4 (Conv(256, 3, 2) at P2 -> P3) in the paper YAML
// (cfg yolov12-sod-fusion-v5-simple.yaml rows 1-2 and 4-5). The gate's output y = x * a (SE,
// smallobj_modules.py:92) or y = (x * ca) * sa (CBAM, cbam_block.py:53-54) is formed in registers with exactly the
// reference's fp32 products and goes straight into the convolution (conv.py:37-55 with the BN folded by fuse(),
// torch_utils.py:238-265): the gate's apply pass (read x, write y) and the convolution's re-read of y disappear.
//
// Method as conv3x3.hip: v = h + l fp16 two-term splits, products ah.bh + ah.bl + al.bh on v_mfma_f32_16x16x32_f16,
// weights x 64 split once per parameter version into fragment-major planes (for tap t, 32-channel input chunk q,
// 16-channel output block cb and plane p, the 64 lanes' fragments are 1 KB contiguous).
//
// Persistent: one 512-thread workgroup per CU (LDS 94 KB: the two fp16 planes of a 9 x 65 input halo), each looping
// over output tiles of 4 x 32 pixels and all Cout (64 or 128) channels, tiles taken from a contiguous per-XCD range.
// Per (tile, input chunk): the staged chunk (gated, split) in LDS; the next (tile, chunk)'s input loads are spread
// over the current chunk's nine taps (prefetch in registers); each tap's weight fragments are loaded one tap ahead.
// Wave w computes output channel block w % NCB for NCB of the tile's 8 pixel blocks (16 output pixels of one row);
// the pixels are the MFMA A operand, so a lane holds 4 consecutive output pixels of one channel (16-byte stores).
#include "common.h"

namespace ys {
namespace c3s2 {

constexpr float WSC = 64.0f;
constexpr int TH = 4, TW = 32;              // output tile
constexpr int HR = 2 * TH + 1, HC = 2 * TW + 1;  // 9 x 65 input halo
constexpr int NPX = HR * HC;                // 585 halo pixels
constexpr int PS = 32 + 8;                  // plane row stride (halves): stride-2 pixel reads of 16 lanes are 160 B
                                            // apart, which puts the ds_read_b128 lane groups on distinct bank quads
constexpr int PL = NPX * PS;                // plane (halves)
constexpr int NT = 512;
constexpr int NQUAD = NPX * 8;              // staged items per chunk: (4-channel quad, halo pixel)
constexpr int NIT = (NQUAD + NT - 1) / NT;  // 10
constexpr int NGP = (NPX + NT - 1) / NT;    // 2 spatial-gate values per thread

struct Args {
  const float* x;      // [B][Cin][H][W]
  const h16_t* wp;     // prepared planes (fragment-major, x 64)
  const float* bias;   // [Cout]
  const float* gc;     // [B][Cin] channel gate (GATE & 1), 16-byte aligned
  const float* gp;     // [B][H][W] spatial gate (GATE & 2)
  float* y;            // image b's output at y + b ybs: [Cout][Ho][Wo] (ybs >= Cout Ho Wo: a channel slice of a
                       // concat buffer)
  long ybs;
  int B, cin, H, W, Ho, Wo, tiles_x, tiles_y, ntiles;
  int ncb_all;         // channel blocks of the prepared weights (Cout / 16); the t2 kernel: ncb_all / NCB groups
  unsigned* range_flag;
  const unsigned* prep_flag;
};

// NCB: output channel blocks of 16 (Cout = 16 NCB: 4 or 8); GATE: bit 0 channel gate, bit 1 spatial gate.
// ABL: timing ablations (wrong results; yolosod_debug_set_conv3x3s2_abl): 1 no input loads, 2 every weight fragment
// from one address, 4 no MFMA (a VALU stand-in keeps the LDS reads), 8 no output stores
template <int NCB, int GATE, int ABL = 0>
__global__ __launch_bounds__(NT, 1) void conv3x3s2_kernel(Args p) {
  static_assert(NCB == 4 || NCB == 8, "Cout 64 or 128");
  constexpr int NPB = NCB;  // pixel blocks per wave (8 waves: 8 / NCB waves per channel block, 8 blocks per tile)
  __shared__ __attribute__((aligned(16))) h16_t Pl[2 * PL];
  __shared__ __attribute__((aligned(16))) float gcs[32];
  __shared__ float gps[NPX];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, g = lane >> 4;
  const int H = p.H, W = p.W, HWi = H * W, nq = p.cin >> 5;
  const int cb = wid % NCB, pb0 = (wid / NCB) * NPB;
  float rng = 0.f;

  // this workgroup's tiles: XCD x = blockIdx % 8 takes the contiguous range [x per, (x + 1) per), its j-th
  // workgroup tiles j, j + nj, ... of it (vertically / horizontally adjacent tiles share halo lines in one L2)
  const int nj = gridDim.x >> 3, j = blockIdx.x >> 3, xcd = blockIdx.x & 7;
  const int per = (p.ntiles + 7) >> 3;
  const int t_beg = xcd * per + j, t_end = min((xcd + 1) * per, p.ntiles);
  if (t_beg >= t_end) return;
  const int n_it = ((t_end - t_beg + nj - 1) / nj) * nq;  // (tile, chunk) iterations

  auto rsrc = [&](const void* base, unsigned bytes) {
    const unsigned long long a = (unsigned long long)base;
    return __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(a >> 32)) << 32) |
                (unsigned)__builtin_amdgcn_readfirstlane((unsigned)a)),
        (short)0, __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rx = rsrc(p.x, 0xffffffffu);  // per-image base in the scalar offset (checked < 2^32)
  const __amdgpu_buffer_rsrc_t rw = rsrc(p.wp, (unsigned)(9L * nq * NCB * 2 * 1024));

  // staging item e = tid + NT i: quad = e / NPX (channels 4 quad .. + 3 of the chunk), halo pixel e % NPX
  // (consecutive threads, consecutive pixels of a halo row); packed (quad, hy, hx)
  int pk[NIT];
#pragma unroll
  for (int i = 0; i < NIT; ++i) {
    const int e = min(tid + NT * i, NQUAD - 1);
    const int quad = e / NPX, px = e - quad * NPX;
    const int hy = px / HC, hx = px - hy * HC;
    pk[i] = (quad << 16) | (hy << 8) | hx;
  }
  auto tile_of = [&](int it, int& b, int& ty, int& tx, int& q) __attribute__((always_inline)) {
    const int t = t_beg + (it / nq) * nj;
    q = it - (it / nq) * nq;
    tx = t % p.tiles_x;
    ty = (t / p.tiles_x) % p.tiles_y;
    b = t / (p.tiles_x * p.tiles_y);
  };
  // loads of (tile, chunk) iteration `it` into sv (item i, channel c = k & 3 for k = 4 i + c in [k0, k1)); okb: bit
  // i = item i's pixel inside the image (zero padding otherwise; the load reads a clamped in-image address)
  f32x4 sv[NIT];
  float gcv = 0.f, gpv[NGP];
  unsigned okb_ld = 0;
  auto load_part = [&](int it, int k0, int k1) __attribute__((always_inline)) {
    int b, ty, tx, q;
    tile_of(it, b, ty, tx, q);
    const int iy0 = 2 * TH * ty - 1, ix0 = 2 * TW * tx - 1;
    const unsigned sb = __builtin_amdgcn_readfirstlane((unsigned)(((long)b * p.cin + 32 * q) * HWi * 4));
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      if (4 * i + 3 < k0 || 4 * i >= k1) continue;
      const int quad = pk[i] >> 16, hy = (pk[i] >> 8) & 255, hx = pk[i] & 255;
      const int yy = iy0 + hy, xx = ix0 + hx;
      if (4 * i >= k0) {  // the item's first load: its in-image bit
        const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
        okb_ld = ok ? (okb_ld | (1u << i)) : (okb_ld & ~(1u << i));
      }
      const unsigned vo = (unsigned)((4 * quad * HWi + min(max(yy, 0), H - 1) * W + min(max(xx, 0), W - 1)) * 4);
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (4 * i + c >= k0 && 4 * i + c < k1)
          sv[i][c] = (ABL & 1) ? 0.25f + (float)c
                               : __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, vo, sb + c * HWi * 4, 0));
    }
  };
  // the gates of iteration `it`: channel gate of the chunk's 32 channels (thread t < 32: channel t), spatial gate of
  // the halo pixels (thread t: pixels t + NT k), clamped unconditional loads
  auto load_gates = [&](int it) __attribute__((always_inline)) {
    int b, ty, tx, q;
    tile_of(it, b, ty, tx, q);
    if constexpr ((GATE & 1) != 0) gcv = p.gc[b * p.cin + 32 * q + (tid & 31)];
    if constexpr ((GATE & 2) != 0) {
      const int iy0 = 2 * TH * ty - 1, ix0 = 2 * TW * tx - 1;
#pragma unroll
      for (int k = 0; k < NGP; ++k) {
        const int px = min(tid + NT * k, NPX - 1);
        const int hy = px / HC, hx = px - hy * HC;
        gpv[k] = p.gp[(long)b * HWi + min(max(iy0 + hy, 0), H - 1) * W + min(max(ix0 + hx, 0), W - 1)];
      }
    }
  };
  // weight fragments of (tap t, chunk q) for this wave's channel block, planes 0 / 1
  auto wfrag = [&](int t, int q, int pl) __attribute__((always_inline)) {
    const int st = (ABL & 2) ? pl * 1024 : __builtin_amdgcn_readfirstlane((((t * nq + q) * NCB + cb) * 2 + pl) * 1024);
    return __builtin_bit_cast(f16x8_t, __builtin_amdgcn_raw_buffer_load_b128(rw, (unsigned)(lane * 16), st, 0));
  };
  // pixel block pb: output row pb >> 1, columns (pb & 1) 16 .. + 15; lane's halo pixel at tap (0, 0)
  int bpx[NPB];
#pragma unroll
  for (int k = 0; k < NPB; ++k) {
    const int pb = pb0 + k;
    bpx[k] = 2 * (pb >> 1) * HC + 2 * ((pb & 1) * 16 + l15);
  }
  f32x4 acc[NPB];
#pragma unroll
  for (int k = 0; k < NPB; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nw = __builtin_amdgcn_readfirstlane(p.Wo);
  const int o_ch = 16 * cb + l15;
  const float bo = p.bias[o_ch];  // loaded once: an epilogue load would wait behind every prefetch in flight

  load_part(0, 0, 4 * NIT);
  load_gates(0);
  for (int it = 0; it < n_it; ++it) {
    int b, ty, tx, q;
    tile_of(it, b, ty, tx, q);
    const unsigned okb = okb_ld;
    __syncthreads();  // every wave is done with the previous chunk's planes (and gates)
    if constexpr (GATE != 0) {
      if constexpr ((GATE & 1) != 0)
        if (tid < 32) gcs[tid] = gcv;
      if constexpr ((GATE & 2) != 0) {
#pragma unroll
        for (int k = 0; k < NGP; ++k)
          if (tid + NT * k < NPX) gps[tid + NT * k] = gpv[k];
      }
      __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int e = tid + NT * i;
      if (e < NQUAD) {
        const int quad = pk[i] >> 16, px = e - quad * NPX;
        f32x4 v = sv[i];
        if constexpr ((GATE & 1) != 0) v = v * *reinterpret_cast<const f32x4*>(gcs + 4 * quad);  // x * a (SE, CBAM ca)
        if constexpr ((GATE & 2) != 0) v = v * gps[px];  // (x * ca) * sa
        if (!((okb >> i) & 1u)) v = f32x4{0.f, 0.f, 0.f, 0.f};
        uint2 hh, ll;
        split4x(v, hh, ll);
        rng = range_acc(rng, v);
        h16_t* d = Pl + px * PS + 4 * quad;
        *reinterpret_cast<uint2*>(d) = hh;
        *reinterpret_cast<uint2*>(d + PL) = ll;
      }
    }
    __syncthreads();
    // next (tile, chunk)'s loads, spread over the taps behind each tap's weight prefetch (vmcnt counts in order);
    // the last iteration reloads itself (unconditional loads: no phis waiting on every load in flight)
    const int itn = it + 1 < n_it ? it + 1 : it;
    f16x8_t wa[2], wn[2];
    wa[0] = wfrag(0, q, 0);
    wa[1] = wfrag(0, q, 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int tn = t + 1 < 9 ? t + 1 : t;
      wn[0] = wfrag(tn, q, 0);
      wn[1] = wfrag(tn, q, 1);
      if (t < 8) load_part(itn, 5 * t, t == 7 ? 4 * NIT : 5 * t + 5);
      else load_gates(itn);
      __builtin_amdgcn_sched_barrier(0);
      const int toff = (t / 3) * HC + (t % 3);
#pragma unroll
      for (int k = 0; k < NPB; ++k) {
        const h16_t* src = Pl + (bpx[k] + toff) * PS + 8 * g;
        const f16x8_t xh = *reinterpret_cast<const f16x8_t*>(src);
        const f16x8_t xl = *reinterpret_cast<const f16x8_t*>(src + PL);
        if constexpr ((ABL & 4) != 0) {
          acc[k][0] += (float)xh[0] * (float)wa[0][0] + (float)xl[1] * (float)wa[1][1];
        } else {
          f32x4 c = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh, wa[1], acc[k], 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(xl, wa[0], c, 0, 0, 0);
          acc[k] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh, wa[0], c, 0, 0, 0);
        }
      }
      wa[0] = wn[0];
      wa[1] = wn[1];
    }
    if (q == nq - 1) {
      // epilogue: lane (g, l15) of pixel block pb holds output channel 16 cb + l15, pixels (row pb >> 1, columns
      // (pb & 1) 16 + 4 g .. + 3); every value first, then the non-temporal 16-byte stores (Wo % 4 == 0: 4 pixels
      // all in or all out; interleaved, each store's data registers were reused behind a full vmcnt wait)
      float* yo = p.y + (long)b * p.ybs + (long)o_ch * p.Ho * nw;
      f32x4 v[NPB];
#pragma unroll
      for (int k = 0; k < NPB; ++k)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) v[k][jj] = silu_fast_(acc[k][jj] * (1.0f / WSC) + bo);
#pragma unroll
      for (int k = 0; k < NPB; ++k) {
        const int pb = pb0 + k;
        const int oy = ty * TH + (pb >> 1), ox = tx * TW + (pb & 1) * 16 + 4 * g;
        if (oy < p.Ho && ox < nw && (!(ABL & 8) || v[k][0] == -1.2345e30f))
          __builtin_nontemporal_store(v[k], reinterpret_cast<f32x4*>(yo + oy * nw + ox));
        acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
  range_report(p.range_flag, rng);
  if (p.prep_flag && p.range_flag && blockIdx.x == 0 && threadIdx.x == 0 && *p.prep_flag) *p.range_flag = 1u;
}

// Cout 64 / Cin 32 (one input chunk: the SE L1 -> Conv L2 shape): the weights are held in registers for the kernel's
// lifetime (wave w: output channel block w & 3, all taps, 72 VGPRs), so no load but the next tile's input is in flight
// during the taps and all of them are issued right after the staging (no wait for a tap's weights waits behind them);
// wave w computes output rows 2 (w >> 2), + 1 (four pixel blocks) of its 16 channels. The epilogue goes through an
// LDS tile [row][channel][32 px (+4)] and leaves as 128-byte rows (8 lanes per row) while the next tile is staged (the
// general kernel's 64-byte lane-group stores were store-issue bound).
constexpr int ES = TW + 4;  // epilogue row stride (floats): 144-byte channel rows, conflict-free 16-byte writes
// THk output rows per tile, NTk threads per workgroup (THk = 2, NTk = 256: 72 KB of LDS, two workgroups per CU whose
// staging / compute phases interleave and whose input prefetches are both in flight)
template <int GATE, int ABL, int THk, int NTk>
__global__ __launch_bounds__(NTk, 512 / NTk) void conv3x3s2_rw_kernel(Args p) {
  constexpr int HRk = 2 * THk + 1, NPXk = HRk * HC, PLk = NPXk * PS, NQUADk = NPXk * 8;
  constexpr int NITk = (NQUADk + NTk - 1) / NTk, NGPk = (NPXk + NTk - 1) / NTk;
  static_assert(NITk <= 32, "okb bits");
  __shared__ __attribute__((aligned(16))) h16_t Pl[2 * PLk];
  __shared__ __attribute__((aligned(16))) float Ep[THk * 64 * ES];
  __shared__ __attribute__((aligned(16))) float gcs[32];
  __shared__ float gps[(GATE & 2) ? NPXk : 1];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, g = lane >> 4;
  const int H = p.H, W = p.W, HWi = H * W;
  const int rp = wid >> 2, cb = wid & 3;  // output rows 2 rp, 2 rp + 1 of the tile; channel block cb
  float rng = 0.f;

  const int nj = gridDim.x >> 3, j = blockIdx.x >> 3, xcd = blockIdx.x & 7;
  const int per = (p.ntiles + 7) >> 3;
  const int t_beg = xcd * per + j, t_end = min((xcd + 1) * per, p.ntiles);
  if (t_beg >= t_end) return;
  const int n_it = (t_end - t_beg + nj - 1) / nj;

  auto rsrc = [&](const void* base, unsigned bytes) {
    const unsigned long long a = (unsigned long long)base;
    return __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(a >> 32)) << 32) |
                (unsigned)__builtin_amdgcn_readfirstlane((unsigned)a)),
        (short)0, __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rx = rsrc(p.x, 0xffffffffu);
  const __amdgpu_buffer_rsrc_t rw = rsrc(p.wp, (unsigned)(9L * 4 * 2 * 1024));

  // this wave's weights: channel block cb, taps t, planes 0 / 1
  f16x8_t wr[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int pl = 0; pl < 2; ++pl)
      wr[t][pl] = __builtin_bit_cast(
          f16x8_t, __builtin_amdgcn_raw_buffer_load_b128(rw, (unsigned)(lane * 16), ((t * 4 + cb) * 2 + pl) * 1024, 0));
  // staging item e = tid + NTk i: quad = e / NPXk (channels 4 quad .. + 3), halo pixel e % NPXk = (hy, hx); its element
  // offset in the image for tile origin (0, 0) and its (hy, hx)
  int pk[NITk], el0[NITk];
#pragma unroll
  for (int i = 0; i < NITk; ++i) {
    const int e = min(tid + NTk * i, NQUADk - 1);
    const int quad = e / NPXk, px = e - quad * NPXk;
    const int hy = px / HC, hx = px - hy * HC;
    pk[i] = (quad << 16) | (hy << 8) | hx;
    el0[i] = 4 * quad * HWi + hy * W + hx;
  }
  struct Tile {
    int b, ty, tx;
  };
  auto tile_of = [&](int it) __attribute__((always_inline)) {
    const int t = t_beg + it * nj;
    Tile tl;
    tl.tx = t % p.tiles_x;
    tl.ty = (t / p.tiles_x) % p.tiles_y;
    tl.b = t / (p.tiles_x * p.tiles_y);
    return tl;
  };
  f32x4 sv[NITk];
  float gcv = 0.f, gpv[NGPk];
  unsigned okb_ld = 0;
  // the tile's input: one buffer resource per image (range = the image): offsets of rows above the image are
  // negative (huge as unsigned: out of range, the load returns 0) and every other out-of-image pixel reads some
  // in-image value that okb masks to the zero padding - no clamping on the load path
  auto load_tile = [&](const Tile& tl) __attribute__((always_inline)) {
    const int iy0 = 2 * THk * tl.ty - 1, ix0 = 2 * TW * tl.tx - 1;
    const __amdgpu_buffer_rsrc_t ri = rsrc(p.x + (long)tl.b * 32 * HWi, (unsigned)(32 * HWi * 4));
    const int toff = iy0 * W + ix0;
    const bool interior = iy0 >= 0 && ix0 >= 0 && iy0 + HRk <= H && ix0 + HC <= W;
    unsigned okb = 0xffffffffu;
    if (!interior) {
      okb = 0;
#pragma unroll
      for (int i = 0; i < NITk; ++i) {
        const int hy = (pk[i] >> 8) & 255, hx = pk[i] & 255;
        okb |= ((unsigned)(iy0 + hy) < (unsigned)H && (unsigned)(ix0 + hx) < (unsigned)W) ? (1u << i) : 0u;
      }
    }
#pragma unroll
    for (int i = 0; i < NITk; ++i) {
      const unsigned vo = (unsigned)((el0[i] + toff) * 4);
#pragma unroll
      for (int c = 0; c < 4; ++c)
        sv[i][c] = (ABL & 1) ? 0.25f + (float)c
                             : __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ri, vo + c * HWi * 4, 0, 0));
    }
    okb_ld = okb;
    if constexpr ((GATE & 1) != 0) gcv = p.gc[tl.b * 32 + (tid & 31)];
    if constexpr ((GATE & 2) != 0) {
#pragma unroll
      for (int k = 0; k < NGPk; ++k) {
        const int px = min(tid + NTk * k, NPXk - 1);
        const int hy = px / HC, hx = px - hy * HC;
        gpv[k] = p.gp[(long)tl.b * HWi + min(max(iy0 + hy, 0), H - 1) * W + min(max(ix0 + hx, 0), W - 1)];
      }
    }
  };
  int bpx[4];  // pixel block k: output row 2 rp + (k >> 1), columns (k & 1) 16 .. + 15
#pragma unroll
  for (int k = 0; k < 4; ++k) bpx[k] = 2 * (2 * rp + (k >> 1)) * HC + 2 * ((k & 1) * 16 + l15);
  const int nw = __builtin_amdgcn_readfirstlane(p.Wo);
  const float bo = p.bias[16 * cb + l15];
  // global stores of the epilogue tile: item idx = tid + NTk m: row idx >> 9, channel (idx >> 3) & 63, pixels
  // 4 (idx & 7) .. + 3 (8 lanes per 128-byte row)
  auto store_tile = [&](const Tile& tl) __attribute__((always_inline)) {
#pragma unroll
    for (int m = 0; m < THk * 512 / NTk; ++m) {
      const int idx = tid + NTk * m;
      const int r = idx >> 9, ch = (idx >> 3) & 63, px4 = idx & 7;
      const int ox = tl.tx * TW + 4 * px4, oy = tl.ty * THk + r;
      const f32x4 v = *reinterpret_cast<const f32x4*>(Ep + (r * 64 + ch) * ES + 4 * px4);
      if (oy < p.Ho && ox < nw && (!(ABL & 8) || v[0] == -1.2345e30f))
        __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p.y + (long)tl.b * p.ybs + ((long)ch * p.Ho + oy) * nw + ox));
    }
  };

  Tile cur = tile_of(0), prev = cur;
  load_tile(cur);
  for (int it = 0; it < n_it; ++it) {
    const unsigned okb = okb_ld;
    __syncthreads();  // every wave is done with the previous tile's planes, gates and epilogue tile writes
    if constexpr (GATE != 0) {
      if constexpr ((GATE & 1) != 0)
        if (tid < 32) gcs[tid] = gcv;
      if constexpr ((GATE & 2) != 0) {
#pragma unroll
        for (int k = 0; k < NGPk; ++k)
          if (tid + NTk * k < NPXk) gps[tid + NTk * k] = gpv[k];
      }
      __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < NITk; ++i) {
      const int e = tid + NTk * i;
      if (e < NQUADk) {
        const int quad = pk[i] >> 16, px = e - quad * NPXk;
        f32x4 v = sv[i];
        if constexpr ((GATE & 1) != 0) v = v * *reinterpret_cast<const f32x4*>(gcs + 4 * quad);
        if constexpr ((GATE & 2) != 0) v = v * gps[px];
        if (!((okb >> i) & 1u)) v = f32x4{0.f, 0.f, 0.f, 0.f};
        uint2 hh, ll;
        split4x(v, hh, ll);
        rng = range_acc(rng, v);
        h16_t* d = Pl + px * PS + 4 * quad;
        *reinterpret_cast<uint2*>(d) = hh;
        *reinterpret_cast<uint2*>(d + PLk) = ll;
      }
    }
    // the previous tile's output rows, issued after the staging's waits for this tile's input (a store ahead of
    // them made every wait a full vmcnt(0): the store count under its bounds branch is unknown)
    if (it > 0) store_tile(prev);
    __syncthreads();
    prev = cur;
    if (it + 1 < n_it) cur = tile_of(it + 1);
    load_tile(cur);  // the next tile's input (the last iteration reloads its own): in flight during every tap
    __builtin_amdgcn_sched_barrier(0);
    f32x4 acc[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int toff = (t / 3) * HC + (t % 3);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const h16_t* src = Pl + (bpx[k] + toff) * PS + 8 * g;
        const f16x8_t xh = *reinterpret_cast<const f16x8_t*>(src);
        const f16x8_t xl = *reinterpret_cast<const f16x8_t*>(src + PLk);
        if constexpr ((ABL & 4) != 0) {
          acc[k][0] += (float)xh[0] * (float)wr[t][0][0] + (float)xl[1] * (float)wr[t][1][1];
        } else {
          f32x4 c = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh, wr[t][1], acc[k], 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(xl, wr[t][0], c, 0, 0, 0);
          acc[k] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh, wr[t][0], c, 0, 0, 0);
        }
      }
    }
    // epilogue tile: lane (g, l15) of pixel block k holds channel 16 cb + l15, pixels (k & 1) 16 + 4 g .. + 3 of
    // row 2 rp + (k >> 1)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = silu_fast_(acc[k][e] * (1.0f / WSC) + bo);
      *reinterpret_cast<f32x4*>(Ep + ((2 * rp + (k >> 1)) * 64 + 16 * cb + l15) * ES + 16 * (k & 1) + 4 * g) = v;
    }
  }
  __syncthreads();
  store_tile(prev);
  range_report(p.range_flag, rng);
  if (p.prep_flag && p.range_flag && blockIdx.x == 0 && threadIdx.x == 0 && *p.prep_flag) *p.range_flag = 1u;
}

// Any (Cout 64 / 128, Cin multiple of 32) with 2-row tiles and 256-thread workgroups, three per CU (LDS 54 KB): the
// general kernel's streamed weights (one tap ahead, the next (tile, chunk)'s input spread over the taps behind them;
// two per CU at Cout 128, whose 8 accumulator tiles per wave need more than 168 registers)
// with the register-weight kernel's unclamped per-image buffer addressing; wave w computes channel blocks
// CBW w .. + CBW - 1 (CBW = NCB / 4) for all four pixel blocks of the tile (rows 0, 1 x two 16-column blocks).
template <int NCB, int GATE>
__global__ __launch_bounds__(256, NCB == 8 ? 2 : 3) void conv3x3s2_t2_kernel(Args p) {
  constexpr int THk = 2, NTk = 256, HRk = 2 * THk + 1, NPXk = HRk * HC, PLk = NPXk * PS, NQUADk = NPXk * 8;
  constexpr int NITk = (NQUADk + NTk - 1) / NTk, NGPk = (NPXk + NTk - 1) / NTk, CBW = NCB / 4;
  static_assert(NCB == 4 || NCB == 8, "Cout 64 or 128");
  __shared__ __attribute__((aligned(16))) h16_t Pl[2 * PLk];
  __shared__ __attribute__((aligned(16))) float gcs[32];
  __shared__ float gps[(GATE & 2) ? NPXk : 1];
  __shared__ float bsh[512];  // the bias of every output channel (Cout <= 512): an epilogue load would wait behind
                              // every prefetch in flight
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, g = lane >> 4;
  const int H = p.H, W = p.W, HWi = H * W, nq = p.cin >> 5;
  float rng = 0.f;
  for (int o = tid; o < 16 * p.ncb_all; o += 256) bsh[o] = p.bias[o];  // ordered before use by the loop's barriers

  const int nj = gridDim.x >> 3, j = blockIdx.x >> 3, xcd = blockIdx.x & 7;
  const int ngrp = p.ncb_all / NCB;  // output channel groups of 16 NCB: work item = (tile, group), group fastest
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
  int pk[NITk], el0[NITk];
#pragma unroll
  for (int i = 0; i < NITk; ++i) {
    const int e = min(tid + NTk * i, NQUADk - 1);
    const int quad = e / NPXk, px = e - quad * NPXk;
    const int hy = px / HC, hx = px - hy * HC;
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
  f32x4 sv[NITk];
  float gcv = 0.f, gpv[NGPk];
  unsigned okb_ld = 0;
  // part [k0, k1) of loads k = 4 i + c of (tile, chunk) r: per-image buffer resource (range = the chunk's planes to the
  // image end); rows above the image are negative offsets (out of range: 0), other out-of-image pixels masked by okb
  auto load_part = [&](const It& r, int k0, int k1) __attribute__((always_inline)) {
    const int iy0 = 2 * THk * r.ty - 1, ix0 = 2 * TW * r.tx - 1;
    const __amdgpu_buffer_rsrc_t ri =
        rsrc(p.x + ((long)r.b * p.cin + 32 * r.q) * HWi, (unsigned)((p.cin - 32 * r.q) * HWi * 4));
    const int toff = iy0 * W + ix0;
    if (k0 == 0) {
      const bool interior = iy0 >= 0 && ix0 >= 0 && iy0 + HRk <= H && ix0 + HC <= W;
      unsigned okb = 0xffffffffu;
      if (!interior) {
        okb = 0;
#pragma unroll
        for (int i = 0; i < NITk; ++i) {
          const int hy = (pk[i] >> 8) & 255, hx = pk[i] & 255;
          okb |= ((unsigned)(iy0 + hy) < (unsigned)H && (unsigned)(ix0 + hx) < (unsigned)W) ? (1u << i) : 0u;
        }
      }
      okb_ld = okb;
    }
#pragma unroll
    for (int i = 0; i < NITk; ++i) {
      if (4 * i + 3 < k0 || 4 * i >= k1) continue;
      const unsigned vo = (unsigned)((el0[i] + toff) * 4);
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (4 * i + c >= k0 && 4 * i + c < k1)
          sv[i][c] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ri, vo + c * HWi * 4, 0, 0));
    }
  };
  auto load_gates = [&](const It& r) __attribute__((always_inline)) {
    if constexpr ((GATE & 1) != 0) gcv = p.gc[r.b * p.cin + 32 * r.q + (tid & 31)];
    if constexpr ((GATE & 2) != 0) {
      const int iy0 = 2 * THk * r.ty - 1, ix0 = 2 * TW * r.tx - 1;
#pragma unroll
      for (int k = 0; k < NGPk; ++k) {
        const int px = min(tid + NTk * k, NPXk - 1);
        const int hy = px / HC, hx = px - hy * HC;
        gpv[k] = p.gp[(long)r.b * HWi + min(max(iy0 + hy, 0), H - 1) * W + min(max(ix0 + hx, 0), W - 1)];
      }
    }
  };
  auto wfrag = [&](int t, int q, int cb, int pl) __attribute__((always_inline)) {  // cb: over all ncb_all blocks
    const int st = __builtin_amdgcn_readfirstlane((((t * nq + q) * p.ncb_all + cb) * 2 + pl) * 1024);
    return __builtin_bit_cast(f16x8_t, __builtin_amdgcn_raw_buffer_load_b128(rw, (unsigned)(lane * 16), st, 0));
  };
  int bpx[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) bpx[k] = 2 * (k >> 1) * HC + 2 * ((k & 1) * 16 + l15);
  f32x4 acc[4][CBW];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int u = 0; u < CBW; ++u) acc[k][u] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nw = __builtin_amdgcn_readfirstlane(p.Wo);
  constexpr int NLD = 4 * NITk;               // loads per (tile, chunk)
  constexpr int PER_TAP = (NLD + 7) / 8;      // spread over taps 0..7

  It cur = it_of(0);
  load_part(cur, 0, NLD);
  load_gates(cur);
  for (int it = 0; it < n_it; ++it) {
    const It r = cur;
    const unsigned okb = okb_ld;
    __syncthreads();
    if constexpr (GATE != 0) {
      if constexpr ((GATE & 1) != 0)
        if (tid < 32) gcs[tid] = gcv;
      if constexpr ((GATE & 2) != 0) {
#pragma unroll
        for (int k = 0; k < NGPk; ++k)
          if (tid + NTk * k < NPXk) gps[tid + NTk * k] = gpv[k];
      }
      __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < NITk; ++i) {
      const int e = tid + NTk * i;
      if (e < NQUADk) {
        const int quad = pk[i] >> 16, px = e - quad * NPXk;
        f32x4 v = sv[i];
        if constexpr ((GATE & 1) != 0) v = v * *reinterpret_cast<const f32x4*>(gcs + 4 * quad);
        if constexpr ((GATE & 2) != 0) v = v * gps[px];
        if (!((okb >> i) & 1u)) v = f32x4{0.f, 0.f, 0.f, 0.f};
        uint2 hh, ll;
        split4x(v, hh, ll);
        rng = range_acc(rng, v);
        h16_t* d = Pl + px * PS + 4 * quad;
        *reinterpret_cast<uint2*>(d) = hh;
        *reinterpret_cast<uint2*>(d + PLk) = ll;
      }
    }
    __syncthreads();
    if (it + 1 < n_it) cur = it_of(it + 1);
    const int cb0 = r.grp * NCB + CBW * wid;  // this wave's first channel block (of all ncb_all)
    f16x8_t wa[CBW][2], wn[CBW][2];
#pragma unroll
    for (int u = 0; u < CBW; ++u) {
      wa[u][0] = wfrag(0, r.q, cb0 + u, 0);
      wa[u][1] = wfrag(0, r.q, cb0 + u, 1);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int tn = t + 1 < 9 ? t + 1 : t;
#pragma unroll
      for (int u = 0; u < CBW; ++u) {
        wn[u][0] = wfrag(tn, r.q, cb0 + u, 0);
        wn[u][1] = wfrag(tn, r.q, cb0 + u, 1);
      }
      if (t < 8) load_part(cur, PER_TAP * t, min(PER_TAP * t + PER_TAP, NLD));
      else load_gates(cur);
      __builtin_amdgcn_sched_barrier(0);
      const int toff = (t / 3) * HC + (t % 3);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const h16_t* src = Pl + (bpx[k] + toff) * PS + 8 * g;
        const f16x8_t xh = *reinterpret_cast<const f16x8_t*>(src);
        const f16x8_t xl = *reinterpret_cast<const f16x8_t*>(src + PLk);
#pragma unroll
        for (int u = 0; u < CBW; ++u) {
          f32x4 c = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh, wa[u][1], acc[k][u], 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(xl, wa[u][0], c, 0, 0, 0);
          acc[k][u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh, wa[u][0], c, 0, 0, 0);
        }
      }
#pragma unroll
      for (int u = 0; u < CBW; ++u) {
        wa[u][0] = wn[u][0];
        wa[u][1] = wn[u][1];
      }
    }
    if (r.q == nq - 1) {
      float bo[CBW];
#pragma unroll
      for (int u = 0; u < CBW; ++u) bo[u] = bsh[16 * (cb0 + u) + l15];
      f32x4 v[4][CBW];
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int u = 0; u < CBW; ++u)
#pragma unroll
          for (int e = 0; e < 4; ++e) v[k][u][e] = silu_fast_(acc[k][u][e] * (1.0f / WSC) + bo[u]);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int oy = r.ty * THk + (k >> 1), ox = r.tx * TW + (k & 1) * 16 + 4 * g;
#pragma unroll
        for (int u = 0; u < CBW; ++u) {
          const int o = 16 * (cb0 + u) + l15;
          if (oy < p.Ho && ox < nw)
            __builtin_nontemporal_store(
                v[k][u], reinterpret_cast<f32x4*>(p.y + (long)r.b * p.ybs + ((long)o * p.Ho + oy) * nw + ox));
          acc[k][u] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    }
  }
  range_report(p.range_flag, rng);
  if (p.prep_flag && p.range_flag && blockIdx.x == 0 && threadIdx.x == 0 && *p.prep_flag) *p.range_flag = 1u;
}

// W [Cout][Cin][3][3] -> fragment-major planes of 64 W: one thread per (output channel, input channel, tap). The
// block's own range word records whether 64 W left fp16's range (re-reported by every launch).
__global__ __launch_bounds__(256) void conv3x3s2_prep_kernel(const float* __restrict__ w, int cin, int cout,
                                                             h16_t* __restrict__ wp, unsigned* range_flag,
                                                             unsigned* prep_flag) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long n_all = (long)cout * cin * 9;
  if (i >= n_all) return;
  const int t = (int)(i % 9), k = (int)((i / 9) % cin), n = (int)(i / (9L * cin));
  const float v = w[i] * WSC;
  const _Float16 hh = (_Float16)v;
  const _Float16 ll = (_Float16)(v - (float)hh);
  const int nq = cin >> 5, q = k >> 5, kk = k & 31, cbk = n >> 4, ncb = cout >> 4;
  const int ln = ((kk >> 3) << 4) + (n & 15);
  const long base = ((long)((t * nq + q) * ncb + cbk) * 2) * 512 + ln * 8 + (kk & 7);
  wp[base] = __builtin_bit_cast(h16_t, hh);
  wp[base + 512] = __builtin_bit_cast(h16_t, ll);
  const float m = fabsf(v);
  range_report(range_flag, m);
  range_report(prep_flag, m);
}

}  // namespace c3s2
}  // namespace ys

using namespace ys;

static int g_s2_abl = 0;
YS_EXPORT int yolosod_debug_set_conv3x3s2_abl(int abl) {
  const int old = g_s2_abl;
  g_s2_abl = abl;
  return old;
}

static int s2_cu_count() {
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

// 3x3 / stride 2 / pad 1 conv with Cout 64 or a multiple of 128 (<= 512) and Cin a multiple of 32 (<= 2048)
YS_EXPORT size_t yolosod_conv3x3s2_prep_bytes(int cin, int cout) {
  if (cin <= 0 || cin % 32 || cin > 2048 || !(cout == 64 || (cout % 128 == 0 && cout <= 512))) return 0;
  Sizer s;
  s.take<h16_t>((size_t)2 * cout * cin * 9);
  s.take<unsigned>(1);
  return s.off;
}

static bool s2_carve(void* buf, size_t bytes, int cin, int cout, h16_t** wp, unsigned** flag) {
  Carver cv(buf, bytes);
  *wp = cv.take<h16_t>((size_t)2 * cout * cin * 9);
  *flag = cv.take<unsigned>(1);
  return *flag != nullptr;
}

// Weight preparation (re-run whenever the weights change): w [cout][cin][3][3] fp32 (BN folded) -> prep block.
YS_EXPORT int yolosod_conv3x3s2_prepare(const float* w, int cin, int cout, void* prep, size_t prep_bytes,
                                        void* stream) {
  YS_CHECK_ARG(w && prep, "conv3x3s2_prepare: null pointer");
  YS_CHECK_ARG(yolosod_conv3x3s2_prep_bytes(cin, cout) > 0, "conv3x3s2_prepare: (cin=%d, cout=%d) unsupported", cin,
               cout);
  h16_t* wp;
  unsigned* flag;
  YS_CHECK_ARG(s2_carve(prep, prep_bytes, cin, cout, &wp, &flag), "conv3x3s2_prepare: block too small (%zu)",
               prep_bytes);
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(flag, 0, sizeof(unsigned), st) != hipSuccess) {
    set_error("conv3x3s2_prepare: flag reset failed");
    return -1;
  }
  const long n = (long)cout * cin * 9;
  hipLaunchKernelGGL(c3s2::conv3x3s2_prep_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, w, cin, cout,
                     wp, range_flag_dev(), flag);
  YS_CHECK_LAUNCH("conv3x3s2_prep");
  return 0;
}

// y = SiLU(conv3x3_s2((x * gc) * gp, W) + bias): x [B][cin][H][W] -> image b's output [cout][Ho][Wo] at
// y + b y_bstride (y_bstride >= cout Ho Wo: a channel slice of a concat buffer), Ho = (H + 1) / 2, Wo = (W + 1) / 2
// (Wo % 4 == 0); gc [B][cin] (16-byte aligned) and gp [B][H][W] may each be NULL (no gate).
YS_EXPORT int yolosod_conv3x3s2_silu_out(const float* x, float* y, long y_bstride, int B, int cin, int cout, int H,
                                         int W, const float* bias, const float* gc, const float* gp, const void* prep,
                                         size_t prep_bytes, void* stream) {
  YS_CHECK_ARG(x && y && bias && prep, "conv3x3s2: null pointer");
  YS_CHECK_ARG(B >= 0 && H > 0 && W > 0 && yolosod_conv3x3s2_prep_bytes(cin, cout) > 0, "conv3x3s2: bad shape");
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  YS_CHECK_ARG(Wo % 4 == 0, "conv3x3s2: output width %d not a multiple of 4", Wo);
  YS_CHECK_ARG(y_bstride >= (long)cout * Ho * Wo, "conv3x3s2: output batch stride %ld < %ld", y_bstride,
               (long)cout * Ho * Wo);
  YS_CHECK_ARG(((uintptr_t)y & 15) == 0 && y_bstride % 4 == 0, "conv3x3s2: output not 16-byte aligned");
  YS_CHECK_ARG((long)B * cin * H * W * 4 < (1L << 32) && (long)cin * H * W < (1L << 31),
               "conv3x3s2: input too large for 32-bit buffer offsets");
  YS_CHECK_ARG(!gc || ((uintptr_t)gc & 15) == 0, "conv3x3s2: channel gate must be 16-byte aligned");
  if (B == 0) return 0;
  h16_t* wp;
  unsigned* flag;
  YS_CHECK_ARG(s2_carve(const_cast<void*>(prep), prep_bytes, cin, cout, &wp, &flag),
               "conv3x3s2: prepared block too small");
  const int tx = (Wo + c3s2::TW - 1) / c3s2::TW, ty = (Ho + c3s2::TH - 1) / c3s2::TH;
  const long ntiles = (long)B * tx * ty;
  YS_CHECK_ARG(ntiles < (1L << 30), "conv3x3s2: too many tiles");
  c3s2::Args a{x, wp, bias, gc, gp, y, y_bstride, B, cin, H, W, Ho, Wo, tx, ty, (int)ntiles, cout / 16,
               range_flag_dev(), flag};
  // persistent grid: one workgroup per CU (a multiple of 8 = one per XCD slot), at most one per tile
  long grid = s2_cu_count();
  grid = grid < ((ntiles + 7) / 8) * 8 ? grid : ((ntiles + 7) / 8) * 8;
  grid = (grid + 7) / 8 * 8;
  const int gate = (gc ? 1 : 0) | (gp ? 2 : 0);
  hipStream_t st = (hipStream_t)stream;
#define S2_LAUNCH(NCB_, G_) \
  hipLaunchKernelGGL((c3s2::conv3x3s2_kernel<NCB_, G_>), dim3((unsigned)grid), dim3(c3s2::NT), 0, st, a)
  // Cout 64 / Cin 32 (the gated L2 conv): register-resident weights, 2-row tiles, two 256-thread workgroups per CU
  // (4-row tiles in one 512-thread workgroup measured slower); other shapes: 2-row tiles of the general kernel
  if (cout == 64 && cin == 32 && g_s2_abl < 100) {
    c3s2::Args a2 = a;
    a2.tiles_y = (Ho + 1) / 2;
    const long nt2 = (long)B * a2.tiles_y * tx;
    a2.ntiles = (int)nt2;
    long g2 = 2L * s2_cu_count();
    g2 = g2 < ((nt2 + 7) / 8) * 8 ? g2 : ((nt2 + 7) / 8) * 8;
    g2 = (g2 + 7) / 8 * 8;
#define S2RW_LAUNCH(G_, A_) \
  hipLaunchKernelGGL((c3s2::conv3x3s2_rw_kernel<G_, A_, 2, 256>), dim3((unsigned)g2), dim3(256), 0, st, a2)
    if (gate == 1) {
      switch (g_s2_abl) {
        case 1: S2RW_LAUNCH(1, 1); break;
        case 4: S2RW_LAUNCH(1, 4); break;
        case 8: S2RW_LAUNCH(1, 8); break;
        case 13: S2RW_LAUNCH(1, 13); break;
        default: S2RW_LAUNCH(1, 0); break;
      }
    } else if (gate == 0) S2RW_LAUNCH(0, 0);
    else if (gate == 2) S2RW_LAUNCH(2, 0);
    else S2RW_LAUNCH(3, 0);
#undef S2RW_LAUNCH
  } else if (g_s2_abl < 100 || cout > 128) {  // 2-row tiles, 3 (Cout 64) / 2 workgroups per CU
    c3s2::Args a2 = a;
    a2.tiles_y = (Ho + 1) / 2;
    const long nt2 = (long)B * a2.tiles_y * tx * (cout == 64 ? 1 : cout / 128);  // work items: (tile, group)
    a2.ntiles = (int)((long)B * a2.tiles_y * tx);
    long g2 = (cout == 64 ? 3L : 2L) * s2_cu_count();
    g2 = g2 < ((nt2 + 7) / 8) * 8 ? g2 : ((nt2 + 7) / 8) * 8;
    g2 = (g2 + 7) / 8 * 8;
#define S2T2_LAUNCH(NCB_, G_) \
  hipLaunchKernelGGL((c3s2::conv3x3s2_t2_kernel<NCB_, G_>), dim3((unsigned)g2), dim3(256), 0, st, a2)
    if (cout == 64) {
      if (gate == 0) S2T2_LAUNCH(4, 0);
      else if (gate == 1) S2T2_LAUNCH(4, 1);
      else if (gate == 2) S2T2_LAUNCH(4, 2);
      else S2T2_LAUNCH(4, 3);
    } else {
      if (gate == 0) S2T2_LAUNCH(8, 0);
      else if (gate == 1) S2T2_LAUNCH(8, 1);
      else if (gate == 2) S2T2_LAUNCH(8, 2);
      else S2T2_LAUNCH(8, 3);
    }
#undef S2T2_LAUNCH
  } else if (g_s2_abl && cout == 64 && gate == 1) {  // timing ablations of the general kernel (abl + 100)
    switch (g_s2_abl - 100) {
      case 1: hipLaunchKernelGGL((c3s2::conv3x3s2_kernel<4, 1, 1>), dim3((unsigned)grid), dim3(c3s2::NT), 0, st, a); break;
      case 2: hipLaunchKernelGGL((c3s2::conv3x3s2_kernel<4, 1, 2>), dim3((unsigned)grid), dim3(c3s2::NT), 0, st, a); break;
      case 4: hipLaunchKernelGGL((c3s2::conv3x3s2_kernel<4, 1, 4>), dim3((unsigned)grid), dim3(c3s2::NT), 0, st, a); break;
      case 8: hipLaunchKernelGGL((c3s2::conv3x3s2_kernel<4, 1, 8>), dim3((unsigned)grid), dim3(c3s2::NT), 0, st, a); break;
      case 12: hipLaunchKernelGGL((c3s2::conv3x3s2_kernel<4, 1, 12>), dim3((unsigned)grid), dim3(c3s2::NT), 0, st, a); break;
      case 15: hipLaunchKernelGGL((c3s2::conv3x3s2_kernel<4, 1, 15>), dim3((unsigned)grid), dim3(c3s2::NT), 0, st, a); break;
      default: S2_LAUNCH(4, 1); break;
    }
  } else if (cout == 64) {
    if (gate == 0) S2_LAUNCH(4, 0);
    else if (gate == 1) S2_LAUNCH(4, 1);
    else if (gate == 2) S2_LAUNCH(4, 2);
    else S2_LAUNCH(4, 3);
  } else {
    if (gate == 0) S2_LAUNCH(8, 0);
    else if (gate == 1) S2_LAUNCH(8, 1);
    else if (gate == 2) S2_LAUNCH(8, 2);
    else S2_LAUNCH(8, 3);
  }
#undef S2_LAUNCH
  YS_CHECK_LAUNCH("conv3x3s2");
  return 0;
}

// As yolosod_conv3x3s2_silu_out with a contiguous y [B][cout][Ho][Wo].
YS_EXPORT int yolosod_conv3x3s2_silu(const float* x, float* y, int B, int cin, int cout, int H, int W,
                                     const float* bias, const float* gc, const float* gp, const void* prep,
                                     size_t prep_bytes, void* stream) {
  return yolosod_conv3x3s2_silu_out(x, y, (long)cout * ((H + 1) / 2) * ((W + 1) / 2), B, cin, cout, H, W, bias, gc, gp,
                                    prep, prep_bytes, stream);
}
