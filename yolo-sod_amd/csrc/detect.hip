// Detect-head post-processing on gfx950: DFL box decode + class sigmoid, and class-wise greedy NMS.
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
// NMS design (no host sync, no n^2 memory):
//   nms_prep   : one thread per anchor - xywh->xyxy (optionally in place), candidate class mask (score > conf,
//                class filter, best-class or multi-label).
//   nms_image  : one 512-thread workgroup per image -
//                (a) order-preserving compaction of (anchor, class) candidates (block scan), so that the
//                    candidate position equals the reference's row order;
//                (b) stable LSD radix sort on the descending fp32 score (4 x 8-bit passes in L2-resident scratch,
//                    wave-ballot ranking, trivially-uniform passes skipped) -> reference order incl. ties;
//                (c) max_nms cut, then greedy NMS over 512-candidate chunks: every candidate is tested against the
//                    boxes already kept (LDS), the survivors' in-chunk IoU bitmask (512x512 bits in LDS) is built
//                    in parallel, and one wave resolves the chunk sequentially; stops as soon as max_det boxes are
//                    kept (later boxes can never enter the [:max_det] output).
#include "common.h"
#include <math.h>

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
// logits, cv3[i][-1]: c3 -> nc class logits, head.py:45-48,70) run as fp32 MFMA v_mfma_f32_16x16x4_f32 straight
// into the DFL / dist2bbox / sigmoid decode, so the [B, 64+nc, H, W] raw maps never exist in HBM.
//   A = conv weights [out][k] (held in registers for the wave's lifetime), B = tower features [k][pixel] (NCHW,
//   loaded straight from HBM), D[out][pixel]: lane (g = lane>>4, j = lane&15) holds outputs 4g..4g+3 of pixel j.
//   Box tile s (16 rows) is exactly side s's 16 DFL bins, so the softmax max / sum / expectation are 4 local
//   values plus two permlane swaps (xor16, xor32). Class tile: rows 0..15 (nc <= 16).
// Each wave owns NTS consecutive 16-pixel groups of one level of one image.
// ------------------------------------------------------------------------------------------------
struct HeadArgs {
  const float* fb[4];  // box tower features  [B][C2][HW]
  const float* fc[4];  // class tower features [B][C3][HW]
  const float* wb[4];  // [64][C2]
  const float* bb[4];  // [64]
  const float* wc[4];  // [nc][C3]
  const float* bc[4];  // [nc]
  int hw[4], w[4], a_off[4], blk_off[5];
  float stride[4];
  int nl, nc, A;
  float* y;
};

template <int C2, int C3, int NTS>
__global__ __launch_bounds__(256) void detect_head_kernel(HeadArgs d) {
  const int b = blockIdx.y;
  int l = 0;
#pragma unroll
  for (int i = 1; i < 4; ++i)
    if (i < d.nl && (int)blockIdx.x >= d.blk_off[i]) l = i;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int g = lane >> 4, j = lane & 15;
  const int HW = d.hw[l];
  const int px0 = (((int)blockIdx.x - d.blk_off[l]) * 4 + wv) * (NTS * 16);
  if (px0 >= HW) return;  // whole wave; the kernel has no workgroup barrier
  const int nc = d.nc;

  // A operands: W[row = 16t + j][k = 4q + g]; biases of the rows this lane's accumulators hold (4g + r)
  float wbr[4][C2 / 4], wcr[C3 / 4], bbr[4][4], bcr[4];
  {
    const float* wb = d.wb[l];
    const float* wc = d.wc[l];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int q = 0; q < C2 / 4; ++q) wbr[t][q] = wb[(16 * t + j) * C2 + 4 * q + g];
#pragma unroll
    for (int q = 0; q < C3 / 4; ++q) wcr[q] = (j < nc) ? wc[j * C3 + 4 * q + g] : 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) bbr[t][r] = d.bb[l][16 * t + 4 * g + r];
#pragma unroll
    for (int r = 0; r < 4; ++r) bcr[r] = (4 * g + r < nc) ? d.bc[l][4 * g + r] : 0.f;
  }
  const float* fbb = d.fb[l] + (long)b * C2 * HW;
  const float* fcb = d.fc[l] + (long)b * C3 * HW;
  const int W = d.w[l];
  const float st = d.stride[l];
  float* yb = d.y + (long)b * (4 + nc) * d.A + d.a_off[l];

  for (int ts = 0; ts < NTS; ++ts) {
    const int p0 = px0 + ts * 16;
    if (p0 >= HW) break;
    const int p = p0 + j;
    const bool ok = p < HW;
    float xb[C2 / 4], xc[C3 / 4];
#pragma unroll
    for (int q = 0; q < C2 / 4; ++q) xb[q] = ok ? fbb[(long)(4 * q + g) * HW + p] : 0.f;
#pragma unroll
    for (int q = 0; q < C3 / 4; ++q) xc[q] = ok ? fcb[(long)(4 * q + g) * HW + p] : 0.f;
    f32x4 acc[5];
#pragma unroll
    for (int t = 0; t < 5; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < C2 / 4; ++q)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wbr[t][q], xb[q], acc[t], 0, 0, 0);
#pragma unroll
    for (int q = 0; q < C3 / 4; ++q) acc[4] = __builtin_amdgcn_mfma_f32_16x16x4f32(wcr[q], xc[q], acc[4], 0, 0, 0);

    // DFL (block.py:79-82): softmax over the 16 bins of each side, expectation with weights 0..15
    float dist[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[s][r] + bbr[s][r];
      float mx = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
      mx = xor32_max(xor16_max(mx));
      float sum = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = expf(v[r] - mx);
        sum += v[r];
      }
      sum = xor32_sum(xor16_sum(sum));
      const float inv = 1.0f / sum;
      float e = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) e += (float)(4 * g + r) * (v[r] * inv);
      dist[s] = xor32_sum(xor16_sum(e));
    }
    if (!ok) continue;
    const int iy = p / W, ix = p - iy * W;
    const float ax = (float)ix + 0.5f, ay = (float)iy + 0.5f;
    const float x1 = ax - dist[0], y1 = ay - dist[1];
    const float x2 = ax + dist[2], y2 = ay + dist[3];
    // dist2bbox xywh (tal.py:348-357) * stride; lane group g writes component g
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
  }
}

// ------------------------------------------------------------------------------------------------
// NMS
// ------------------------------------------------------------------------------------------------
struct NmsArgs {
  float* pred;  // [B][4+nc][A]
  int B, nc, A;
  float conf;
  double iou;
  const int* classes;
  int n_classes;
  int agnostic, multi_label, max_det, max_nms, in_place;
  float max_wh;
  float4* boxes;                 // [B][A] xyxy
  unsigned long long* amask;     // [B][A] candidate class mask
  unsigned* keyA;                // [B][cap]
  unsigned* posA;
  unsigned* keyB;
  unsigned* posB;
  long cap;
  float* out;                    // [B][max_det][6]
  int* counts;                   // [B]
  int* out_index;                // [B][max_det]  (anchor index)
};

__global__ __launch_bounds__(256) void nms_prep_kernel(NmsArgs g) {
  const int b = blockIdx.y;
  const int a = blockIdx.x * 256 + threadIdx.x;
  if (a >= g.A) return;
  float* pb = g.pred + (long)b * (4 + g.nc) * g.A + a;
  const long As = g.A;
  const float cx = pb[0], cy = pb[As], w = pb[2 * As], h = pb[3 * As];
  const float hw = w / 2.0f, hh = h / 2.0f;
  const float x1 = cx - hw, y1 = cy - hh, x2 = cx + hw, y2 = cy + hh;
  if (g.in_place) {
    pb[0] = x1;
    pb[As] = y1;
    pb[2 * As] = x2;
    pb[3 * As] = y2;
  }
  g.boxes[(long)b * g.A + a] = make_float4(x1, y1, x2, y2);
  unsigned long long mask = 0ull;
  float best = -INFINITY;
  int bj = 0;
  for (int j = 0; j < g.nc; ++j) {
    const float s = pb[(4 + j) * As];
    if (s > best) {  // strict: first maximal index wins (torch max(dim) / amax)
      best = s;
      bj = j;
    }
    if (g.multi_label && s > g.conf) mask |= 1ull << j;
  }
  if (!g.multi_label) mask = (best > g.conf) ? (1ull << bj) : 0ull;
  if (mask && g.classes) {
    unsigned long long allow = 0ull;
    for (int k = 0; k < g.n_classes; ++k) {
      const int c = g.classes[k];
      if (c >= 0 && c < 64) allow |= 1ull << c;
    }
    mask &= allow;
  }
  g.amask[(long)b * g.A + a] = mask;
}

constexpr int NMS_T = 512;  // threads per image workgroup
constexpr int NMS_W = NMS_T / 64;
constexpr int NMS_MAXDET = 1024;

__device__ __forceinline__ unsigned long long lanemask_lt() {
  const int lane = threadIdx.x & 63;
  return (lane == 0) ? 0ull : (~0ull >> (64 - lane));
}

// block-wide exclusive scan of one int per thread; returns the exclusive prefix, *total gets the sum
__device__ int block_exclusive_scan(int v, int* wsum, int* total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    int run = 0;
    for (int i = 0; i < NMS_W; ++i) {
      const int t = wsum[i];
      wsum[i] = run;
      run += t;
    }
    wsum[NMS_W] = run;
  }
  __syncthreads();
  const int ex = wsum[wv] + inc - v;
  *total = wsum[NMS_W];
  __syncthreads();
  return ex;
}

__device__ __forceinline__ bool iou_gt(const float4 bi, float ai, const float4 bj, float aj, double thr) {
  // torchvision CPU nms_kernel: i = the earlier (kept) box, j = the later one
  const float xx1 = fmaxf(bi.x, bj.x), yy1 = fmaxf(bi.y, bj.y);
  const float xx2 = fminf(bi.z, bj.z), yy2 = fminf(bi.w, bj.w);
  const float w = fmaxf(0.0f, xx2 - xx1), h = fmaxf(0.0f, yy2 - yy1);
  const float inter = w * h;
  const float ovr = inter / ((ai + aj) - inter);
  return (double)ovr > thr;
}

__global__ __launch_bounds__(NMS_T) void nms_image_kernel(NmsArgs g) {
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  __shared__ int wsum[NMS_W + 1];
  __shared__ unsigned hist[256];
  __shared__ unsigned wcnt[NMS_W][256];
  __shared__ int flag;
  __shared__ float4 kept_box[NMS_MAXDET];
  __shared__ float kept_area[NMS_MAXDET];
  __shared__ float4 cb[NMS_T];
  __shared__ float ca[NMS_T];
  __shared__ int alive[NMS_T];
  __shared__ unsigned long long rows[NMS_T][NMS_T / 64];
  __shared__ int nkept_sh, done_sh;

  const long A = g.A;
  const int nc = g.nc;
  const unsigned long long* am = g.amask + (long)b * A;
  const float* pb = g.pred + (long)b * (4 + nc) * A;
  unsigned* kA = g.keyA + (long)b * g.cap;
  unsigned* pA = g.posA + (long)b * g.cap;
  unsigned* kB = g.keyB + (long)b * g.cap;
  unsigned* pB = g.posB + (long)b * g.cap;

  // (a) ordered compaction: entries in (anchor, class) order = reference row order
  int n = 0;
  for (long t0 = 0; t0 < A; t0 += NMS_T) {
    const long a = t0 + tid;
    const unsigned long long m = (a < A) ? am[a] : 0ull;
    const int c = __popcll(m);
    int total;
    const int ex = block_exclusive_scan(c, wsum, &total);
    if (c) {
      int k = 0;
      unsigned long long mm = m;
      while (mm) {
        const int j = __ffsll((long long)mm) - 1;
        mm &= mm - 1;
        const float s = pb[(long)(4 + j) * A + a];
        kA[n + ex + k] = ~__float_as_uint(s);  // ascending ~bits == descending positive score
        pA[n + ex + k] = (unsigned)(a * nc + j);
        ++k;
      }
    }
    n += total;
  }
  __syncthreads();

  // (b) stable LSD radix sort on the 32-bit key
  unsigned *ks = kA, *ps = pA, *kd = kB, *pd = pB;
  for (int pass = 0; pass < 4 && n > 1; ++pass) {
    const int shift = pass * 8;
    __syncthreads();  // previous pass fully done with hist / flag
    if (tid < 256) hist[tid] = 0;
    if (tid == 0) flag = 0;
    __syncthreads();
    for (int i = tid; i < n; i += NMS_T) atomicAdd(&hist[(ks[i] >> shift) & 255u], 1u);
    __syncthreads();
    if (tid < 256 && hist[tid] == (unsigned)n) flag = 1;
    __syncthreads();
    if (flag) continue;  // every key has the same digit: the pass is the identity
    if (tid == 0) {
      unsigned run = 0;
      for (int d = 0; d < 256; ++d) {
        const unsigned t = hist[d];
        hist[d] = run;
        run += t;
      }
    }
    __syncthreads();
    for (int t0 = 0; t0 < n; t0 += NMS_T) {
      for (int e = tid; e < NMS_W * 256; e += NMS_T) (&wcnt[0][0])[e] = 0;
      __syncthreads();
      const int i = t0 + tid;
      const bool valid = i < n;
      const unsigned key = valid ? ks[i] : 0u;
      const unsigned pos = valid ? ps[i] : 0u;
      const unsigned d = (key >> shift) & 255u;
      unsigned long long peers = __ballot(valid);
#pragma unroll
      for (int bt = 0; bt < 8; ++bt) {
        const bool bit = (d >> bt) & 1u;
        const unsigned long long bal = __ballot(bit);
        peers &= bit ? bal : ~bal;
      }
      const unsigned long long lower = peers & lanemask_lt();
      const int rank = __popcll(lower);
      if (valid && lower == 0ull) wcnt[wv][d] = (unsigned)__popcll(peers);
      __syncthreads();
      if (tid < 256) {
        unsigned run = hist[tid];
        for (int w = 0; w < NMS_W; ++w) {
          const unsigned c = wcnt[w][tid];
          wcnt[w][tid] = run;
          run += c;
        }
        hist[tid] = run;
      }
      __syncthreads();
      if (valid) {
        const unsigned dst = wcnt[wv][d] + rank;
        kd[dst] = key;
        pd[dst] = pos;
      }
      __syncthreads();
    }
    unsigned* t;
    t = ks; ks = kd; kd = t;
    t = ps; ps = pd; pd = t;
  }
  __syncthreads();

  // (c) max_nms cut + greedy NMS with early exit at max_det kept
  const int neff = (n > g.max_nms) ? g.max_nms : n;
  const float4* bx = g.boxes + (long)b * A;
  float* ob = g.out + (long)b * g.max_det * 6;
  int* oi = g.out_index + (long)b * g.max_det;
  if (tid == 0) {
    nkept_sh = 0;
    done_sh = 0;
  }
  __syncthreads();
  for (int c0 = 0; c0 < neff; c0 += NMS_T) {
    const int i = c0 + tid;
    const bool valid = i < neff;
    unsigned pos = 0;
    float4 obox = make_float4(0, 0, 0, 0);
    float area = 0.f;
    if (valid) {
      pos = ps[i];
      const unsigned a = pos / nc, j = pos % nc;
      const float4 bb = bx[a];
      const float off = g.agnostic ? 0.0f : (float)j * g.max_wh;
      obox = make_float4(bb.x + off, bb.y + off, bb.z + off, bb.w + off);
      area = (obox.z - obox.x) * (obox.w - obox.y);
    }
    cb[tid] = obox;
    ca[tid] = area;
    const int nk = nkept_sh;
    bool al = valid;
    for (int k = 0; k < nk && al; ++k)
      if (iou_gt(kept_box[k], kept_area[k], obox, area, g.iou)) al = false;
    alive[tid] = al ? 1 : 0;
    __syncthreads();
    // in-chunk suppression rows: bit j of row t set iff t < j, both alive, IoU(t, j) > thr
#pragma unroll
    for (int wd = 0; wd < NMS_T / 64; ++wd) {
      unsigned long long bits = 0ull;
      if (al) {
        for (int q = 0; q < 64; ++q) {
          const int jj = wd * 64 + q;
          if (jj > tid && alive[jj] && iou_gt(obox, area, cb[jj], ca[jj], g.iou)) bits |= 1ull << q;
        }
      }
      rows[tid][wd] = bits;
    }
    __syncthreads();
    if (wv == 0) {
      unsigned long long removed = 0ull;  // lane wd (< 8) owns word wd
      int nkk = nk;
      const int lim = (neff - c0 < NMS_T) ? neff - c0 : NMS_T;
      bool done = false;
      for (int t = 0; t < lim && !done; ++t) {
        if (!alive[t]) continue;
        const unsigned long long word = __shfl(removed, t >> 6, 64);
        if ((word >> (t & 63)) & 1ull) continue;
        // keep t
        if (lane == 0) {
          kept_box[nkk] = cb[t];
          kept_area[nkk] = ca[t];
          const unsigned p = ps[c0 + t];
          const unsigned a = p / nc, j = p % nc;
          const float4 bb = bx[a];
          float* o = ob + (long)nkk * 6;
          o[0] = bb.x; o[1] = bb.y; o[2] = bb.z; o[3] = bb.w;
          o[4] = pb[(long)(4 + j) * A + a];
          o[5] = (float)j;
          oi[nkk] = (int)a;
        }
        ++nkk;
        if (nkk >= g.max_det) done = true;
        if (lane < NMS_T / 64) removed |= rows[t][lane];
      }
      if (lane == 0) {
        nkept_sh = nkk;
        done_sh = done ? 1 : 0;
      }
    }
    __syncthreads();
    if (done_sh) break;
  }
  __syncthreads();
  const int nk = nkept_sh;
  for (int e = nk * 6 + tid; e < g.max_det * 6; e += NMS_T) ob[e] = 0.f;
  for (int e = nk + tid; e < g.max_det; e += NMS_T) oi[e] = -1;
  if (tid == 0) g.counts[b] = nk;
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

YS_EXPORT int yolosod_detect_head(int nl, const float* const* box_feat, const float* const* cls_feat, int c2, int c3,
                                  const float* const* box_w, const float* const* box_b, const float* const* cls_w,
                                  const float* const* cls_b, const int* heights, const int* widths,
                                  const float* strides, int B, int nc, int reg_max, float* y, void* stream) {
  YS_CHECK_ARG(nl >= 1 && nl <= 4, "detect_head: nl=%d unsupported (1..4)", nl);
  YS_CHECK_ARG(box_feat && cls_feat && box_w && box_b && cls_w && cls_b && heights && widths && strides && y,
               "detect_head: null pointer");
  YS_CHECK_ARG(reg_max == 16, "detect_head: reg_max=%d unsupported (16)", reg_max);
  YS_CHECK_ARG(nc >= 1 && nc <= 16, "detect_head: nc=%d unsupported (1..16)", nc);
  YS_CHECK_ARG(c2 == 64 && (c3 == 64 || c3 == 128), "detect_head: (c2=%d, c3=%d) unsupported ((64, 64|128))", c2, c3);
  HeadArgs d{};
  d.nl = nl;
  d.nc = nc;
  constexpr int NTS = 8;  // 16-pixel groups per wave -> 512 pixels per workgroup
  int off = 0, blk = 0;
  for (int i = 0; i < nl; ++i) {
    YS_CHECK_ARG(box_feat[i] && cls_feat[i] && box_w[i] && box_b[i] && cls_w[i] && cls_b[i],
                 "detect_head: null pointer at level %d", i);
    d.fb[i] = box_feat[i];
    d.fc[i] = cls_feat[i];
    d.wb[i] = box_w[i];
    d.bb[i] = box_b[i];
    d.wc[i] = cls_w[i];
    d.bc[i] = cls_b[i];
    d.hw[i] = heights[i] * widths[i];
    d.w[i] = widths[i];
    d.stride[i] = strides[i];
    d.a_off[i] = off;
    d.blk_off[i] = blk;
    off += d.hw[i];
    blk += (d.hw[i] + 4 * NTS * 16 - 1) / (4 * NTS * 16);
  }
  d.blk_off[nl] = blk;
  d.A = off;
  d.y = y;
  if (B == 0 || off == 0) return 0;
  const dim3 grid(blk, B);
  if (c3 == 64)
    hipLaunchKernelGGL((detect_head_kernel<64, 64, NTS>), grid, dim3(256), 0, (hipStream_t)stream, d);
  else
    hipLaunchKernelGGL((detect_head_kernel<64, 128, NTS>), grid, dim3(256), 0, (hipStream_t)stream, d);
  YS_CHECK_LAUNCH("detect_head");
  return 0;
}

static long nms_cap(int nc, int A, int multi_label) { return (long)A * (multi_label ? nc : 1); }

YS_EXPORT size_t yolosod_nms_workspace(int B, int nc, int A, int multi_label) {
  const long cap = nms_cap(nc, A, multi_label);
  Sizer s;
  s.take<float4>((size_t)B * A);
  s.take<unsigned long long>((size_t)B * A);
  for (int i = 0; i < 4; ++i) s.take<unsigned>((size_t)B * cap);
  return s.off;
}

YS_EXPORT int yolosod_nms(float* pred, int B, int nc, int A, float conf_thres, double iou_thres, const int* classes,
                          int n_classes, int agnostic, int multi_label, int max_det, int max_nms, float max_wh,
                          int in_place, float* out, int* counts, int* out_index, void* workspace,
                          size_t workspace_bytes, void* stream) {
  YS_CHECK_ARG(pred && out && counts && out_index, "nms: null pointer");
  YS_CHECK_ARG(nc >= 1 && nc <= 64, "nms: nc=%d unsupported (1..64)", nc);
  YS_CHECK_ARG(max_det >= 1 && max_det <= NMS_MAXDET, "nms: max_det=%d unsupported (1..%d)", max_det, NMS_MAXDET);
  YS_CHECK_ARG(max_nms >= 0, "nms: bad max_nms");
  YS_CHECK_ARG((long)A * nc < (1L << 32), "nms: A*nc too large");
  if (B == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const long cap = nms_cap(nc, A, multi_label);
  Carver cv(workspace, workspace_bytes);
  NmsArgs g{};
  g.pred = pred;
  g.B = B;
  g.nc = nc;
  g.A = A;
  g.conf = conf_thres;
  g.iou = iou_thres;
  g.classes = (n_classes > 0) ? classes : nullptr;
  g.n_classes = n_classes;
  g.agnostic = agnostic;
  g.multi_label = multi_label;
  g.max_det = max_det;
  g.max_nms = max_nms;
  g.in_place = in_place;
  g.max_wh = max_wh;
  g.boxes = cv.take<float4>((size_t)B * A);
  g.amask = cv.take<unsigned long long>((size_t)B * A);
  g.keyA = cv.take<unsigned>((size_t)B * cap);
  g.posA = cv.take<unsigned>((size_t)B * cap);
  g.keyB = cv.take<unsigned>((size_t)B * cap);
  g.posB = cv.take<unsigned>((size_t)B * cap);
  YS_CHECK_ARG(g.posB, "nms: workspace too small (%zu)", workspace_bytes);
  g.cap = cap;
  g.out = out;
  g.counts = counts;
  g.out_index = out_index;
  if (A > 0) hipLaunchKernelGGL(nms_prep_kernel, dim3((A + 255) / 256, B), dim3(256), 0, st, g);
  hipLaunchKernelGGL(nms_image_kernel, dim3(B), dim3(NMS_T), 0, st, g);
  YS_CHECK_LAUNCH("nms");
  return 0;
}
