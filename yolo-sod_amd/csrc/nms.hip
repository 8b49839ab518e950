// Class-wise greedy NMS on gfx950, bit-exact with the reference (compile with -ffp-contract=off).
//
// Reference semantics: non_max_suppression ultralytics/utils/ops.py:167-316 (xywh2xyxy :416-434) around
// torchvision==0.20.1 ops.nms (CPU kernel: stable descending score sort, strict IoU > thr, area without +1);
// classes are separated by offsetting boxes with cls * max_wh (ops.py:289,295).
//
// Design (no host sync; the per-image candidate count lives on the device):
//   nms_prep    one thread per anchor: xywh -> xyxy (optionally in place, as the reference mutates its input),
//               candidate class mask (score > conf, class filter, best class or multi-label), and the candidate
//               count of each 256-anchor block.
//   nms_scatter order-preserving compaction of the (anchor, class) candidates (= the reference's row order) over
//               the whole GPU: each block sums its image's preceding block counts for its offset and scatters
//               (~score bits, anchor*nc+class).
//   nms_select  one 512-thread workgroup per image: the score order of the first <= KCAP candidates, sorted in
//               LDS. For n <= KCAP a stable LSD radix sort of all; for n > KCAP a radix *select* first finds the
//               key T such that the keys below T (at most KCAP of them) are exactly a prefix of the stable sorted
//               order (keys held in registers for n <= 36864, common digits skipped, bank-replicated histograms),
//               and only that prefix is sorted. Writes the prefix's class-offset boxes / areas / ids.
//   nms_mask    one wave per (row block, column block) pair of the upper triangle (528 equal tasks per image): the
//               IoU > thr bitmask of the prefix, one 64-bit word per (row, 64-column block).
//   nms_resolve one workgroup per image: greedy in score order over the bitmask, 64 rows staged in LDS at a time,
//               only alive candidates visited (bit scan); stops at max_det. Only if the prefix is exhausted before
//               max_det boxes are kept and more candidates exist (keys >= T) does it sort that remainder and
//               continue with the chunked in-LDS greedy (each chunk of 512 tested against the kept boxes, then
//               its own IoU bitmask). Kept rows are written in parallel.
#include "common.h"
#include <math.h>
#include <stdlib.h>

namespace ys {

constexpr int NMS_T = 512;  // threads per image workgroup
constexpr int NMS_W = NMS_T / 64;
constexpr int NMS_MAXDET = 1024;     // kept lists up to this length live in LDS; longer ones in the workspace
constexpr int NMS_MAXDET_BIG = 1 << 20;
constexpr int KCAP = 2048;  // candidates covered by the multi-CU IoU bitmask
constexpr int KW = KCAP / 64;
static_assert(KW == 32, "nms_resolve maps one 32-word mask row onto 32 threads");
constexpr int RK = 72;      // keys per thread nms_select holds in registers: n <= NMS_T * RK (A = 34000 single-label)

#ifdef YS_DIAG_STAMPS  // diagnostic builds only (scripts/diag_nms.sh): s_memtime of thread 0 at phase boundaries
__device__ unsigned long long g_nms_stamps[32 * 24];
#define YS_NSTAMP(k) \
  if (threadIdx.x == 0 && blockIdx.x < 32) g_nms_stamps[blockIdx.x * 24 + (k)] = __builtin_amdgcn_s_memtime();
#else
#define YS_NSTAMP(k) ;  // a statement in both builds (never the body of an if)
#endif

struct NmsArgs {
  float* pred;  // [B][4+nc][A]
  int B, nc, A;
  float conf;
  double iou;
  float iou_f;     // the largest float <= iou: for a float ratio r, (double)r > iou <=> r > iou_f (no f64 compare)
  const int* classes;
  int n_classes;
  int agnostic, multi_label, max_det, max_nms, in_place;
  float max_wh;
  float4* boxes;                 // [B][A] xyxy
  unsigned long long* amask;     // [B][A] candidate class mask
  unsigned* keyA;                // [B][cap] compaction output (kept for the fallback)
  unsigned* posA;
  unsigned* keyB;                // [B][cap] scratch
  unsigned* posB;
  long cap;
  float4* sbox;                  // [B][KCAP] score-ordered prefix: class-offset boxes
  float* sarea;                  // [B][KCAP]
  unsigned* spos;                // [B][KCAP] anchor * nc + class
  unsigned long long* mask;      // [B][KCAP][KW]
  int* meta;                     // [B][4]: n, neff, K (prefix length), T (prefix = keys < T)
  int* blkcnt;                   // [B][nblk_a] candidates per 256-anchor block (prep), then exclusive offsets
  float* out;                    // [B][max_det][6]
  int* counts;                   // [B]
  int* out_index;                // [B][max_det]  (anchor index)
  int* kept_t;                   // [B][max_det] kept entries when max_det > NMS_MAXDET (else LDS), else nullptr
  float4* kbox;                  // [B][max_det] kept class-offset boxes (fallback), idem
  float* karea;                  // [B][max_det]
};


__device__ __forceinline__ int block256_exclusive_scan(int v, int* wsum4, int* total);

// also the candidate count of this 256-anchor block (the ordered compaction's per-block counts). Only candidate
// anchors' xyxy boxes are stored (every later reader indexes candidates), and the block's candidate masks only when
// it has any (nms_scatter skips blocks whose count is 0): an image without candidates costs the read of its scores
// plus the in-place rewrite the reference's in_place=True asks for.
__global__ __launch_bounds__(256) void nms_prep_kernel(NmsArgs g) {
  __shared__ int wsum4[4];
  const int b = blockIdx.y;
  const int a = blockIdx.x * 256 + threadIdx.x;
  unsigned long long mask = 0ull;
  float4 box = make_float4(0.f, 0.f, 0.f, 0.f);
  if (a < g.A) {
    float* pb = g.pred + (long)b * (4 + g.nc) * g.A + a;
    const long As = g.A;
    // the class scores first (up to 16 loaded unconditionally, class index clamped; classes past nc skipped), then
    // the box: every anchor's when the reference's in-place xyxy rewrite is asked for, else only a candidate's (the
    // predictor's call: an empty image reads its scores only, 10 of the 14 rows)
    float s16[16];
    if (g.nc <= 16) {
#pragma unroll
      for (int u = 0; u < 16; ++u) s16[u] = pb[(4 + (u < g.nc ? u : g.nc - 1)) * As];
    }
    float best = -INFINITY;
    int bj = 0;
    if (g.nc <= 16) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        if (j < g.nc) {
          const float sc = s16[j];
          if (sc > best) {  // strict: first maximal index wins (torch max(dim) / amax)
            best = sc;
            bj = j;
          }
          if (g.multi_label && sc > g.conf) mask |= 1ull << j;
        }
      }
    }
    for (int j0 = 0; g.nc > 16 && j0 < g.nc; j0 += 8) {  // 8 score loads in flight, then scanned in class order
      float sv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) sv[u] = (j0 + u < g.nc) ? pb[(4 + j0 + u) * As] : -INFINITY;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int j = j0 + u;
        if (j < g.nc) {
          const float s = sv[u];
          if (s > best) {  // strict: first maximal index wins (torch max(dim) / amax)
            best = s;
            bj = j;
          }
          if (g.multi_label && s > g.conf) mask |= 1ull << j;
        }
      }
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
    if (g.in_place || mask) {
      const float cx = pb[0], cy = pb[As], w = pb[2 * As], h = pb[3 * As];
      const float hw = w / 2.0f, hh = h / 2.0f;
      const float x1 = cx - hw, y1 = cy - hh, x2 = cx + hw, y2 = cy + hh;
      if (g.in_place) {
        pb[0] = x1;
        pb[As] = y1;
        pb[2 * As] = x2;
        pb[3 * As] = y2;
      }
      box = make_float4(x1, y1, x2, y2);
    }
  }
  int total;
  (void)block256_exclusive_scan(__popcll(mask), wsum4, &total);
  if (threadIdx.x == 0) g.blkcnt[(long)b * gridDim.x + blockIdx.x] = total;
  if (total != 0 && a < g.A) {
    g.amask[(long)b * g.A + a] = mask;
    if (mask) g.boxes[(long)b * g.A + a] = box;
  }
}

// block-wide (256 threads) exclusive scan; returns the exclusive prefix, *total gets the block sum
__device__ __forceinline__ int block256_exclusive_scan(int v, int* wsum4, int* total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) wsum4[wv] = inc;
  __syncthreads();
  int base = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) base += (w < wv) ? wsum4[w] : 0;
  *total = wsum4[0] + wsum4[1] + wsum4[2] + wsum4[3];
  return base + inc - v;
}

// ordered scatter: entry (anchor, class) in (anchor, class) order = the reference's row order; each block sums its
// image's preceding block counts itself (no separate scan launch)
__global__ __launch_bounds__(256) void nms_scatter_kernel(NmsArgs g) {
  __shared__ int wsum4[4];
  const int b = blockIdx.y;
  const long A = g.A;
  const long a = (long)blockIdx.x * 256 + threadIdx.x;
  // this block's output offset: the candidates of the image's preceding blocks (their counts from nms_prep)
  const int* bc = g.blkcnt + (long)b * gridDim.x;
  if (bc[blockIdx.x] == 0) return;  // no candidates here (nms_prep did not store this block's masks)
  const unsigned long long m = (a < A) ? g.amask[(long)b * A + a] : 0ull;
  int before = 0;
  for (int i = threadIdx.x; i < (int)blockIdx.x; i += 256) before += bc[i];
  int base;
  (void)block256_exclusive_scan(before, wsum4, &base);
  __syncthreads();  // wsum4 is reused by the scan below
  int total;
  const int ex = block256_exclusive_scan(__popcll(m), wsum4, &total);
  if (!m) return;
  int k = base + ex;
  const float* pb = g.pred + (long)b * (4 + g.nc) * A + a;
  unsigned* kA = g.keyA + (long)b * g.cap;
  unsigned* pA = g.posA + (long)b * g.cap;
  for (int j = 0; j < g.nc; ++j)
    if ((m >> j) & 1ull) {
      kA[k] = ~__float_as_uint(pb[(long)(4 + j) * A]);  // ascending ~bits == descending positive score
      pA[k] = (unsigned)(a * g.nc + j);
      ++k;
    }
}

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

// thr_f: the largest float <= the double threshold (NmsArgs::iou_f), so `ovr > thr_f` is exactly the reference's
// `(double)ovr > thr` for every float ovr (NaN included) without an f64 conversion and compare
__device__ __forceinline__ bool iou_gt(const float4 bi, float ai, const float4 bj, float aj, float thr_f) {
  // torchvision CPU nms_kernel: i = the earlier (kept) box, j = the later one
  const float xx1 = fmaxf(bi.x, bj.x), yy1 = fmaxf(bi.y, bj.y);
  const float xx2 = fminf(bi.z, bj.z), yy2 = fminf(bi.w, bj.w);
  const float w = fmaxf(0.0f, xx2 - xx1), h = fmaxf(0.0f, yy2 - yy1);
  const float inter = w * h;
  const float ovr = inter / ((ai + aj) - inter);
  return ovr > thr_f;
}

// iou_gt with the division skipped where it cannot matter: inter is >= 0 or NaN (w, h >= 0), and with inter not
// > 0 the ratio is +-0 or NaN, which is > thr for no thr >= 0 (the reference asserts 0 <= iou_thres). all_pairs
// (thr < 0) keeps every division. Same operations in the same order as iou_gt where it divides: bit-identical.
__device__ __forceinline__ bool iou_gt_sparse(const float4 bi, float ai, const float4 bj, float aj, float thr_f,
                                              bool all_pairs) {
  const float xx1 = fmaxf(bi.x, bj.x), yy1 = fmaxf(bi.y, bj.y);
  const float xx2 = fminf(bi.z, bj.z), yy2 = fminf(bi.w, bj.w);
  const float w = fmaxf(0.0f, xx2 - xx1), h = fmaxf(0.0f, yy2 - yy1);
  const float inter = w * h;
  bool hit = false;
  // divergent branch: a wave divides only if one of its pairs overlaps (a cheaper xx2 > xx1 && yy2 > yy1 pre-test
  // in front of w, h and inter measured 24 % slower: one more divergent branch per pair)
  if (inter > 0.0f || all_pairs) {
    const float ovr = inter / ((ai + aj) - inter);
    hit = ovr > thr_f;
  }
  return hit;
}

// hist[d] += 1 for every lane with valid (wave-uniform call)
__device__ __forceinline__ void hist_add_digit(unsigned* hist, unsigned d, bool valid) {
  const unsigned long long act = __ballot(valid);
  if (act == 0ull) return;
  // common case (score keys share their top digits): every valid lane has the leader's digit, one atomic
  const int leader = __builtin_amdgcn_readfirstlane(__ffsll((long long)act) - 1);
  const unsigned dl = __builtin_amdgcn_readlane(d, leader);
  if (__ballot(valid && d != dl) == 0ull) {
    if ((int)(threadIdx.x & 63) == leader) atomicAdd(&hist[dl], (unsigned)__popcll(act));
    return;
  }
  // mixed digits: plain per-lane atomics (the LDS serialises only lanes that share an address; grouping equal
  // digits by 8 ballots first cost more VALU work than the conflicts it avoids)
  if (valid) atomicAdd(&hist[d], 1u);
}


// exclusive scan of hist[0..256) in place by the first 256 threads of the (512-thread) block; returns nothing,
// block-uniform (contains barriers). tmp: 4 words.
__device__ void scan256_exclusive(unsigned* hist, unsigned* tmp) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  unsigned v = 0, inc = 0;
  if (tid < 256) {
    v = hist[tid];
    inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
    if (lane == 63) tmp[wv] = inc;
  }
  __syncthreads();
  if (tid < 256) {
    unsigned base = 0;
    for (int w = 0; w < wv; ++w) base += tmp[w];
    hist[tid] = base + inc - v;
  }
  __syncthreads();
}

struct SortShared {
  unsigned hist[256];
  unsigned wcnt[NMS_W][256];
  int flag;
  int wsum[NMS_W + 1];
  unsigned tmp4[4];
};

// One stable scatter of n (key, pos) pairs by the 8-bit digit at `shift` from (ks, ps) to (kd, pd), 512 pairs per
// step; sh.hist holds the digit's exclusive prefix on entry (the digit's end offsets on return). Block-uniform.
__device__ void radix_scatter(const unsigned* ks, const unsigned* ps, unsigned* kd, unsigned* pd, int n, int shift,
                              SortShared& sh) {
  const int tid = threadIdx.x, wv = tid >> 6;
  for (int t0 = 0; t0 < n; t0 += NMS_T) {
    for (int e = tid; e < NMS_W * 256; e += NMS_T) (&sh.wcnt[0][0])[e] = 0;
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
    if (valid && lower == 0ull) sh.wcnt[wv][d] = (unsigned)__popcll(peers);
    __syncthreads();
    if (tid < 256) {
      unsigned run = sh.hist[tid];
      for (int w = 0; w < NMS_W; ++w) {
        const unsigned c = sh.wcnt[w][tid];
        sh.wcnt[w][tid] = run;
        run += c;
      }
      sh.hist[tid] = run;
    }
    __syncthreads();
    if (valid) {
      const unsigned dst = sh.wcnt[wv][d] + rank;
      kd[dst] = key;
      pd[dst] = pos;
    }
    __syncthreads();
  }
}

// Stable LSD radix sort (4 x 8-bit digits, ascending) of n (key, pos) pairs, ping-ponging between (ks, ps) and
// (kd, pd); on return (ks, ps) hold the sorted pairs. Passes whose digit is uniform are skipped. Block-uniform.
__device__ __forceinline__ void radix_sort_pairs(unsigned*& ks, unsigned*& ps, unsigned*& kd, unsigned*& pd, int n, SortShared& sh) {
  const int tid = threadIdx.x;
  for (int pass = 0; pass < 4 && n > 1; ++pass) {
    const int shift = pass * 8;
    __syncthreads();  // previous pass fully done with hist / flag
    if (tid < 256) sh.hist[tid] = 0;
    if (tid == 0) sh.flag = 0;
    __syncthreads();
    for (int i0 = 0; i0 < n; i0 += NMS_T) {
      const int i = i0 + tid;
      hist_add_digit(sh.hist, (i < n) ? (ks[i] >> shift) & 255u : 0u, i < n);
    }
    __syncthreads();
    if (tid < 256 && sh.hist[tid] == (unsigned)n) sh.flag = 1;
    __syncthreads();
    if (sh.flag) continue;  // every key has the same digit: the pass is the identity
    scan256_exclusive(sh.hist, sh.tmp4);
    radix_scatter(ks, ps, kd, pd, n, shift, sh);
    unsigned* t;
    t = ks; ks = kd; kd = t;
    t = ps; ps = pd; pd = t;
  }
  __syncthreads();
}

// Stable LSD radix sort of n <= KCAP (key, pos) pairs in LDS, as radix_sort_pairs but one counting step per digit
// pass: wave w owns pairs [256 w, 256 w + 256) (four rounds of 64 lanes, in index order), ranks each round's keys by
// matching digits (8 ballots) on top of its running per-digit counts, and one prefix over the 8 waves per digit
// (wave order = index order) gives every pair its destination. radix_sort_pairs works in 512-pair chunks, each with
// its own four barriers and an 8-step serial prefix per digit (~32k cycles for 2048 pairs). Block-uniform.
__device__ __forceinline__ void radix_sort_lds(unsigned*& ks, unsigned*& ps, unsigned*& kd, unsigned*& pd, int n, SortShared& sh) {
  static_assert(KCAP == NMS_W * 256, "one 256-pair range per wave");
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int pass = 0; pass < 4 && n > 1; ++pass) {
    const int shift = pass * 8;
    for (int e = tid; e < NMS_W * 256; e += NMS_T) (&sh.wcnt[0][0])[e] = 0;
    __syncthreads();
    unsigned key[4], pos[4], dg[4];
    int lr[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = wv * 256 + r * 64 + lane;
      const bool valid = i < n;
      key[r] = valid ? ks[i] : 0u;
      pos[r] = valid ? ps[i] : 0u;
      const unsigned d = (key[r] >> shift) & 255u;
      dg[r] = d;
      unsigned long long peers = __ballot(valid);
#pragma unroll
      for (int bt = 0; bt < 8; ++bt) {
        const bool bit = (d >> bt) & 1u;
        const unsigned long long bal = __ballot(bit);
        peers &= bit ? bal : ~bal;
      }
      const unsigned long long lower = peers & lanemask_lt();
      lr[r] = valid ? (int)sh.wcnt[wv][d] + __popcll(lower) : 0;  // the wave's earlier rounds + earlier lanes
      // same-wave LDS accesses complete in order: every lane's read above precedes the leader's update
      if (valid && lower == 0ull) sh.wcnt[wv][d] += (unsigned)__popcll(peers);
    }
    __syncthreads();
    if (tid < 256) {  // per digit: exclusive offsets over the waves (index order), total into hist
      unsigned run = 0;
#pragma unroll
      for (int w = 0; w < NMS_W; ++w) {
        const unsigned c = sh.wcnt[w][tid];
        sh.wcnt[w][tid] = run;
        run += c;
      }
      sh.hist[tid] = run;
    }
    if (tid == 0) sh.flag = 0;
    __syncthreads();
    if (tid < 256 && sh.hist[tid] == (unsigned)n) sh.flag = 1;
    __syncthreads();
    if (sh.flag) continue;  // every key has the same digit: the pass is the identity
    scan256_exclusive(sh.hist, sh.tmp4);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = wv * 256 + r * 64 + lane;
      if (i < n) {
        const unsigned dst = sh.hist[dg[r]] + sh.wcnt[wv][dg[r]] + (unsigned)lr[r];
        kd[dst] = key[r];
        pd[dst] = pos[r];
      }
    }
    __syncthreads();
    unsigned* t;
    t = ks; ks = kd; kd = t;
    t = ps; ps = pd; pd = t;
  }
  __syncthreads();
}

// Order-preserving compaction of the pairs whose key is < T (below) or >= T (!below) into (kd, pd); returns
// the count. Block-uniform.
__device__ int compact_range(const unsigned* ks, const unsigned* ps, int n, unsigned lo, unsigned long long hi,
                             unsigned* kd, unsigned* pd, SortShared& sh) {
  // order-preserving compaction of the pairs with lo <= key < hi (hi up to 2^32)
  constexpr int CPT = 4;
  const int tid = threadIdx.x;
  int m = 0;
  for (int t0 = 0; t0 < n; t0 += NMS_T * CPT) {
    const int i0 = t0 + tid * CPT;
    unsigned k[CPT], p[CPT];
    int c = 0;
#pragma unroll
    for (int u = 0; u < CPT; ++u) {
      const bool v = i0 + u < n;
      k[u] = v ? ks[i0 + u] : 0u;
      p[u] = v ? ps[i0 + u] : 0u;
      const bool take = v && k[u] >= lo && (unsigned long long)k[u] < hi;
      c += take ? 1 : 0;
      if (!take) k[u] = 0u, p[u] = 0xFFFFFFFFu;
    }
    int total;
    const int ex = block_exclusive_scan(c, sh.wsum, &total);
    int o = m + ex;
#pragma unroll
    for (int u = 0; u < CPT; ++u)
      if (p[u] != 0xFFFFFFFFu) {
        kd[o] = k[u];
        pd[o] = p[u];
        ++o;
      }
    m += total;
  }
  return m;
}

__device__ int compact_by_key(const unsigned* ks, const unsigned* ps, int n, unsigned T, bool below, unsigned* kd,
                              unsigned* pd, SortShared& sh) {
  return below ? compact_range(ks, ps, n, 0u, T, kd, pd, sh) : compact_range(ks, ps, n, T, 1ull << 32, kd, pd, sh);
}

// -------------------------------------------------------------------------------------------------
// nms_select: compaction + score order of the first <= KCAP candidates (see header)
// -------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(NMS_T) void nms_select_kernel(NmsArgs g) {
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  __shared__ SortShared sh;
  __shared__ unsigned sel_below, sel_prefix;
  const long A = g.A;
  const int nc = g.nc;
  unsigned* kA = g.keyA + (long)b * g.cap;
  unsigned* pA = g.posA + (long)b * g.cap;
  unsigned* kB = g.keyB + (long)b * g.cap;
  unsigned* pB = g.posB + (long)b * g.cap;

  YS_NSTAMP(0)
  // (a) the ordered compaction ran over the whole GPU (nms_prep counts, nms_scatter); n = the image's candidates
  __shared__ int nsum[NMS_W + 1];
  int n;
  {
    const int nblk = (int)((A + 255) / 256);
    int v = 0;
    for (int i = tid; i < nblk; i += NMS_T) v += g.blkcnt[(long)b * nblk + i];
    (void)block_exclusive_scan(v, nsum, &n);
  }
  const int neff = (n > g.max_nms) ? g.max_nms : n;
  YS_NSTAMP(1)

  // (b) score order of the prefix
  unsigned *ks, *ps, *kd, *pd;
  unsigned T = 0xFFFFFFFFu;
  int m;
  __shared__ unsigned lk[2][KCAP], lp[2][KCAP];  // the prefix is sorted in LDS
  if (n <= KCAP) {
    for (int i = tid; i < n; i += NMS_T) {
      lk[0][i] = kA[i];
      lp[0][i] = pA[i];
    }
    ks = lk[0]; ps = lp[0]; kd = lk[1]; pd = lp[1];
    radix_sort_lds(ks, ps, kd, pd, n, sh);
    m = n;
  } else if (n <= NMS_T * RK) {
    // the same radix select with the keys held in registers: one read of the keys instead of one per pass, and a
    // single ordered compaction. Wave w holds keys [w RK 64, (w + 1) RK 64), lane l the keys w RK 64 + 64 u + l:
    // each load instruction reads 64 consecutive keys (thread-contiguous runs of 72 keys made every 16-byte load
    // touch 64 cache lines: 17 us of key loads at 30k candidates)
    const int lane = tid & 63, wv = tid >> 6;
    const int wbase = wv * RK * 64;
    unsigned kr[RK];
    // every load unconditional (a clamped index; entries past n masked afterwards), so all of a thread's loads
    // are in flight together (loads under a bounds branch were merged into phis that each waited for the memory)
#pragma unroll
    for (int u = 0; u < RK; ++u) kr[u] = kA[min(wbase + 64 * u + lane, n - 1)];
#pragma unroll
    for (int u = 0; u < RK; ++u)
      if (wbase + 64 * u + lane >= n) kr[u] = 0xFFFFFFFFu;
    // digits above the highest bit in which two keys differ are common to all keys: their passes would find one
    // bucket holding all n (> KCAP) keys and only extend the prefix, so the select starts below them (the same T)
    // Entries past n hold 0xFFFFFFFF, the largest key: counted in the histograms they only add to the top bucket,
    // which never moves the crossing digit (n > KCAP valid keys cross at or below it), and `key < T` never takes
    // them; so no per-entry validity test is needed below (72 of them kept live spilled the SGPRs). kmax excludes
    // them, unless a valid key is 0xFFFFFFFF itself (a score of +0 with conf < 0): then no digit is skipped.
    unsigned kmin = 0xFFFFFFFFu, kmax = 0u;
    int nff = 0;
#pragma unroll
    for (int u = 0; u < RK; ++u) {
      kmin = min(kmin, kr[u]);
      if (kr[u] != 0xFFFFFFFFu) kmax = max(kmax, kr[u]);
      nff += (kr[u] == 0xFFFFFFFFu) ? 1 : 0;
    }
    if (nff > RK - max(0, min(RK, (n - wbase - lane + 63) / 64))) kmax = 0xFFFFFFFFu;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      kmin = min(kmin, (unsigned)__shfl_xor((int)kmin, o, 64));
      kmax = max(kmax, (unsigned)__shfl_xor((int)kmax, o, 64));
    }
    __shared__ unsigned kminmax[2];
    if (tid == 0) {
      kminmax[0] = 0xFFFFFFFFu;
      kminmax[1] = 0u;
    }
    __syncthreads();
    if ((tid & 63) == 0) {
      atomicMin(&kminmax[0], kmin);
      atomicMax(&kminmax[1], kmax);
    }
    __syncthreads();
    kmin = kminmax[0];
    kmax = kminmax[1];
    const unsigned diff = kmin ^ kmax;
    unsigned prefix = kmin, below = 0u;  // all keys equal: none is below T = that key
    YS_NSTAMP(2)
    if (diff != 0u) {
      const int top = ((31 - __clz(diff)) / 8) * 8;  // shift of the digit holding the highest differing bit
      unsigned pmask = (top == 24) ? 0u : (0xFFFFFFFFu << (top + 8));
      prefix = kmin & pmask;
      // 32 replicas of the histogram, replica r in LDS bank r: lane l adds into replica l & 31, so the 32 lanes an
      // LDS atomic serves per cycle never share a bank. (One shared histogram: random digits over 256 bins put ~5
      // lanes in one bank and each ds_add took ~100 cycles - 56k cycles for the first pass at 30k keys.)
      __shared__ unsigned hrep[256 * 32];
      for (int shift = top; shift >= 0; shift -= 8) {
        for (int e = tid; e < 256 * 32; e += NMS_T) hrep[e] = 0;
        __syncthreads();
#pragma unroll
        for (int u = 0; u < RK; ++u)
          if ((kr[u] & pmask) == prefix) atomicAdd(&hrep[(((kr[u] >> shift) & 255u) << 5) | (lane & 31)], 1u);
        __syncthreads();
        unsigned h = 0u;
        if (tid < 256) {
#pragma unroll
          for (int r = 0; r < 32; ++r) h += hrep[(tid << 5) | ((r + tid) & 31)];  // rotated: conflict-free reads
          sh.hist[tid] = h;
        }
        scan256_exclusive(sh.hist, sh.tmp4);
        if (tid < 256) {
          const unsigned run = below + sh.hist[tid];
          if (run <= (unsigned)KCAP && run + h > (unsigned)KCAP) {
            sel_below = run;
            sel_prefix = prefix | ((unsigned)tid << shift);
          }
        }
        __syncthreads();
        below = sel_below;
        prefix = sel_prefix;
        pmask |= 255u << shift;
        __syncthreads();
        YS_NSTAMP(16 + shift / 8)
      }
    }
    T = prefix;
    YS_NSTAMP(3)
    // ordered compaction of the keys < T: wave order is (u, lane), the waves' ranges follow each other
    int wt = 0;
#pragma unroll
    for (int u = 0; u < RK; ++u) wt += __popcll(__ballot(kr[u] < T));
    __shared__ int wtot[NMS_W];
    if (lane == 0) wtot[wv] = wt;
    __syncthreads();
    int o = 0;
    m = 0;
#pragma unroll
    for (int w = 0; w < NMS_W; ++w) {
      o += (w < wv) ? wtot[w] : 0;
      m += wtot[w];
    }
#pragma unroll
    for (int u = 0; u < RK; ++u) {
      const bool take = kr[u] < T;
      const unsigned long long bal = __ballot(take);
      if (take) {
        const int idx = o + __popcll(bal & lanemask_lt());
        lk[0][idx] = kr[u];
        lp[0][idx] = (unsigned)(wbase + 64 * u + lane);  // index into the compaction; its position is gathered below
      }
      o += __popcll(bal);
    }
    __syncthreads();
    for (int i = tid; i < m; i += NMS_T) lp[0][i] = pA[lp[0][i]];
    __syncthreads();
    YS_NSTAMP(4)
    ks = lk[0]; ps = lp[0]; kd = lk[1]; pd = lp[1];
    radix_sort_lds(ks, ps, kd, pd, m, sh);
  } else {
    // radix select, MSB first: the key T with #(key < T) <= KCAP, taking whole digit buckets while they fit
    unsigned prefix = 0u, pmask = 0u;
    unsigned below = 0u;
    for (int pass = 0; pass < 4; ++pass) {
      const int shift = 24 - 8 * pass;
      if (tid < 256) sh.hist[tid] = 0;
      __syncthreads();
      // 8 key loads in flight per thread; equal digits grouped per wave (the top digits of score keys are nearly
      // all equal: one LDS atomic per wave and digit, not one per key)
      for (int i0 = 0; i0 < n; i0 += NMS_T * 8) {
        unsigned kk[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int i = i0 + u * NMS_T + tid;
          kk[u] = (i < n) ? kA[i] : 0u;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int i = i0 + u * NMS_T + tid;
          hist_add_digit(sh.hist, (kk[u] >> shift) & 255u, i < n && (kk[u] & pmask) == prefix);
        }
      }
      __syncthreads();
      // the digit d where the running count crosses KCAP: below + excl[d] <= KCAP < below + excl[d] + hist[d]
      // (unique; it exists because the keys under the current prefix do not all fit, else the previous pass
      // would have taken that whole bucket)
      const unsigned h = (tid < 256) ? sh.hist[tid] : 0u;
      scan256_exclusive(sh.hist, sh.tmp4);
      if (tid < 256) {
        const unsigned run = below + sh.hist[tid];
        if (run <= (unsigned)KCAP && run + h > (unsigned)KCAP) {
          sel_below = run;
          sel_prefix = prefix | ((unsigned)tid << shift);
        }
      }
      __syncthreads();
      below = sel_below;
      prefix = sel_prefix;
      pmask |= 255u << shift;
      __syncthreads();  // sel_* and hist are rewritten by the next pass
    }
    T = prefix;  // keys < T: exactly `below` of them, a prefix of the stable ascending order
    m = compact_by_key(kA, pA, n, T, true, lk[0], lp[0], sh);
    __syncthreads();
    ks = lk[0]; ps = lp[0]; kd = lk[1]; pd = lp[1];
    radix_sort_lds(ks, ps, kd, pd, m, sh);
  }
  YS_NSTAMP(5)
  const int K = (m < neff) ? m : neff;
#ifdef YS_DIAG_STAMPS
  if (tid == 0 && b < 32) {
    g_nms_stamps[b * 24 + 11] = (unsigned)n;
    g_nms_stamps[b * 24 + 12] = (unsigned)m;
    g_nms_stamps[b * 24 + 13] = (unsigned)K;
    g_nms_stamps[b * 24 + 14] = T;
  }
#endif
  // prefix boxes with the class offset (ops.py:289,295), areas, ids
  const float4* bx = g.boxes + (long)b * A;
  float4* sb = g.sbox + (long)b * KCAP;
  float* sa = g.sarea + (long)b * KCAP;
  unsigned* sp = g.spos + (long)b * KCAP;
  for (int i = tid; i < K; i += NMS_T) {
    const unsigned pos = ps[i];
    const unsigned a = pos / nc, j = pos % nc;
    const float4 bb = bx[a];
    const float off = g.agnostic ? 0.0f : (float)j * g.max_wh;
    const float4 o = make_float4(bb.x + off, bb.y + off, bb.z + off, bb.w + off);
    sb[i] = o;
    sa[i] = (o.z - o.x) * (o.w - o.y);
    sp[i] = pos;
  }
  if (tid == 0) {
    int* mt = g.meta + 4 * b;
    mt[0] = n;
    mt[1] = neff;
    mt[2] = K;
    mt[3] = (int)T;
  }
  YS_NSTAMP(6)
}

// -------------------------------------------------------------------------------------------------
// nms_mask: bit q of mask[b][i][cb] set iff j = cb*64+q > i, j < K and IoU(i, j) > thr. grid = (KW, B).
// -------------------------------------------------------------------------------------------------
// One wave per (row block rb, column block cb >= rb) pair: task t of image b enumerates the pairs column-major
// (t = cb (cb + 1) / 2 + rb), so the pairs of the image's nblk blocks are tasks [0, nblk (nblk + 1) / 2) and later
// tasks exit at once. Every wave has the same work (the per-row-block workgroups of round 5 gave the rb = 0 workgroup
// 32 column blocks and the rb = 31 one a single one); the waves share no data, so there is no workgroup barrier.
// grid = (KW (KW + 1) / 8, B).
__global__ __launch_bounds__(256) void nms_mask_kernel(NmsArgs g) {
  const int b = blockIdx.y;
  const int K = __builtin_amdgcn_readfirstlane(g.meta[4 * b + 2]);
  const int nblk = (K + 63) / 64;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int t = (int)blockIdx.x * 4 + wv;
  if (t >= nblk * (nblk + 1) / 2) return;  // whole wave
  int cb = (int)((sqrtf(8.0f * (float)t + 1.0f) - 1.0f) * 0.5f);
  if (cb * (cb + 1) / 2 > t) --cb;  // float rounding guards (t < 528)
  if ((cb + 1) * (cb + 2) / 2 <= t) ++cb;
  const int rb = t - cb * (cb + 1) / 2;
  __shared__ float4 cbx[4][64];
  __shared__ float car[4][64];
  const float4* sb = g.sbox + (long)b * KCAP;
  const float* sa = g.sarea + (long)b * KCAP;
  const int i = rb * 64 + lane;
  const int j = cb * 64 + lane;
  const float4 bi = (i < K) ? sb[i] : make_float4(0, 0, 0, 0);
  const float ai = (i < K) ? sa[i] : 0.f;
  // the wave's own LDS slice: written and read back by the same wave (in-order LDS), no barrier
  cbx[wv][lane] = (j < K) ? sb[j] : make_float4(0, 0, 0, 0);
  car[wv][lane] = (j < K) ? sa[j] : 0.f;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const float thr_f = g.iou_f;
  const bool all_pairs = !(g.iou >= 0.0);
  // every lane walks the same columns (uniform LDS addresses: broadcast reads, 8 in flight); the diagonal block
  // keeps only columns q > lane
  const int qhi = (K - cb * 64 < 64) ? K - cb * 64 : 64;
  const float4* cx = cbx[wv];
  const float* ca = car[wv];
  unsigned long long bits = 0ull;
  for (int q0 = 0; q0 < qhi; q0 += 8) {
    float4 bj[8];
    float aj[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      bj[u] = cx[q0 + u];
      aj[u] = ca[q0 + u];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (iou_gt_sparse(bi, ai, bj[u], aj[u], thr_f, all_pairs)) bits |= 1ull << (q0 + u);
  }
  if (qhi < 64) bits &= (1ull << qhi) - 1ull;  // columns past K
  if (cb == rb) bits &= (lane == 63) ? 0ull : (~0ull << (lane + 1));
  if (i < K) g.mask[((long)b * KCAP + i) * KW + cb] = bits;
}

// -------------------------------------------------------------------------------------------------
// nms_resolve: greedy over the prefix bitmask, then (rarely) the chunked fallback over the remainder
// -------------------------------------------------------------------------------------------------
// BIG: max_det > NMS_MAXDET (the reference has no cap, ops.py:297): the kept lists live in the workspace instead
// of LDS (same algorithm; only a caller asking for more than 1024 detections per image pays for global accesses)
template <bool BIG>
__global__ __launch_bounds__(NMS_T) void nms_resolve_kernel(NmsArgs g) {
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: the wave-0 branch below stays scalar
  __shared__ unsigned long long mrows[2][64][KW];
  __shared__ int kept_t_lds[BIG ? 1 : NMS_MAXDET];
  // kept entries: < KCAP -> prefix index, else KCAP + remainder index
  int* kept_t = BIG ? g.kept_t + (long)b * g.max_det : kept_t_lds;
  __shared__ int nkept_sh, done_sh;
  const int* mt = g.meta + 4 * b;
  // wave-uniform by construction; readfirstlane tells the compiler so (the greedy below must stay a scalar loop)
  const int n = __builtin_amdgcn_readfirstlane(mt[0]), neff = __builtin_amdgcn_readfirstlane(mt[1]);
  const int K = __builtin_amdgcn_readfirstlane(mt[2]);
  const unsigned T = (unsigned)__builtin_amdgcn_readfirstlane(mt[3]);
  const long A = g.A;
  const int nc = g.nc;
  const float* pb = g.pred + (long)b * (4 + nc) * A;
  const float4* bx = g.boxes + (long)b * A;
  const unsigned* sp = g.spos + (long)b * KCAP;
  float* ob = g.out + (long)b * g.max_det * 6;
  int* oi = g.out_index + (long)b * g.max_det;

  YS_NSTAMP(8)
  if (tid == 0) {
    nkept_sh = 0;
    done_sh = 0;
  }
  __syncthreads();
  // (1) greedy over the prefix, 64 rows (one block) at a time. Per block: wave 0 runs the greedy over the block's
  // diagonal word (a scalar loop, readlane), while waves 1..7 store the next block's mask rows into the other LDS
  // buffer and issue the loads of the block after it (in flight across the barriers: one block of prefetch in
  // registers, one in LDS); then all 8 waves OR the kept rows into the removed words of the later blocks.
  {
    const int nblk = (K + 63) / 64;
    __shared__ unsigned long long rem_w[KW];  // removed bits of each 64-column word
    __shared__ unsigned long long keptm_sh;
    constexpr int SPT = (64 * KW + (NMS_T - 64) - 1) / (NMS_T - 64);  // mask words per helper thread and block
    const int ht = tid - 64;                                           // helper thread index (waves 1..7)
    unsigned long long v[SPT];
    auto load_block = [&](int rb) {
      const unsigned long long* src = g.mask + ((long)b * KCAP + rb * 64) * KW;
#pragma unroll
      for (int u = 0; u < SPT; ++u) {
        const int e = ht + u * (NMS_T - 64), r = e / KW, w = e % KW;
        v[u] = (e < 64 * KW && rb * 64 + r < K && w >= rb && w < nblk) ? src[(long)r * KW + w] : 0ull;
      }
    };
    auto store_block = [&](int buf) {
#pragma unroll
      for (int u = 0; u < SPT; ++u) {
        const int e = ht + u * (NMS_T - 64);
        if (e < 64 * KW) mrows[buf][e / KW][e % KW] = v[u];
      }
    };
    if (tid < KW) rem_w[tid] = 0ull;
    if (wv != 0 && nblk > 0) {
      load_block(0);
      store_block(0);
      if (nblk > 1) load_block(1);
    }
    __syncthreads();
    int nkk = 0;
    for (int rb = 0; rb < nblk; ++rb) {
      const int buf = rb & 1;
      if (wv != 0) {
        if (rb + 1 < nblk) store_block(buf ^ 1);
        if (rb + 2 < nblk) load_block(rb + 2);
      } else {
        // lane q holds row q's bits inside this block (the diagonal word). The block's greedy is the fixed point of
        // kept = cand & ~OR_{j in kept} diag[j]: diag[j] only has bits above j, so the rows whose suppression
        // chain is at most t long are settled after t rounds, and the fixed point is unique (= the sequential
        // greedy). Each round is one wave-wide 64-bit OR; a few rounds replace a scalar loop of ~190 cycles per
        // kept row (one wave issuing alone, readlane -> SALU dependencies). cand / kept / rem stay wave-uniform
        // (readfirstlane), so the loop is scalar control flow.
        const unsigned long long diag = mrows[buf][lane][rb];
        const int rows_here = (K - rb * 64 < 64) ? K - rb * 64 : 64;
        const unsigned long long remv = rem_w[rb];
        const unsigned long long rem =
            ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(remv >> 32)) << 32) |
            (unsigned)__builtin_amdgcn_readfirstlane((unsigned)remv);
        const unsigned long long cand = (rows_here == 64 ? ~0ull : ((1ull << rows_here) - 1ull)) & ~rem;
        unsigned long long keptm = cand;
        for (int it = 0; it < 64; ++it) {
          unsigned lo = ((keptm >> lane) & 1ull) ? (unsigned)diag : 0u;
          unsigned hi = ((keptm >> lane) & 1ull) ? (unsigned)(diag >> 32) : 0u;
#pragma unroll
          for (int o = 1; o < 64; o <<= 1) {
            lo |= (unsigned)__shfl_xor((int)lo, o, 64);
            hi |= (unsigned)__shfl_xor((int)hi, o, 64);
          }
          const unsigned long long sup = ((unsigned long long)__builtin_amdgcn_readfirstlane(hi) << 32) |
                                         (unsigned)__builtin_amdgcn_readfirstlane(lo);
          const unsigned long long nk = cand & ~sup;
          if (nk == keptm) break;
          keptm = nk;
        }
        const int nk0 = nkk;
        bool done = false;
        if (nkk + __popcll(keptm) >= g.max_det) {  // max_det reached inside this block: its first rows only
          while (nkk + __popcll(keptm) > g.max_det) keptm &= ~(1ull << (63 - __builtin_clzll(keptm)));
          done = true;
        }
        nkk += __popcll(keptm);
        // the block's kept rows, in order, written by their own lanes
        if ((keptm >> lane) & 1ull) kept_t[nk0 + __popcll(keptm & lanemask_lt())] = rb * 64 + lane;
        if (lane == 0) {
          keptm_sh = keptm;
          nkept_sh = nkk;
          done_sh = done ? 1 : 0;
        }
      }
      __syncthreads();
      if (done_sh) break;
      // kept rows of this block into the later words: thread (word w, group gq) ORs the kept rows among rows gq,
      // gq + 16, gq + 32, gq + 48 (four bit tests; walking every kept row of the block and taking every 16th cost up
      // to 64 iterations per thread and block)
      {
        const int w = tid & 31, gq = tid >> 5;
        if (w > rb && w < nblk) {
          const unsigned long long km = keptm_sh;
          unsigned long long acc = 0ull;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int q = gq + 16 * r;
            if ((km >> q) & 1ull) acc |= mrows[buf][q][w];
          }
          if (acc) atomicOr(&rem_w[w], acc);
        }
      }
      __syncthreads();
    }
  }
  const int nk_prefix = nkept_sh;
  YS_NSTAMP(9)
  for (int k = tid; k < nk_prefix; k += NMS_T) {
    const unsigned p = sp[kept_t[k]];
    const unsigned a = p / nc, j = p % nc;
    const float4 bb = bx[a];
    float* o = ob + (long)k * 6;
    o[0] = bb.x; o[1] = bb.y; o[2] = bb.z; o[3] = bb.w;
    o[4] = pb[(long)(4 + j) * A + a];
    o[5] = (float)j;
    oi[k] = (int)a;
  }

  // (2) fallback: prefix exhausted, fewer than max_det kept, more candidates (keys >= T) within max_nms
  if (!done_sh && K < neff) {
    __shared__ SortShared sh;
    __shared__ float4 kept_box_lds[BIG ? 1 : NMS_MAXDET];
    __shared__ float kept_area_lds[BIG ? 1 : NMS_MAXDET];
    float4* kept_box = BIG ? g.kbox + (long)b * g.max_det : kept_box_lds;
    float* kept_area = BIG ? g.karea + (long)b * g.max_det : kept_area_lds;
    __shared__ float4 cb[NMS_T];
    __shared__ float ca[NMS_T];
    __shared__ int alive[NMS_T];
    __shared__ unsigned long long alive_w[NMS_W];
    __shared__ unsigned long long rows[NMS_T][NMS_T / 64];
    const float4* sb = g.sbox + (long)b * KCAP;
    const float* sa = g.sarea + (long)b * KCAP;
    for (int k = tid; k < nk_prefix; k += NMS_T) {
      kept_box[k] = sb[kept_t[k]];
      kept_area[k] = sa[kept_t[k]];
    }
    unsigned* kA = g.keyA + (long)b * g.cap;
    unsigned* pA = g.posA + (long)b * g.cap;
    unsigned* kB = g.keyB + (long)b * g.cap;
    unsigned* pB = g.posB + (long)b * g.cap;
    const int m = compact_by_key(kA, pA, n, T, false, kB, pB, sh);
    __syncthreads();
    const int cap_total = (m < neff - K) ? m : neff - K;  // max_nms
#ifdef YS_DIAG_STAMPS
    unsigned long long f_t0 = __builtin_amdgcn_s_memtime(), f_t1, f_keep = 0, f_mask = 0, f_greedy = 0, f_out = 0;
    int f_chunks = 0;
    if (threadIdx.x == 0 && blockIdx.x < 32) g_nms_stamps[blockIdx.x * 24 + 19] = (unsigned long long)cap_total;
#define YS_FACC(acc) f_t1 = __builtin_amdgcn_s_memtime(); acc += f_t1 - f_t0; f_t0 = f_t1;
#else
#define YS_FACC(acc)
#endif
#ifdef YS_DIAG_STAMPS
    YS_FACC(f_out)
    f_out = 0;
#endif
    // the remainder's candidates [0, cnt) in score order (positions ps_r): chunks of 512 against the kept list, then
    // their own IoU bits and greedy; stops at max_det
    auto run_chunks = [&](const unsigned* ps_r, int cnt) __attribute__((always_inline)) {
      for (int c0 = 0; c0 < cnt; c0 += NMS_T) {
        const int i = c0 + tid;
        const bool valid = i < cnt;
        float4 obox = make_float4(0, 0, 0, 0);
        float area = 0.f;
        if (valid) {
          const unsigned pos = ps_r[i];
          const unsigned a = pos / nc, j = pos % nc;
          const float4 bb = bx[a];
          const float off = g.agnostic ? 0.0f : (float)j * g.max_wh;
          obox = make_float4(bb.x + off, bb.y + off, bb.z + off, bb.w + off);
          area = (obox.z - obox.x) * (obox.w - obox.y);
        }
        cb[tid] = obox;
        ca[tid] = area;
        const int nk = nkept_sh;
        const bool all_pairs = !(g.iou >= 0.0);
        // against the kept list: 8 kept boxes read per step (uniform LDS addresses, all in flight), the wave leaves
        // the loop once none of its candidates is alive (a per-lane exit made every LDS read wait on its own)
        bool al = valid;
        for (int k0 = 0; k0 < nk; k0 += 8) {
          if (__ballot(al) == 0ull) break;
          float4 kb[8];
          float ka[8];
  #pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int k = (k0 + u < nk) ? k0 + u : nk - 1;
            kb[u] = kept_box[k];
            ka[u] = kept_area[k];
          }
  #pragma unroll
          for (int u = 0; u < 8; ++u)
            if (k0 + u < nk && iou_gt_sparse(kb[u], ka[u], obox, area, g.iou_f, all_pairs)) al = false;
        }
        alive[tid] = al ? 1 : 0;
        const unsigned long long aw = __ballot(al);
        if (lane == 0) alive_w[wv] = aw;
        __syncthreads();
        YS_FACC(f_keep)
        // the chunk's own IoU bits: only words at or after the wave's own (later candidates) and only words with an
        // alive candidate (the others stay 0: the greedy reads bits of alive candidates only)
  #pragma unroll
        for (int wd = 0; wd < NMS_T / 64; ++wd) {
          unsigned long long bits = 0ull;
          const unsigned long long awd = alive_w[wd];
          if (wd >= wv && awd != 0ull && __ballot(al) != 0ull) {
            for (int q0 = 0; q0 < 64; q0 += 8) {  // 8 candidates' reads in flight (uniform addresses)
              float4 jb[8];
              float ja[8];
  #pragma unroll
              for (int u = 0; u < 8; ++u) {
                jb[u] = cb[wd * 64 + q0 + u];
                ja[u] = ca[wd * 64 + q0 + u];
              }
  #pragma unroll
              for (int u = 0; u < 8; ++u) {
                const int q = q0 + u, jj = wd * 64 + q;
                if (al && jj > tid && ((awd >> q) & 1ull) &&
                    iou_gt_sparse(obox, area, jb[u], ja[u], g.iou_f, all_pairs))
                  bits |= 1ull << q;
              }
            }
          }
          rows[tid][wd] = bits;
        }
        __syncthreads();
        YS_FACC(f_mask)
        if (wv == 0) {
          unsigned long long removed = 0ull;
          int nkk = nk;
          bool done = false;
          for (int w = 0; w < NMS_T / 64 && !done; ++w) {
            unsigned long long cand = alive_w[w] & ~__shfl(removed, w, 64);
            while (cand) {
              const int q = __ffsll((long long)cand) - 1;
              const int t = w * 64 + q;
              if (lane == 0) {
                kept_box[nkk] = cb[t];
                kept_area[nkk] = ca[t];
                kept_t[nkk] = c0 + t;  // remainder index
              }
              ++nkk;
              if (nkk >= g.max_det) {
                done = true;
                break;
              }
              if (lane < NMS_T / 64) removed |= rows[t][lane];
              const unsigned long long upto = (q == 63) ? ~0ull : ((2ull << q) - 1ull);
              cand &= ~upto & ~__shfl(removed, w, 64);
            }
          }
          if (lane == 0) {
            nkept_sh = nkk;
            done_sh = done ? 1 : 0;
          }
        }
        __syncthreads();
        YS_FACC(f_greedy)
        const int nk_new = nkept_sh;
        for (int k = nk + tid; k < nk_new; k += NMS_T) {
          const unsigned p = ps_r[kept_t[k]];
          const unsigned a = p / nc, j = p % nc;
          const float4 bb = bx[a];
          float* o = ob + (long)k * 6;
          o[0] = bb.x; o[1] = bb.y; o[2] = bb.z; o[3] = bb.w;
          o[4] = pb[(long)(4 + j) * A + a];
          o[5] = (float)j;
          oi[k] = (int)a;
        }
        YS_FACC(f_out)
  #ifdef YS_DIAG_STAMPS
        ++f_chunks;
  #endif
        if (done_sh) break;
      }
    };
    // The remainder is consumed in rounds of at most KCAP candidates (a greedy that reaches max_det early reads
    // only the first rounds; sorting the whole remainder in global memory cost ~0.34 ms at 28k keys): buckets of the
    // 8 key bits from the highest one in which the remainder keys differ (one stable scatter pass puts them in bucket order), as many
    // whole buckets per round as fit, each round copied into LDS and sorted there. A single bucket above KCAP (e.g.
    // equal scores) sorts everything from that bucket on in global memory.
    __shared__ unsigned rk[2][KCAP], rp[2][KCAP];
    __shared__ unsigned rmin, rmax;
    __shared__ unsigned rbase[256];
    __shared__ int rnd_d2;
    if (m <= KCAP) {
      for (int i = tid; i < m; i += NMS_T) {
        rk[0][i] = kB[i];
        rp[0][i] = pB[i];
      }
      __syncthreads();
      unsigned *ks = rk[0], *ps = rp[0], *kd = rk[1], *pd = rp[1];
      radix_sort_lds(ks, ps, kd, pd, m, sh);
      run_chunks(ps, cap_total);
    } else {
      if (tid == 0) {
        rmin = 0xFFFFFFFFu;
        rmax = 0u;
      }
      __syncthreads();
      unsigned kmn = 0xFFFFFFFFu, kmx = 0u;
      for (int i = tid; i < m; i += NMS_T) {
        const unsigned k = kB[i];
        kmn = min(kmn, k);
        kmx = max(kmx, k);
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        kmn = min(kmn, (unsigned)__shfl_xor((int)kmn, o, 64));
        kmx = max(kmx, (unsigned)__shfl_xor((int)kmx, o, 64));
      }
      if (lane == 0) {
        atomicMin(&rmin, kmn);
        atomicMax(&rmax, kmx);
      }
      if (tid < 256) sh.hist[tid] = 0;
      __syncthreads();
      const unsigned diffk = rmin ^ rmax;
      const int shiftB = diffk ? max(31 - __clz(diffk) - 7, 0) : 0;  // the 8 bits from the highest differing one
      for (int i0 = 0; i0 < m; i0 += NMS_T) {
        const int i = i0 + tid;
        hist_add_digit(sh.hist, (i < m) ? (kB[i] >> shiftB) & 255u : 0u, i < m);
      }
      __syncthreads();
      scan256_exclusive(sh.hist, sh.tmp4);
      if (tid < 256) rbase[tid] = sh.hist[tid];  // keys in buckets < d (the sorts below reuse sh.hist)
      radix_scatter(kB, pB, kA, pA, m, shiftB, sh);  // bucket d = [rbase[d], rbase[d + 1]) of (kA, pA)
      __syncthreads();
      int d = 0, processed = 0;
      bool full = false;
      while (processed < cap_total && !done_sh) {
        if (tid == 0) rnd_d2 = d;
        __syncthreads();
        if (tid < 256 && tid + 1 > d) {  // candidate end t = tid + 1 in (d, 256]
          const int t = tid + 1;
          const unsigned et = (t < 256) ? rbase[t] : (unsigned)m;
          if (et - rbase[d] <= (unsigned)KCAP) atomicMax(&rnd_d2, t);
        }
        __syncthreads();
        const int d2 = rnd_d2;
        if (d2 == d) {
          full = true;
          break;
        }
        const int s0 = (int)rbase[d];
        const int cnt = ((d2 < 256) ? (int)rbase[d2] : m) - s0;
        for (int i = tid; i < cnt; i += NMS_T) {
          rk[0][i] = kA[s0 + i];
          rp[0][i] = pA[s0 + i];
        }
        __syncthreads();
        unsigned *ks = rk[0], *ps = rp[0], *kd = rk[1], *pd = rp[1];
        radix_sort_lds(ks, ps, kd, pd, cnt, sh);
        run_chunks(ps, min(cnt, cap_total - processed));
        __syncthreads();
        processed += cnt;
        d = d2;
      }
      if (full && processed < cap_total && !done_sh) {
        const int s0 = (int)rbase[d];
        const int cnt = m - s0;
        unsigned *ks = kA + s0, *ps = pA + s0, *kd = kB + s0, *pd = pB + s0;
        radix_sort_pairs(ks, ps, kd, pd, cnt, sh);
        run_chunks(ps, min(cnt, cap_total - processed));
      }
    }
#ifdef YS_DIAG_STAMPS
    if (threadIdx.x == 0 && blockIdx.x < 32) {
      g_nms_stamps[blockIdx.x * 24 + 20] = f_keep;
      g_nms_stamps[blockIdx.x * 24 + 21] = f_mask;
      g_nms_stamps[blockIdx.x * 24 + 22] = f_greedy;
      g_nms_stamps[blockIdx.x * 24 + 23] = f_chunks;
    }
#endif
#undef YS_FACC
  }
  __syncthreads();
  const int nk = nkept_sh;
  for (int e = nk * 6 + tid; e < g.max_det * 6; e += NMS_T) ob[e] = 0.f;
  for (int e = nk + tid; e < g.max_det; e += NMS_T) oi[e] = -1;
  if (tid == 0) {
    g.counts[b] = nk;
  }
  YS_NSTAMP(10)
}


}  // namespace ys

using namespace ys;

#ifdef YS_DIAG_STAMPS
YS_EXPORT int yolosod_diag_nms_stamps(unsigned long long* host) {  // [32][24] of the last call
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_nms_stamps), sizeof(g_nms_stamps)) == hipSuccess ? 0 : -1;
}
#endif


static long nms_cap(int nc, int A, int multi_label) { return (long)A * (multi_label ? nc : 1); }

YS_EXPORT size_t yolosod_nms_workspace_v2(int B, int nc, int A, int multi_label, int max_det) {
  const long cap = nms_cap(nc, A, multi_label);
  Sizer s;
  s.take<float4>((size_t)B * A);
  s.take<unsigned long long>((size_t)B * A);
  for (int i = 0; i < 4; ++i) s.take<unsigned>((size_t)B * cap);
  s.take<float4>((size_t)B * KCAP);
  s.take<float>((size_t)B * KCAP);
  s.take<unsigned>((size_t)B * KCAP);
  s.take<unsigned long long>((size_t)B * KCAP * KW);
  s.take<int>((size_t)B * 4);
  s.take<int>((size_t)B * ((A + 255) / 256));
  if (max_det > NMS_MAXDET) {
    s.take<int>((size_t)B * max_det);
    s.take<float4>((size_t)B * max_det);
    s.take<float>((size_t)B * max_det);
  }
  return s.off;
}

YS_EXPORT size_t yolosod_nms_workspace(int B, int nc, int A, int multi_label) {
  return yolosod_nms_workspace_v2(B, nc, A, multi_label, NMS_MAXDET);
}

YS_EXPORT int yolosod_nms(float* pred, int B, int nc, int A, float conf_thres, double iou_thres, const int* classes,
                          int n_classes, int agnostic, int multi_label, int max_det, int max_nms, float max_wh,
                          int in_place, float* out, int* counts, int* out_index, void* workspace,
                          size_t workspace_bytes, void* stream) {
  YS_CHECK_ARG(pred && out && counts && out_index, "nms: null pointer");
  YS_CHECK_ARG(nc >= 1 && nc <= 64, "nms: nc=%d unsupported (1..64)", nc);
  YS_CHECK_ARG(max_det >= 1 && max_det <= NMS_MAXDET_BIG, "nms: max_det=%d unsupported (1..%d)", max_det,
               NMS_MAXDET_BIG);
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
  {  // round toward -inf: the largest float <= iou_thres (NaN stays NaN: every comparison false, as in double)
    float t = (float)iou_thres;
    if ((double)t > iou_thres) t = nextafterf(t, -INFINITY);
    g.iou_f = t;
  }
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
  g.sbox = cv.take<float4>((size_t)B * KCAP);
  g.sarea = cv.take<float>((size_t)B * KCAP);
  g.spos = cv.take<unsigned>((size_t)B * KCAP);
  g.mask = cv.take<unsigned long long>((size_t)B * KCAP * KW);
  g.meta = cv.take<int>((size_t)B * 4);
  const int nblk_a = (A + 255) / 256;
  g.blkcnt = cv.take<int>((size_t)B * nblk_a);
  const bool big = max_det > NMS_MAXDET;
  if (big) {
    g.kept_t = cv.take<int>((size_t)B * max_det);
    g.kbox = cv.take<float4>((size_t)B * max_det);
    g.karea = cv.take<float>((size_t)B * max_det);
  }
  YS_CHECK_ARG(g.blkcnt && (!big || g.karea), "nms: workspace too small (%zu)", workspace_bytes);
  g.cap = cap;
  g.out = out;
  g.counts = counts;
  g.out_index = out_index;
  if (A > 0) {
    hipLaunchKernelGGL(nms_prep_kernel, dim3(nblk_a, B), dim3(256), 0, st, g);
    hipLaunchKernelGGL(nms_scatter_kernel, dim3(nblk_a, B), dim3(256), 0, st, g);
  }
  hipLaunchKernelGGL(nms_select_kernel, dim3(B), dim3(NMS_T), 0, st, g);
  hipLaunchKernelGGL(nms_mask_kernel, dim3(KW * (KW + 1) / 8, B), dim3(256), 0, st, g);
  if (big)
    hipLaunchKernelGGL(nms_resolve_kernel<true>, dim3(B), dim3(NMS_T), 0, st, g);
  else
    hipLaunchKernelGGL(nms_resolve_kernel<false>, dim3(B), dim3(NMS_T), 0, st, g);
  YS_CHECK_LAUNCH("nms");
  return 0;
}
