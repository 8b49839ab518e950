// Fused SwinBlock for C = 64 (the P2 instance L28 of the paper model) with every matrix product - projections,
// MLP, pw conv and the attention - on the fp16 matrix cores at fp32 accuracy.
//
// Why: on gfx950 the fp32 MFMA (v_mfma_f32_16x16x4_f32, 157 TF/s) shares the SIMD with the VALU - they never
// co-execute - and the fused fp32 kernel (swin_fused.hip) spends ~58 % of its cycles in it. The fp16 MFMA runs 16x
// faster per instruction-cycle and beside other waves' VALU. An fp32 operand splits into two fp16 terms, v = h + l
// (h = fp16(v), l = fp16(v - h), round to nearest even; v - h is exact in fp32), with |v - h - l| <= 2^-22 |v| while
// l stays a normal fp16 number, and a product into the three terms of order >= 2^-11,
//   a.b ~ ah.bh + ah.bl + al.bh     (dropped: al.bl <= 2^-22 |a.b|),
// each an exact fp16 x fp16 product accumulated in fp32 by the MFMA - the same accumulation as the fp32 MFMA, with a
// representation error of a few fp32 ulps. Three v_mfma_f32_16x16x32_f16 (16 cycles each) replace eight
// v_mfma_f32_16x16x4_f32 (32 cycles each) per 16x16x32 block: 5.3x fewer matrix cycles. Weights are split once per
// call by a prep kernel (with the LayerNorm affine terms folded in: W' = W diag(gamma), b' = b + W beta, so the
// kernel's LayerNorms only normalise), scaled by 64 (exact) so that the low terms of small weights stay out of
// fp16's subnormal range; the accumulators start from 64 b and are scaled back by 1/64 (exact) in each epilogue
// (Q, K and V keep the factor: it folds into the softmax's exp2 scale and the 1/sum applied to O).
// Activations are split by their producer (LayerNorm, the QKV epilogue, attention, GELU, the last residual add) when
// they are written to LDS, two fp16 planes per operand. fp16's range (65504) bounds the activations and 64 W.
//
// One 256-thread workgroup per 7x7 window, three per CU (LDS 48 KB): T (fp32 residual stream [49][68]) | X (halo
// patch -> two fp16 planes [64][72] of U1 -> K planes [49][72] + V^T planes [64][72] -> O planes -> U2 planes -> MLP
// hidden half planes -> final T planes for the pw GEMM) | parameters. Each producer keeps its result in registers
// until every wave has read X's previous content. GEMM tiles cover token rows 0..63 (four 16-row blocks; rows 49..63
// are finite padding whose outputs are dropped) and are transposed (the weight planes are the MFMA A operand): lane
// (g, l15) holds out[token rb*16 + l15][n = cb*16 + 4g .. +3]. Wave w computes the Q of its own 16 queries, which
// stay in registers as the B operand of S^T = K Q^T; the S^T accumulators are split in registers into the P^T
// operand of O^T = V^T P^T (keys 49..63 masked to P = 0).
//
// Reference semantics as swin_fused.hip (ultralytics/nn/modules/blocks_transformer.py:8-171).
#include "common.h"
#include <math.h>
#include <stdlib.h>

namespace ys {
namespace x3 {

constexpr float WSC = 64.0f;  // weight planes hold 64 W (exact): keeps their low terms out of fp16's subnormal range

#ifdef YS_DIAG_STAMPS  // diagnostic builds only (scripts/diag_x3.sh): per-stage s_memtime of wave 0, first 256 windows
__device__ unsigned long long ys_x3_stamps[256 * 32];
#define X3_STAMP(k)                                                                                                  \
  do {                                                                                                               \
    if (threadIdx.x == 0 && blockIdx.x < 256) ys_x3_stamps[blockIdx.x * 32 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define X3_STAMP(k) \
  do {              \
  } while (0)
#endif


constexpr int NR = 49;   // tokens per 7x7 window
constexpr int HPW = 12;  // halo patch row stride (9 used)

struct Args {
  const float* x;
  float* y;
  int B, H, W, nWx, nWin;
  const float* dw;     // [C][9]
  float ln1_eps, ln2_eps;
  const h16_t* win;    // planes [2][3C][C] of 64 W, LN1 affine folded
  const float* bin;    // [3C] folded
  const h16_t* wo;     // [2][C][C]
  const float* bo;
  const h16_t* w1;     // [2][HID][C], LN2 affine folded
  const float* b1;     // [HID] folded
  const h16_t* w2;     // [2][C][HID]
  const float* b2;
  const h16_t* wpw;    // [2][C][C]
  const float* bn_scale;
  const float* bn_shift;
  float scale;
  unsigned* range_flag;  // split-range guard (common.h range_report), may be null
  const unsigned* prep_flag;  // the prepared block's own range word (swin_x3_prep_kernel), reported on every launch
};

// The weight preparation's range result is kept in the prepared block and re-reported by every launch that uses the
// block (the block is cached across calls, so the prep kernel's own report fires only once per parameter version)
__device__ __forceinline__ void prep_report(const unsigned* prep_flag, unsigned* flag) {
  if (prep_flag && flag && blockIdx.x == 0 && threadIdx.x == 0 && *prep_flag) *flag = 1u;
}

__device__ __forceinline__ f32x4 mfma16(f16x8_t a, f16x8_t b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float dot4_acc(float4 a, float4 b, float acc) {
  acc = fmaf(a.x, b.x, acc);
  acc = fmaf(a.y, b.y, acc);
  acc = fmaf(a.z, b.z, acc);
  return fmaf(a.w, b.w, acc);
}
__device__ __forceinline__ float group4_sum(float v) { return xor32_sum(xor16_sum(v)); }

// Element (row, col) of a [rows][PS] fp16 plane. SWZ: the 16-byte chunks of a row are XOR-swizzled by the row's low
// three bits (chunk c -> c ^ (row & 7)) in an unpadded row (PS = 64): the GEMM operand reads (ds_read_b128, lane =
// (row l15, chunk g)), the LN plane stores (ds_write_b128, 4 lanes per row) and the accumulator stores
// (ds_write_b64, 16 rows x one column group) are then conflict-free / 2-way instead of 0 / 2-way / 4-way at PS = 80.
template <int PS, bool SWZ>
__device__ __forceinline__ int plane_off(int row, int col) {
  if constexpr (SWZ) return row * PS + ((((col >> 3) ^ (row & 7))) << 3) + (col & 7);
  else return row * PS + col;
}
// The same for planes that are only read 8 bytes at a time (the attention's K and V^T planes: ds_read_b64 and
// ds_write_b64 of 4 elements, lane = (row l15, column group g)): 8-byte chunks swizzled by the row's low four bits,
// which makes both the reads and the 16-row column stores conflict-free (at the padded stride 72 the stores were
// 2-way)
template <int PS, bool SWZ>
__device__ __forceinline__ int plane_off8(int row, int col) {
  if constexpr (SWZ) return row * PS + ((((col >> 2) ^ (row & 15))) << 2) + (col & 3);
  else return row * PS + col;
}

// the two planes of 4 consecutive elements of row `row`, column `col` (a multiple of 4)
template <int PS, int PL, bool SWZ = false, bool SWZ8 = false>
__device__ __forceinline__ void store_planes4(h16_t* P, int row, int col, f32x4 v) {
  uint2 h, l;
  split4(v, h, l);
  h16_t* d = P + (SWZ8 ? plane_off8<PS, true>(row, col) : plane_off<PS, SWZ>(row, col));
  *reinterpret_cast<uint2*>(d) = h;
  *reinterpret_cast<uint2*>(d + PL) = l;
}

// Weight-plane fragments of one GEMM for this wave's column blocks cb = cb0 + 4j: lane (g, l15) holds
// W_p[cb*16 + l15][koff + 32s + 8g .. +7] (16-byte global loads, L2-resident).
template <int K, int NJ>
struct WP {
  f16x8_t v[NJ][K / 32][2];
};
template <int K, int NJ>
__device__ __forceinline__ void load_wp(const h16_t* __restrict__ Wp, int N, int KT, int koff, int cb0, WP<K, NJ>& f,
                                        int lane) {
  // fragment-major planes (swin_x3_prep_kernel): the 64 lanes' fragments of one (column block, 32-k step) are 1 KB
  // contiguous, so a wave-instruction reads 8 whole cache lines (16 half lines row-major)
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int s = 0; s < K / 32; ++s)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        f.v[j][s][p] = *reinterpret_cast<const f16x8_t*>(
            Wp + (long)p * N * KT + ((long)((cb0 + 4 * j) * (KT / 32) + koff / 32 + s) * 64 + lane) * 8);
}

// acc[rb][j] += (A[rows rb*16 .. +15][0, K) . W^T)^T: A = three LDS planes (row stride PS, plane stride PL), the
// weight planes as the MFMA A operand, so the lane holds out[token rb*16 + l15][n = cb*16 + 4g .. +3]. Six products
// per (k-step, row block, column block), smallest terms first. The LDS operand reads run two (k-step, row block)
// steps ahead of the MFMAs (at two waves per SIMD a read waited for right before its MFMAs exposes its latency).
// SWAP: the token rows are the MFMA's A operand and the weight planes its B operand (the same fragments), so the
// lane holds out[token rb*16 + 4g .. +3][n = cb*16 + l15] instead (4 consecutive tokens of one output column).
template <int K, int NJ, int PS, int PL, bool SWAP = false, bool SWZ = false>
__device__ __forceinline__ void gemm_x3(const h16_t* A, const WP<K, NJ>& w, f32x4 (&acc)[4][NJ], int lane) {
  const int l15 = lane & 15, g = lane >> 4;
  constexpr int NS = (K / 32) * 4;  // steps (s, rb), rb fastest
  const h16_t* a0 = A + l15 * PS;
  int coff[K / 32];  // this lane's column offset of k step s (rows l15 + 16 rb share the low row bits)
#pragma unroll
  for (int s = 0; s < K / 32; ++s) coff[s] = plane_off<PS, SWZ>(l15, 32 * s + 8 * g) - l15 * PS;
  f16x8_t u[3][2];
  auto ld = [&](int i, f16x8_t (&v)[2]) {
    const h16_t* ar = a0 + (i & 3) * 16 * PS + coff[i >> 2];
    v[0] = *reinterpret_cast<const f16x8_t*>(ar);
    v[1] = *reinterpret_cast<const f16x8_t*>(ar + PL);
  };
  ld(0, u[0]);
  ld(1, u[1]);
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    if (i + 2 < NS) ld(i + 2, u[(i + 2) % 3]);
    const int s = i >> 2, rb = i & 3;
    const f16x8_t* v = u[i % 3];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      f32x4 c = acc[rb][j];
      if (SWAP) {
        c = mfma16(v[0], w.v[j][s][1], c);
        c = mfma16(v[1], w.v[j][s][0], c);
        acc[rb][j] = mfma16(v[0], w.v[j][s][0], c);
      } else {
        c = mfma16(w.v[j][s][1], v[0], c);
        c = mfma16(w.v[j][s][0], v[1], c);
        acc[rb][j] = mfma16(w.v[j][s][0], v[0], c);
      }
    }
  }
}

// LayerNorm statistics of token rows [0, 49) of T (fp32, stride LT) and the normalised rows (affine folded into the
// next GEMM) as two fp16 planes; rows 49..63 get zeros. 4 lanes per row (a DPP quad), C/4 values each.
template <int C, int LT, int PS, int PL, bool SWZ = false>
__device__ __forceinline__ void ln_planes(const float* T, h16_t* P, float eps, int tid) {
  constexpr int CP = C / 4;
  const int r = tid >> 2, qd = tid & 3;
  const bool valid = r < NR;
  f32x4 v[CP / 4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < CP / 4; ++i) {
    v[i] = valid ? *reinterpret_cast<const f32x4*>(T + r * LT + qd * CP + 4 * i) : f32x4{0.f, 0.f, 0.f, 0.f};
    s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  }
  const float mean = quad_sum(s) * (1.0f / (float)C);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < CP / 4; ++i) {
    v[i] -= mean;
    q += (v[i].x * v[i].x + v[i].y * v[i].y) + (v[i].z * v[i].z + v[i].w * v[i].w);
  }
  const float rs = valid ? __builtin_amdgcn_rsqf(quad_sum(q) * (1.0f / (float)C) + eps) : 0.f;
#pragma unroll
  for (int i = 0; i < CP / 4; i += 2) {
    uint2 h0, l0, h1, l1;
    split4(v[i] * rs, h0, l0);
    split4(v[i + 1] * rs, h1, l1);
    h16_t* d = P + plane_off<PS, SWZ>(r, qd * CP + 4 * i);
    *reinterpret_cast<uint4*>(d) = make_uint4(h0.x, h0.y, h1.x, h1.y);
    *reinterpret_cast<uint4*>(d + PL) = make_uint4(l0.x, l0.y, l1.x, l1.y);
  }
}

template <int C, int NH>
__global__ __launch_bounds__(256, 3) void swin_x3_kernel(Args p) {
  constexpr bool SWZ = true;  // unpadded plane rows with XOR-swizzled chunks (plane_off / plane_off8)
  constexpr int HD = C / NH;
  constexpr int HID = 2 * C;
  constexpr int LT = C + 4;      // T row stride (floats)
  constexpr int PS = C;          // plane row stride (fp16): unpadded, chunk-swizzled rows
  constexpr int PL = 64 * PS;    // plane stride
  constexpr int PSK = C;         // K plane row stride: unpadded, 8-byte chunks swizzled
  constexpr int KPL = NR * PSK;  // K plane stride
  constexpr int PSV = 64;        // V^T plane row stride (keys 0..63)
  constexpr int VPL = C * PSV;   // V^T plane stride
  constexpr int NHS = (C + 2) / 3;
  constexpr int PSH = HID + 8;  // MLP hidden plane row stride (both halves side by side, unswizzled: 272-byte rows put
                                // the 16 rows of an operand read on distinct bank quads)
  constexpr int PLH = 64 * PSH;                        // hidden plane stride
  constexpr int QW_H = 2 * (C / 16) * (C / 32) * 512;  // staged Q weight fragments: [k step][plane][column block][512]
  static_assert(C == 64 && HID / 2 == C, "the plane regions are sized for C = 64 (hidden halves of 64)");
  static_assert(HD == 32, "attention operands: two 16-column blocks per head");
  constexpr int T_B = NR * LT * 4;
  constexpr int KV_B = (2 * VPL + 2 * KPL) * 2;
  constexpr int PLN_B = 2 * PL * 2 + QW_H * 2;  // U1 planes + all Q weight fragments
  constexpr int HID_B = 2 * PLH * 2;            // both MLP hidden halves as planes
  constexpr int HALO_B = 3 * NHS * 9 * HPW * 4;
  constexpr int X_B0 = KV_B > HALO_B ? (KV_B > PLN_B ? KV_B : PLN_B) : (HALO_B > PLN_B ? HALO_B : PLN_B);
  constexpr int X_B = ((X_B0 > HID_B ? X_B0 : HID_B) + 15) / 16 * 16;
  constexpr int NPAR = 3 * C + C + HID + C + 2 * C;
  static_assert(T_B % 16 == 0 && X_B % 16 == 0, "16-byte aligned regions");
  static_assert(T_B + X_B + NPAR * 4 <= 160 * 1024 / 3, "three workgroups per CU");
  static_assert(PLN_B <= X_B && HID_B <= X_B, "staged Q weights after the U1 planes; both hidden halves");
  __shared__ __attribute__((aligned(16))) char smem[T_B + X_B + NPAR * 4];
  float* T = reinterpret_cast<float*>(smem);
  char* X = smem + T_B;
  float* Q = reinterpret_cast<float*>(X);
  h16_t* P = reinterpret_cast<h16_t*>(X);
  float* par = reinterpret_cast<float*>(smem + T_B + X_B);
  constexpr int P_BIN = 0, P_BO = 3 * C, P_B1 = 4 * C, P_B2 = 4 * C + HID, P_SC = 5 * C + HID, P_SH = 6 * C + HID;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  float rng = 0.f;  // largest magnitude this thread splits outside a LayerNorm (split-range guard)
  const int l15 = lane & 15, g = lane >> 4;
  const int H = p.H, W = p.W;
  const int HWi = H * W;  // per-image offsets are 32-bit (the launcher checks C*H*W < 2^30)

  // XCD-aware window order: workgroup i runs on XCD i % 8 and takes windows from that XCD's contiguous range, so
  // horizontally adjacent windows (whose 7-pixel rows share 128-byte lines of x and y) meet in one L2
  const long nwin_total = (long)p.B * p.nWin;
  const long per_xcd = (nwin_total + 7) >> 3;
  const long gwl = (long)(blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  if (gwl >= nwin_total || (blockIdx.x >> 3) >= per_xcd) return;
  const int gw = __builtin_amdgcn_readfirstlane((int)gwl);
  const int img = gw / p.nWin, win = gw - (gw / p.nWin) * p.nWin;
  const int wy = win / p.nWx, wx = win - (win / p.nWx) * p.nWx;
  X3_STAMP(0);
  auto rsrc_of = [&](const float* base) {
    const unsigned long long a = (unsigned long long)base;
    return __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(a >> 32)) << 32) |
                (unsigned)__builtin_amdgcn_readfirstlane((unsigned)a)),
        (short)0, __builtin_amdgcn_readfirstlane(C * HWi * 4), 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rx = rsrc_of(p.x + (long)img * C * HWi);
  constexpr unsigned OOB = 0x80000000u;

  // halo patch [C][9][9] -> registers: row slot s = 7*wid + lane/9 < 27 is (channel 3i + s/9, patch row s%9) at
  // step i, lane%9 the column; out-of-image lanes get an out-of-range voffset (the buffer load returns 0)
  const int hl_r = lane / 9, hl_px = lane - (lane / 9) * 9;
  const int hslot = 7 * wid + hl_r;
  float hv[NHS];
  {
    const int hcs = hslot / 9, hpy = hslot - (hslot / 9) * 9;
    const int hh = wy * 7 - 1 + hpy, wc = wx * 7 - 1 + hl_px;
    const bool ok = hl_r < 7 && hslot < 27 && (unsigned)hh < (unsigned)H && (unsigned)wc < (unsigned)W;
    const unsigned voff = ok ? (unsigned)((hcs * HWi + hh * W + wc) * 4) : OOB;
    const unsigned vlast = (3 * (NHS - 1) + hcs < C) ? voff : OOB;
#pragma unroll
    for (int i = 0; i < NHS; ++i)
      hv[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, i == NHS - 1 ? vlast : voff,
                                                                            i * 3 * HWi * 4, 0));
  }
  for (int e = tid; e < NPAR; e += 256) {
    float v;
    if (e < P_BO) v = p.bin[e];
    else if (e < P_B1) v = p.bo[e - P_BO];
    else if (e < P_B2) v = p.b1[e - P_B1];
    else if (e < P_SC) v = p.b2[e - P_B2];
    else if (e < P_SH) v = p.bn_scale[e - P_SC];
    else v = p.bn_shift[e - P_SH];
    par[e] = e < P_SC ? v * WSC : (e < P_SH ? v * (1.0f / WSC) : v);  // biases x64, BN scale /64 (exact)
  }
  const int dw_c = tid % C;
  float dwk[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) dwk[i] = p.dw[dw_c * 9 + i];
  // The Q weight planes (rows 0..C of in_proj) are staged once per workgroup through X, both 32-k chunks at once
  // behind the U1 planes (every wave needs all of them for its own 16 queries; streamed per wave they were 4x the Q
  // bytes from L2; staged one chunk at a time they cost two more barriers): this thread's 32 bytes of both chunks
  // are in flight during the halo store, the dw conv and LN1
  // chunk s = the fragment blocks (plane, Q column block cq) of k step s: 8 blocks of 512 halves; thread t copies
  // halves 16 (t & 31) .. +15 of block t >> 5
  const int qblk = tid >> 5, qpl = qblk >> 2, qcb = qblk & 3;
  const h16_t* qsrc = p.win + (long)qpl * 3 * C * C + (long)(qcb * (C / 32)) * 512 + 16 * (tid & 31);
  const uint4 qc0a = *reinterpret_cast<const uint4*>(qsrc), qc0b = *reinterpret_cast<const uint4*>(qsrc + 8);
  const uint4 qc1a = *reinterpret_cast<const uint4*>(qsrc + 512), qc1b = *reinterpret_cast<const uint4*>(qsrc + 520);

  // ---- halo -> X (fp32 [27i + slot][HPW]) -> dw3x3 -> T (cropped / padded tokens = 0) ----
  float* halo = Q;
  if (hl_r < 7 && hslot < 27) {
#pragma unroll
    for (int i = 0; i < NHS; ++i) halo[(27 * i + hslot) * HPW + hl_px] = hv[i];
  }
  __syncthreads();
  X3_STAMP(1);
  {
    // wave w computes output rows 2w and 2w + 1 (wave 3: row 6) of channel dw_c: the four halo rows they need are
    // read once (12 16-byte LDS reads for 14 outputs)
    const int iy0 = 2 * wid;
    const int nrow = iy0 + 1 < 7 ? 2 : 1;
    const float* hp = halo + (dw_c * 9 + iy0) * HPW;
    float r[4][12];
#pragma unroll
    for (int ky = 0; ky < 4; ++ky) {
      if (ky < nrow + 2) {
#pragma unroll
        for (int q4 = 0; q4 < 3; ++q4) {
          const float4 v = *reinterpret_cast<const float4*>(hp + ky * HPW + 4 * q4);
          r[ky][4 * q4] = v.x; r[ky][4 * q4 + 1] = v.y; r[ky][4 * q4 + 2] = v.z; r[ky][4 * q4 + 3] = v.w;
        }
      }
    }
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      if (d < nrow) {
        const int iy = iy0 + d;
        const bool rowok = wy * 7 + iy < H;
#pragma unroll
        for (int ix = 0; ix < 7; ++ix) {
          float v = dwk[0] * r[d][ix];  // one FMA per tap (a plain sum of products vectorises into pk_mul + add)
#pragma unroll
          for (int t = 1; t < 9; ++t) v = fmaf(dwk[t], r[d + t / 3][ix + t % 3], v);
          T[(iy * 7 + ix) * LT + dw_c] = (rowok && wx * 7 + ix < W) ? v : 0.f;
        }
      }
    }
  }
  __syncthreads();
  X3_STAMP(2);

  // ---- LN1 -> X planes; Q weight chunk 0 -> X after the U1 planes (the halo there has been read) ----
  ln_planes<C, LT, PS, PL, SWZ>(T, P, p.ln1_eps, tid);
  h16_t* QW = P + 2 * PL;  // [2 k step][2 plane][4 column block][64 lanes][8]
  h16_t* qdst = QW + qblk * 512 + 16 * (tid & 31);
  *reinterpret_cast<uint4*>(qdst) = qc0a;
  *reinterpret_cast<uint4*>(qdst + 8) = qc0b;
  *reinterpret_cast<uint4*>(qdst + 4096) = qc1a;
  *reinterpret_cast<uint4*>(qdst + 4104) = qc1b;
  WP<C, 1> f_q;  // K weight planes of column block wid
  load_wp(p.win, 3 * C, C, 0, C / 16 + wid, f_q, lane);
  __syncthreads();
  X3_STAMP(3);

  // ---- QKV = U1 Win'^T + b_in' (weight planes hold 64 W). Wave w computes Q of its own 16 query rows (four column
  // blocks of one row block: kept in registers for the attention) and the K and V column blocks w of all 64 token
  // rows; K and V replace U1 in X as planes after every wave has read U1 ----
  h16_t* Vt = P;                 // V^T planes [2][C][PSV]: d rows, key columns 0..63 (keys 49..63 finite padding)
  h16_t* Kp = P + 2 * C * PSV;   // K planes [2][NR][PSK]
  f32x4 qa[C / 16];              // lane: 64 Q[q = 16 wid + l15][cb*16 + 4g .. +3], cb = 0..C/16-1
  f32x4 akv[2][4][1];            // 64 K (0) / 64 V (1) of column block wid, row blocks 0..3
  {
    const int l15_ = l15;
    f16x8_t ua[C / 32][2];
#pragma unroll
    for (int s2 = 0; s2 < C / 32; ++s2) {
      const h16_t* ar = P + plane_off<PS, SWZ>(wid * 16 + l15_, 32 * s2 + 8 * g);
      ua[s2][0] = *reinterpret_cast<const f16x8_t*>(ar);
      ua[s2][1] = *reinterpret_cast<const f16x8_t*>(ar + PL);
    }
    WP<C, 1> f_n;  // V weight planes of column block wid
    load_wp(p.win, 3 * C, C, 0, 2 * C / 16 + wid, f_n, lane);
#pragma unroll
    for (int cq = 0; cq < C / 16; ++cq) qa[cq] = *reinterpret_cast<const f32x4*>(par + P_BIN + cq * 16 + 4 * g);
    static_assert(C == 64, "two 32-k chunks");
#pragma unroll
    for (int s2 = 0; s2 < C / 32; ++s2) {
      const h16_t* wq = QW + s2 * 4096 + lane * 8;
#pragma unroll
      for (int cq = 0; cq < C / 16; ++cq)
        qa[cq] = mfma_f16x3(*reinterpret_cast<const f16x8_t*>(wq + cq * 512),
                            *reinterpret_cast<const f16x8_t*>(wq + (4 + cq) * 512), ua[s2][0], ua[s2][1], qa[cq]);
    }
    {
      // K (token-major tile, as the attention reads it) and V (transposed tile: 4 consecutive keys of one head
      // dim per lane, stored as V^T rows with 8-byte writes)
      const f32x4 bk = *reinterpret_cast<const f32x4*>(par + P_BIN + (C / 16 + wid) * 16 + 4 * g);
      const float bv = par[P_BIN + 2 * C + wid * 16 + l15];
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        akv[0][rb][0] = bk;
        akv[1][rb][0] = f32x4{bv, bv, bv, bv};
      }
      gemm_x3<C, 1, PS, PL, false, SWZ>(P, f_q, akv[0], lane);
      gemm_x3<C, 1, PS, PL, true, SWZ>(P, f_n, akv[1], lane);
    }
  }
  WP<C, 1> f_o;
  load_wp(p.wo, C, C, 0, wid, f_o, lane);  // out-proj planes: in flight during attention
  __syncthreads();  // every wave has read U1
  X3_STAMP(6);
#pragma unroll
  for (int rb = 0; rb < 4; ++rb) {
    const int tok = rb * 16 + l15;
    if (tok < NR) store_planes4<PSK, KPL, false, SWZ>(Kp, tok, wid * 16 + 4 * g, akv[0][rb][0]);  // K, V, Q stay x64
    rng = range_acc(range_acc(rng, akv[0][rb][0]), akv[1][rb][0]);
    uint2 h, l;
    split4(akv[1][rb][0], h, l);  // V^T[d = wid*16 + l15][keys rb*16 + 4g .. +3]
    h16_t* vd = Vt + plane_off8<PSV, SWZ>(wid * 16 + l15, rb * 16 + 4 * g);
    *reinterpret_cast<uint2*>(vd) = h;
    *reinterpret_cast<uint2*>(vd + VPL) = l;
  }
  // this wave's queries as the B operand of S^T = K Q^T, per head: k slot j of lane group g is head dim
  // 4g + j (j < 4) or 16 + 4g + j - 4 (the lane's own two Q column blocks); K is read with the same permutation
  f16x8_t qh[NH], ql[NH];
#pragma unroll
  for (int hh = 0; hh < NH; ++hh) {
    uint2 h0, l0, h1, l1;
    split4(qa[2 * hh], h0, l0);
    split4(qa[2 * hh + 1], h1, l1);
    rng = range_acc(range_acc(rng, qa[2 * hh]), qa[2 * hh + 1]);
    qh[hh] = __builtin_bit_cast(f16x8_t, make_uint4(h0.x, h0.y, h1.x, h1.y));
    ql[hh] = __builtin_bit_cast(f16x8_t, make_uint4(l0.x, l0.y, l1.x, l1.y));
  }
  __syncthreads();  // K / V planes complete
  X3_STAMP(7);
  WP<C, 1> f_1a;
  load_wp(p.w1, HID, C, 0, wid, f_1a, lane);  // MLP1 (hidden half 0) planes

  // ---- attention on fp16 two-term splits, wave = 16 queries, all heads: S^T[key][q] (keys 0..63 in four 16-row
  // blocks; keys >= 49 masked) -> softmax over keys (raw scores, exp2, 1/sum applied to O) -> O^T = V^T P^T with
  // the S^T accumulators as the P^T operand (MFMA step s takes key blocks 2s and 2s+1: slot j of lane group g is
  // key 32s + 4g + j (j < 4) or 32s + 16 + 4g + j - 4) ----
  f32x4 ov[NH][HD / 16];
  {
    f32x4 st[NH][4];
#pragma unroll
    for (int hh = 0; hh < NH; ++hh)
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const int row = kb * 16 + l15 < NR ? kb * 16 + l15 : NR - 1;
        const h16_t* kr0 = Kp + plane_off8<PSK, SWZ>(row, hh * HD + 4 * g);
        const h16_t* kr1 = Kp + plane_off8<PSK, SWZ>(row, hh * HD + 4 * g + 16);
        const uint2 a0 = *reinterpret_cast<const uint2*>(kr0), a1 = *reinterpret_cast<const uint2*>(kr1);
        const uint2 b0 = *reinterpret_cast<const uint2*>(kr0 + KPL), b1 = *reinterpret_cast<const uint2*>(kr1 + KPL);
        const f16x8_t kh = __builtin_bit_cast(f16x8_t, make_uint4(a0.x, a0.y, a1.x, a1.y));
        const f16x8_t kl = __builtin_bit_cast(f16x8_t, make_uint4(b0.x, b0.y, b1.x, b1.y));
        f32x4 c = mfma16(kl, qh[hh], f32x4{0.f, 0.f, 0.f, 0.f});
        c = mfma16(kh, ql[hh], c);
        st[hh][kb] = mfma16(kh, qh[hh], c);
      }
    const float c2 = p.scale * 1.44269504088896341f * (1.0f / (WSC * WSC));  // S = 4096 Q K^T
    float inv[NH];
#pragma unroll
    for (int hh = 0; hh < NH; ++hh) {
      float mx = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float sv = (kb * 16 + 4 * g + r < NR) ? st[hh][kb][r] : -INFINITY;
          st[hh][kb][r] = sv;
          mx = fmaxf(mx, sv);
        }
      mx = xor32_max(xor16_max(mx));
      const float mc = -mx * c2;
      float sum = 0.f;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __builtin_amdgcn_exp2f(fmaf(st[hh][kb][r], c2, mc));
          st[hh][kb][r] = e;
          sum += e;
        }
      inv[hh] = __builtin_amdgcn_rcpf(group4_sum(sum)) * (1.0f / WSC);  // V is x64
    }
#pragma unroll
    for (int hh = 0; hh < NH; ++hh) {
#pragma unroll
      for (int db = 0; db < HD / 16; ++db) ov[hh][db] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        uint2 h0, l0, h1, l1;
        split4(st[hh][2 * s2], h0, l0);
        split4(st[hh][2 * s2 + 1], h1, l1);
        const f16x8_t ph = __builtin_bit_cast(f16x8_t, make_uint4(h0.x, h0.y, h1.x, h1.y));
        const f16x8_t pl = __builtin_bit_cast(f16x8_t, make_uint4(l0.x, l0.y, l1.x, l1.y));
#pragma unroll
        for (int db = 0; db < HD / 16; ++db) {
          const h16_t* vr0 = Vt + plane_off8<PSV, SWZ>(hh * HD + db * 16 + l15, 32 * s2 + 4 * g);
          const h16_t* vr1 = Vt + plane_off8<PSV, SWZ>(hh * HD + db * 16 + l15, 32 * s2 + 4 * g + 16);
          const uint2 a0 = *reinterpret_cast<const uint2*>(vr0), a1 = *reinterpret_cast<const uint2*>(vr1);
          const uint2 b0 = *reinterpret_cast<const uint2*>(vr0 + VPL), b1 = *reinterpret_cast<const uint2*>(vr1 + VPL);
          const f16x8_t vh = __builtin_bit_cast(f16x8_t, make_uint4(a0.x, a0.y, a1.x, a1.y));
          const f16x8_t vl = __builtin_bit_cast(f16x8_t, make_uint4(b0.x, b0.y, b1.x, b1.y));
          f32x4 c = mfma16(vl, ph, ov[hh][db]);
          c = mfma16(vh, pl, c);
          ov[hh][db] = mfma16(vh, ph, c);
        }
      }
#pragma unroll
      for (int db = 0; db < HD / 16; ++db) ov[hh][db] *= inv[hh];
    }
  }
  __syncthreads();
  X3_STAMP(8);
#pragma unroll
  for (int h = 0; h < NH; ++h)
#pragma unroll
    for (int db = 0; db < HD / 16; ++db)
    {
      store_planes4<PS, PL, SWZ>(P, wid * 16 + l15, h * HD + db * 16 + 4 * g, ov[h][db]);
      rng = range_acc(rng, ov[h][db]);
    }
  __syncthreads();
  X3_STAMP(9);

  // ---- T += O Wo^T + bo ----
  WP<C, 1> f_1b;
  load_wp(p.w1, HID, C, 0, wid + 4, f_1b, lane);  // MLP1 (hidden half 1) planes
  {
    f32x4 acc[4][1];
    const f32x4 b = *reinterpret_cast<const f32x4*>(par + P_BO + wid * 16 + 4 * g);
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) acc[rb][0] = b;
    gemm_x3<C, 1, PS, PL, false, SWZ>(P, f_o, acc, lane);
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      const int tok = rb * 16 + l15;
      if (rb < 3 || l15 == 0) {
        f32x4* tp = reinterpret_cast<f32x4*>(T + tok * LT + wid * 16 + 4 * g);
        *tp = *tp + acc[rb][0] * (1.0f / WSC);
      }
    }
  }
  __syncthreads();
  X3_STAMP(10);

  // ---- LN2 -> X planes ----
  ln_planes<C, LT, PS, PL, SWZ>(T, P, p.ln2_eps, tid);
  WP<C, 1> f_2a;
  load_wp(p.w2, C, HID, 0, wid, f_2a, lane);  // MLP2 planes, k in [0, 64)
  __syncthreads();
  X3_STAMP(11);

  // ---- MLP: both hidden halves Hh = GELU(U2 W1h'^T + b1h') into registers; then half by half as planes into X,
  // each followed by its MLP2 partial acc2 += Hh W2[:, half]^T ----
  f32x4 hid[2][4];
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    f32x4 acc[4][1];
    const f32x4 b = *reinterpret_cast<const f32x4*>(par + P_B1 + (wid + 4 * half) * 16 + 4 * g);
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) acc[rb][0] = b;
    gemm_x3<C, 1, PS, PL, false, SWZ>(P, half == 0 ? f_1a : f_1b, acc, lane);
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      const f32x4 a = acc[rb][0] * (1.0f / WSC);
      const f32x2 lo = gelu2_fast_(f32x2{a[0], a[1]});
      const f32x2 hi = gelu2_fast_(f32x2{a[2], a[3]});
      hid[half][rb] = f32x4{lo.x, lo.y, hi.x, hi.y};
    }
  }
  WP<C, 1> f_2b;
  load_wp(p.w2, C, HID, C, wid, f_2b, lane);  // MLP2 planes, k in [64, 128)
  f32x4 acc2[4][1];
  {
    const f32x4 b = *reinterpret_cast<const f32x4*>(par + P_B2 + wid * 16 + 4 * g);
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) acc2[rb][0] = b;
  }
  // both hidden halves as planes side by side [64][PSH] (one store, one barrier), then MLP2 over k in [0, 128)
  __syncthreads();  // every wave has read X (U2)
  X3_STAMP(12);
#pragma unroll
  for (int half = 0; half < 2; ++half)
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      store_planes4<PSH, PLH>(P, rb * 16 + l15, 64 * half + wid * 16 + 4 * g, hid[half][rb]);
      rng = range_acc(rng, hid[half][rb]);
    }
  __syncthreads();
  X3_STAMP(13);
  gemm_x3<C, 1, PSH, PLH>(P, f_2a, acc2, lane);
  gemm_x3<C, 1, PSH, PLH>(P + 64, f_2b, acc2, lane);  // hidden columns 64..127

  // pw planes and this lane's residual x / BN terms: in flight during the final T update
  WP<C, 1> f_pw;
  load_wp(p.wpw, C, C, 0, wid, f_pw, lane);
  const __amdgpu_buffer_rsrc_t ry = rsrc_of(p.y + (long)img * C * HWi);
  unsigned vtok[4];  // byte offset of (channel wid*16 + 4g, token tb*16 + l15), or out of range
#pragma unroll
  for (int tb = 0; tb < 4; ++tb) {
    const int tok = tb * 16 + l15;
    const int iy = tok / 7, ix = tok - (tok / 7) * 7;
    const int hh = wy * 7 + iy, wc = wx * 7 + ix;
    vtok[tb] = (tok < NR && hh < H && wc < W) ? (unsigned)(((wid * 16 + 4 * g) * HWi + hh * W + wc) * 4) : OOB;
  }
  float xr[4][4];
#pragma unroll
  for (int tb = 0; tb < 4; ++tb)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      xr[tb][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, vtok[tb], r * HWi * 4, 0));

  // ---- final T = T + MLP -> X planes (rows >= 49 zero): the pw GEMM's operand ----
  __syncthreads();  // every wave has read the hidden planes
  X3_STAMP(16);
#pragma unroll
  for (int rb = 0; rb < 4; ++rb) {
    const int tok = rb * 16 + l15;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (tok < NR) v = *reinterpret_cast<const f32x4*>(T + tok * LT + wid * 16 + 4 * g) + acc2[rb][0] * (1.0f / WSC);
    store_planes4<PS, PL, SWZ>(P, tok, wid * 16 + 4 * g, v);
    rng = range_acc(rng, v);
  }
  range_report(p.range_flag, rng);
  prep_report(p.prep_flag, p.range_flag);
  __syncthreads();
  X3_STAMP(17);

  // ---- y = x + SiLU(BN(Wpw T^T)): tile Y^T[c][tok], lane holds c = wid*16 + 4g + r, token tb*16 + l15 ----
  {
    f32x4 acc[4][1];
#pragma unroll
    for (int tb = 0; tb < 4; ++tb) acc[tb][0] = f32x4{0.f, 0.f, 0.f, 0.f};
    gemm_x3<C, 1, PS, PL, false, SWZ>(P, f_pw, acc, lane);
    const f32x4 sc = *reinterpret_cast<const f32x4*>(par + P_SC + wid * 16 + 4 * g);
    const f32x4 sh = *reinterpret_cast<const f32x4*>(par + P_SH + wid * 16 + 4 * g);
#pragma unroll
    for (int tb = 0; tb < 4; ++tb)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        __builtin_amdgcn_raw_buffer_store_b32(
            __builtin_bit_cast(unsigned, xr[tb][r] + silu_fast_(acc[tb][0][r] * sc[r] + sh[r])), ry, vtok[tb],
            r * HWi * 4, 0);
  }  X3_STAMP(18);
}

// ---- C = 256 (the P4 instance L9: 4 heads of 64, MLP hidden 512) -------------------------------------------------
// One 512-thread workgroup (8 waves, 2 per SIMD) per 7x7 window, one per CU (LDS 154 KB): T (fp32 residual stream
// [49][260]) | U (two fp16 planes [49][264]: LN1 output, then LN2 output, then the final T for the pw GEMM) | WR
// (work region: V^T + K planes of a head pair -> O planes of the pair -> an MLP hidden chunk's planes). The halo of
// the depthwise conv uses U + WR. Rows >= 49 of a B operand are read clamped to row 48 (finite; their outputs are
// dropped). Per head pair: wave (lh, qb) = (local head, 16-query block) computes its Q tile row (four column
// blocks, kept in registers) and K / V column block w of the pair for all token rows; attention as in the C = 64
// kernel; the out-projection's partial product over the pair's 128 input channels accumulates in registers. The
// MLP runs in two hidden chunks of 256 (MLP2 partials in registers). Weight planes stream from L2 per wave in
// 64-k steps with one step of lookahead.
namespace wx {
constexpr int C = 256;
constexpr int HD = 64;
constexpr int HID = 512;
constexpr int NT = 512;
constexpr int LT = C + 4;           // T row stride (floats)
// U / hidden-chunk and O planes: rows padded to 272 / 144 elements with the 16-byte chunks of a row swizzled in their
// low two index bits by row bits 2-3 (swz_row): the GEMM operand reads (ds_read_b128, lane = (row l15, chunk g) + k)
// are then conflict-free and the swizzle stays additive in k (at 264 / 136 unswizzled they were 2-way); the accumulator
// stores (ds_write_b64, 16 rows x one column group) stay 2-way
constexpr int PSU = 272;            // U / hidden-chunk plane row stride (fp16)
constexpr int UPL = NR * PSU;       // plane stride (49 rows)
constexpr int PSK = 128 + 8;        // K planes of a head pair [49][PSK]
constexpr int KPL = NR * PSK;
constexpr int PSV = 56;             // V^T planes of a head pair [128][PSV]: keys 0..55 stored; the MFMA reads keys
constexpr int VPL = 128 * PSV;      // up to 63 (P = 0 there), i.e. into the next row / the K planes (finite)
constexpr int PSO = 144;            // O planes of a head pair [64][PSO]
constexpr int OPL = 64 * PSO;
constexpr int QBUF = 2 * 8 * 512;   // staged Q weight fragments of one 32-k step (2 planes x 8 column blocks)
constexpr int HALF = 128;           // channels per halo half
constexpr int NRH = (HALF + 5) / 6; // halo steps per half (6 channels per step)
constexpr int T_B = NR * LT * 4;
constexpr int U_B = 2 * UPL * 2;
constexpr int KV_B = (2 * VPL + 2 * KPL) * 2;
constexpr int O_B = 2 * OPL * 2;
constexpr int WR_B = KV_B > O_B ? (KV_B > U_B ? KV_B : U_B) : (O_B > U_B ? O_B : U_B);
constexpr int HALO_B = 54 * NRH * HPW * 4;
static_assert(HALO_B <= U_B + WR_B, "halo patch");
static_assert(2 * QBUF * 2 <= WR_B, "staged Q weights");
static_assert(T_B % 16 == 0 && U_B % 16 == 0 && WR_B % 16 == 0, "16-byte aligned regions");
static_assert(T_B + U_B + WR_B <= 160 * 1024, "LDS");

__device__ __forceinline__ int swz_row(int row) { return ((row >> 2) & 1) | (((row >> 3) & 1) << 1); }
// element (row, col) of a swizzled U / hidden / O plane
template <int PS>
__device__ __forceinline__ int poff(int row, int col) {
  return row * PS + ((((col >> 3) ^ swz_row(row))) << 3) + (col & 7);
}
// the two planes of 4 consecutive elements of row `row`, column `col` (a multiple of 4), swizzled
template <int PS, int PL>
__device__ __forceinline__ void store4(h16_t* P, int row, int col, f32x4 v) {
  uint2 h, l;
  split4(v, h, l);
  h16_t* d = P + poff<PS>(row, col);
  *reinterpret_cast<uint2*>(d) = h;
  *reinterpret_cast<uint2*>(d + PL) = l;
}

// acc[rb][j] += (B rows (rb0 + rb)*16 + l15 . W[cb[j]*16 + l15]^T)^T over k in [koff, koff + K): W = two fp16
// planes [2][N][KT] in global memory (L2), the token rows = two LDS planes (row stride PS, plane stride PL; rows
// clamped to 48 when CLAMP). Weight fragments of KS 32-k steps are loaded one step ahead.
template <int K, int NJ, int NRB, int KS, int PS, int PL, bool CLAMP>
__device__ __forceinline__ void gemm_w(const h16_t* __restrict__ Wp, int N, int KT, int koff, const int (&cb)[NJ],
                                       const h16_t* A, int rb0, f32x4 (&acc)[NRB][NJ], int lane) {
  const int l15 = lane & 15, g = lane >> 4;
  constexpr int NST = K / (32 * KS);
  static_assert(K % (32 * KS) == 0, "k steps");
  const long pst = (long)N * KT;
  const h16_t* wr[NJ];  // fragment-major planes: (column block, 32-k step) fragments are 1 KB contiguous
#pragma unroll
  for (int j = 0; j < NJ; ++j) wr[j] = Wp + ((long)(cb[j] * (KT / 32) + koff / 32) * 64 + lane) * 8;
  const h16_t* ar[NRB];
#pragma unroll
  for (int rb = 0; rb < NRB; ++rb) {
    int row = (rb0 + rb) * 16 + l15;
    if (CLAMP) row = row < NR ? row : NR - 1;
    ar[rb] = A + row * PS + 8 * (g ^ swz_row(row));  // k steps are whole 4-chunk groups: the swizzle adds
  }
  f16x8_t w0[KS][NJ][2], w1[KS][NJ][2];
  auto ldw = [&](f16x8_t (&w)[KS][NJ][2], int st) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int p = 0; p < 2; ++p)
          w[ks][j][p] = *reinterpret_cast<const f16x8_t*>(wr[j] + p * pst + 512 * (st * KS + ks));
  };
  auto mma = [&](const f16x8_t (&w)[KS][NJ][2], int st) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k0 = 32 * (st * KS + ks);
#pragma unroll
      for (int rb = 0; rb < NRB; ++rb) {
        const f16x8_t ah = *reinterpret_cast<const f16x8_t*>(ar[rb] + k0);
        const f16x8_t al = *reinterpret_cast<const f16x8_t*>(ar[rb] + PL + k0);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          f32x4 c = mfma16(w[ks][j][1], ah, acc[rb][j]);
          c = mfma16(w[ks][j][0], al, c);
          acc[rb][j] = mfma16(w[ks][j][0], ah, c);
        }
      }
    }
  };
  // The prefetches stay where they are (sched barriers): the scheduler otherwise sinks each step's loads to the end
  // of the previous step, right before their first use. Unconditional (the last step reloads a step, L2-hot): a
  // load under a branch merges into a phi whose copy waits for every load in flight.
  static_assert(NST % 2 == 0 || NST == 1, "steps in pairs");
  ldw(w0, 0);
  if constexpr (NST == 1) {
    mma(w0, 0);
  } else {
#pragma unroll 1
    for (int st = 0; st < NST; st += 2) {
      ldw(w1, st + 1);
      __builtin_amdgcn_sched_barrier(0);
      mma(w0, st);
      ldw(w0, st + 2 < NST ? st + 2 : st);
      __builtin_amdgcn_sched_barrier(0);
      mma(w1, st + 1);
    }
  }
}

// LayerNorm (normalisation only; the affine is folded into the next GEMM's weights) of T rows [0, 49) into the two
// U planes: 8 lanes per row (512 threads = 64 rows), 32 values each - lane `part` takes columns part*8 + 64j .. +7
// (j = 0..3), so the 8 lanes of a row store one contiguous 128-byte run per j (with 32 contiguous columns per lane
// the plane stores were 4-way bank conflicts)
__device__ __forceinline__ void ln_planes8(const float* T, h16_t* U, float eps, int tid) {
  const int r = tid >> 3, part = tid & 7;
  const bool valid = r < NR;
  f32x4 v[8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    v[i] = valid ? *reinterpret_cast<const f32x4*>(T + r * LT + part * 8 + 64 * (i >> 1) + 4 * (i & 1))
                 : f32x4{0.f, 0.f, 0.f, 0.f};
    s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  }
  s = quad_sum(s);
  s += __shfl_xor(s, 4, 64);
  const float mean = s * (1.0f / (float)C);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    v[i] -= mean;
    q += (v[i].x * v[i].x + v[i].y * v[i].y) + (v[i].z * v[i].z + v[i].w * v[i].w);
  }
  q = quad_sum(q);
  q += __shfl_xor(q, 4, 64);
  const float rs = __builtin_amdgcn_rsqf(q * (1.0f / (float)C) + eps);
  if (valid) {
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
      uint2 h0, l0, h1, l1;
      split4(v[i] * rs, h0, l0);
      split4(v[i + 1] * rs, h1, l1);
      h16_t* d = U + poff<PSU>(r, part * 8 + 64 * (i >> 1));
      *reinterpret_cast<uint4*>(d) = make_uint4(h0.x, h0.y, h1.x, h1.y);
      *reinterpret_cast<uint4*>(d + UPL) = make_uint4(l0.x, l0.y, l1.x, l1.y);
    }
  }
}

#ifdef YS_DIAG_STAMPS  // diagnostic builds only (scripts/diag_wx.sh): per-stage s_memtime of wave 0 of the first 256 windows
__device__ unsigned long long ys_wx_stamps[256 * 32];
#define WX_STAMP(k)                                                                                                  \
  do {                                                                                                               \
    if (threadIdx.x == 0 && blockIdx.x < 256) ys_wx_stamps[blockIdx.x * 32 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define WX_STAMP(k) \
  do {              \
  } while (0)
#endif

__device__ __forceinline__ f32x4 ld_bias4(const float* b, int n) { return *reinterpret_cast<const f32x4*>(b + n) * WSC; }

__global__ __launch_bounds__(NT, 1) void swin_wx_kernel(Args p) {
  __shared__ __attribute__((aligned(16))) char smem[T_B + U_B + WR_B];
  float* T = reinterpret_cast<float*>(smem);
  h16_t* UP = reinterpret_cast<h16_t*>(smem + T_B);
  h16_t* WR = reinterpret_cast<h16_t*>(smem + T_B + U_B);
  float* HALO = reinterpret_cast<float*>(smem + T_B);
  h16_t* Vt = WR;              // [2][128][PSV]
  h16_t* Kp = WR + 2 * VPL;    // [2][49][PSK]
  h16_t* Op = WR;              // [2][64][PSO]
  h16_t* Hp = WR;              // [2][49][PSU]

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, g = lane >> 4;
  const int H = p.H, W = p.W;
  const int HWi = H * W;  // per-image offsets are 32-bit (the launcher checks C*H*W < 2^30)
  float rng = 0.f;        // largest magnitude this thread splits outside a LayerNorm (split-range guard)

  const long nwin_total = (long)p.B * p.nWin;
  const long per_xcd = (nwin_total + 7) >> 3;
  const long gwl = (long)(blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  if (gwl >= nwin_total || (blockIdx.x >> 3) >= per_xcd) return;
  const int gw = __builtin_amdgcn_readfirstlane((int)gwl);
  const int img = gw / p.nWin, win = gw - (gw / p.nWin) * p.nWin;
  const int wy = win / p.nWx, wx_ = win - (win / p.nWx) * p.nWx;
  auto rsrc_of = [&](const float* base) {
    const unsigned long long a = (unsigned long long)base;
    return __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(a >> 32)) << 32) |
                (unsigned)__builtin_amdgcn_readfirstlane((unsigned)a)),
        (short)0, __builtin_amdgcn_readfirstlane(C * HWi * 4), 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rx = rsrc_of(p.x + (long)img * C * HWi);
  constexpr unsigned OOB = 0x80000000u;

  // halo of both channel halves into registers: row slot s = 7*wid + lane/9 < 54 is (channel 6i + s/9, patch row
  // s%9) at step i, lane%9 the column; out-of-image lanes get an out-of-range voffset (the buffer load returns 0)
  const int hl_r = lane / 9, hl_px = lane - (lane / 9) * 9;
  const int hslot = 7 * wid + hl_r;
  float hv[2][NRH];
  {
    const int hcs = hslot / 9, hpy = hslot - (hslot / 9) * 9;
    const int hh = wy * 7 - 1 + hpy, wc = wx_ * 7 - 1 + hl_px;
    const bool ok = hl_r < 7 && hslot < 54 && (unsigned)hh < (unsigned)H && (unsigned)wc < (unsigned)W;
    const unsigned voff = ok ? (unsigned)((hcs * HWi + hh * W + wc) * 4) : OOB;
    const unsigned vlast = (6 * (NRH - 1) + hcs < HALF) ? voff : OOB;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)
#pragma unroll
      for (int i = 0; i < NRH; ++i)
        hv[hf][i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                  rx, i == NRH - 1 ? vlast : voff, (hf * HALF + 6 * i) * HWi * 4, 0));
  }
  const int lh = wid >> 2, qb = wid & 3;  // attention: (local head, 16-query block)
  WX_STAMP(0);

  // ---- depthwise 3x3 per channel half: halo -> LDS [c][py][HPW] -> T (cropped / padded tokens = 0) ----
  const int dc = tid % HALF;
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    float dwk[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) dwk[i] = p.dw[(hf * HALF + dc) * 9 + i];
    if (hf) __syncthreads();  // previous half's dw reads done
    if (hl_r < 7 && hslot < 54) {
#pragma unroll
      for (int i = 0; i < NRH; ++i) HALO[(54 * i + hslot) * HPW + hl_px] = hv[hf][i];
    }
    __syncthreads();
    for (int item = tid; item < HALF * 7; item += NT) {
      const int iy = item / HALF;  // item % HALF == dc
      const float* hp = HALO + (dc * 9 + iy) * HPW;
      float r[3][12];
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int q4 = 0; q4 < 3; ++q4) {
          const float4 v = *reinterpret_cast<const float4*>(hp + ky * HPW + 4 * q4);
          r[ky][4 * q4] = v.x; r[ky][4 * q4 + 1] = v.y; r[ky][4 * q4 + 2] = v.z; r[ky][4 * q4 + 3] = v.w;
        }
      const bool rowok = wy * 7 + iy < H;
#pragma unroll
      for (int ix = 0; ix < 7; ++ix) {
        const float v = dwk[0] * r[0][ix] + dwk[1] * r[0][ix + 1] + dwk[2] * r[0][ix + 2] + dwk[3] * r[1][ix] +
                        dwk[4] * r[1][ix + 1] + dwk[5] * r[1][ix + 2] + dwk[6] * r[2][ix] + dwk[7] * r[2][ix + 1] +
                        dwk[8] * r[2][ix + 2];
        T[(iy * 7 + ix) * LT + hf * HALF + dc] = (rowok && wx_ * 7 + ix < W) ? v : 0.f;
      }
    }
  }
  __syncthreads();
  WX_STAMP(1);
  ln_planes8(T, UP, p.ln1_eps, tid);
  __syncthreads();
  WX_STAMP(2);

  // ---- attention on head pairs; out-projection partials (this wave's column blocks wid, wid + 8) in registers ----
  const int cbo[2] = {wid, wid + 8};
  f32x4 acc_o[4][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const f32x4 b = ld_bias4(p.bo, cbo[j] * 16 + 4 * g);
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) acc_o[rb][j] = b;
  }
  const float c2 = p.scale * 1.44269504088896341f * (1.0f / (WSC * WSC));  // S = 4096 Q K^T
#pragma unroll 1
  for (int hp = 0; hp < 2; ++hp) {
    // Q of this wave's queries (head 2hp + lh): in_proj rows hp*128 + lh*64 + [0, 64). The four waves of a head
    // need the same Q weight planes, so the pair's 128 Q rows are staged once per workgroup through WR (free until
    // the K / V stores) in 32-k chunks, double-buffered, instead of being streamed by every wave: the weight
    // stream from L2 (~17 B/clk per CU here) was the Q GEMM's bound, at twice the KV GEMM's time for half its MFMAs
    f32x4 qa[1][4];
    {
#pragma unroll
      for (int t = 0; t < 4; ++t) qa[0][t] = ld_bias4(p.bin, (hp * 128 + lh * 64 + 16 * t) + 4 * g);
      if (hp) __syncthreads();  // the previous pair's out-projection has read its O planes (WR)
      h16_t* QW = WR;  // [2 buf][2 plane][8 column block][64 lanes][8]: the fragment blocks of one 32-k step
      const int qblk = tid >> 5, qpl = qblk >> 3, qcb = qblk & 7;
      const h16_t* qsrc = p.win + (long)qpl * 3 * C * C + (long)((hp * 8 + qcb) * (C / 32)) * 512 + 16 * (tid & 31);
      h16_t* qdst = QW + qblk * 512 + 16 * (tid & 31);
      uint4 qv0 = *reinterpret_cast<const uint4*>(qsrc), qv1 = *reinterpret_cast<const uint4*>(qsrc + 8);
      *reinterpret_cast<uint4*>(qdst) = qv0;
      *reinterpret_cast<uint4*>(qdst + 8) = qv1;
      __syncthreads();
      const int urow = qb * 16 + l15 < NR ? qb * 16 + l15 : NR - 1;
      const h16_t* ub = UP + urow * PSU + 8 * (g ^ swz_row(urow));
#pragma unroll 1
      for (int kc = 0; kc < C / 32; ++kc) {
        const int buf = kc & 1;
        if (kc + 1 < C / 32) {  // next chunk's planes: in flight during this chunk's MFMAs
          qv0 = *reinterpret_cast<const uint4*>(qsrc + 512 * (kc + 1));
          qv1 = *reinterpret_cast<const uint4*>(qsrc + 512 * (kc + 1) + 8);
        }
        const f16x8_t bh = *reinterpret_cast<const f16x8_t*>(ub + 32 * kc);
        const f16x8_t bl = *reinterpret_cast<const f16x8_t*>(ub + UPL + 32 * kc);
        const h16_t* wq = QW + buf * QBUF + (lh * 4) * 512 + lane * 8;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const f16x8_t ah = *reinterpret_cast<const f16x8_t*>(wq + t * 512);
          const f16x8_t al = *reinterpret_cast<const f16x8_t*>(wq + 8 * 512 + t * 512);
          qa[0][t] = mfma_f16x3(ah, al, bh, bl, qa[0][t]);
        }
        if (kc + 1 < C / 32) {
          h16_t* d = qdst + (buf ^ 1) * QBUF;
          *reinterpret_cast<uint4*>(d) = qv0;
          *reinterpret_cast<uint4*>(d + 8) = qv1;
        }
        __syncthreads();
      }
    }
    WX_STAMP(3 + 6 * hp);
    // K / V column block wid of the pair, all token rows
    f32x4 akv[4][2];
    {
      const int cbkv[2] = {(C + hp * 128) / 16 + wid, (2 * C + hp * 128) / 16 + wid};
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const f32x4 b = ld_bias4(p.bin, cbkv[j] * 16 + 4 * g);
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) akv[rb][j] = b;
      }
      gemm_w<C, 2, 4, 2, PSU, UPL, true>(p.win, 3 * C, C, 0, cbkv, UP, 0, akv, lane);
    }
    WX_STAMP(4 + 6 * hp);
    __syncthreads();  // every wave has read the staged Q planes (WR)
    WX_STAMP(5 + 6 * hp);
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      const int tok = rb * 16 + l15;
      if (tok < NR) store_planes4<PSK, KPL>(Kp, tok, wid * 16 + 4 * g, akv[rb][0]);  // K, V, Q stay x64
      rng = range_acc(range_acc(rng, akv[rb][0]), akv[rb][1]);
      if (tok < PSV) {
        uint2 h, l;
        split4(akv[rb][1], h, l);
        h16_t* vd = Vt + (wid * 16 + 4 * g) * PSV + tok;
        vd[0] = (h16_t)(h.x & 0xffffu);
        vd[PSV] = (h16_t)(h.x >> 16);
        vd[2 * PSV] = (h16_t)(h.y & 0xffffu);
        vd[3 * PSV] = (h16_t)(h.y >> 16);
        vd[VPL] = (h16_t)(l.x & 0xffffu);
        vd[VPL + PSV] = (h16_t)(l.x >> 16);
        vd[VPL + 2 * PSV] = (h16_t)(l.y & 0xffffu);
        vd[VPL + 3 * PSV] = (h16_t)(l.y >> 16);
      }
    }
    // Q as the B operand of S^T = K Q^T, per 32-d step s: slot j of lane group g is d = 32s + 4g + j (j < 4) or
    // 32s + 16 + 4g + j - 4 (the lane's own Q tiles 2s, 2s + 1); K is read with the same permutation
    f16x8_t qh[2], ql[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      uint2 h0, l0, h1, l1;
      split4(qa[0][2 * s], h0, l0);
      split4(qa[0][2 * s + 1], h1, l1);
      rng = range_acc(range_acc(rng, qa[0][2 * s]), qa[0][2 * s + 1]);
      qh[s] = __builtin_bit_cast(f16x8_t, make_uint4(h0.x, h0.y, h1.x, h1.y));
      ql[s] = __builtin_bit_cast(f16x8_t, make_uint4(l0.x, l0.y, l1.x, l1.y));
    }
    __syncthreads();  // K / V^T planes complete
    WX_STAMP(6 + 6 * hp);
    f32x4 ov[HD / 16];
    {
      f32x4 st[4];
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const int row = kb * 16 + l15 < NR ? kb * 16 + l15 : NR - 1;
        f32x4 c = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const h16_t* kr = Kp + row * PSK + lh * HD + 32 * s + 4 * g;
          const uint2 a0 = *reinterpret_cast<const uint2*>(kr), a1 = *reinterpret_cast<const uint2*>(kr + 16);
          const uint2 b0 = *reinterpret_cast<const uint2*>(kr + KPL), b1 = *reinterpret_cast<const uint2*>(kr + KPL + 16);
          const f16x8_t kh = __builtin_bit_cast(f16x8_t, make_uint4(a0.x, a0.y, a1.x, a1.y));
          const f16x8_t kl = __builtin_bit_cast(f16x8_t, make_uint4(b0.x, b0.y, b1.x, b1.y));
          c = mfma16(kl, qh[s], c);
          c = mfma16(kh, ql[s], c);
          c = mfma16(kh, qh[s], c);
        }
        st[kb] = c;
      }
      float mx = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float sv = (kb * 16 + 4 * g + r < NR) ? st[kb][r] : -INFINITY;
          st[kb][r] = sv;
          mx = fmaxf(mx, sv);
        }
      mx = xor32_max(xor16_max(mx));
      const float mc = -mx * c2;
      float sum = 0.f;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __builtin_amdgcn_exp2f(fmaf(st[kb][r], c2, mc));
          st[kb][r] = e;
          sum += e;
        }
      const float inv = __builtin_amdgcn_rcpf(group4_sum(sum)) * (1.0f / WSC);  // V is x64
#pragma unroll
      for (int db = 0; db < HD / 16; ++db) ov[db] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        uint2 h0, l0, h1, l1;
        split4(st[2 * s2], h0, l0);
        split4(st[2 * s2 + 1], h1, l1);
        const f16x8_t ph = __builtin_bit_cast(f16x8_t, make_uint4(h0.x, h0.y, h1.x, h1.y));
        const f16x8_t pl = __builtin_bit_cast(f16x8_t, make_uint4(l0.x, l0.y, l1.x, l1.y));
#pragma unroll
        for (int db = 0; db < HD / 16; ++db) {
          const h16_t* vr = Vt + (lh * HD + db * 16 + l15) * PSV + 32 * s2 + 4 * g;
          const uint2 a0 = *reinterpret_cast<const uint2*>(vr), a1 = *reinterpret_cast<const uint2*>(vr + 16);
          const uint2 b0 = *reinterpret_cast<const uint2*>(vr + VPL), b1 = *reinterpret_cast<const uint2*>(vr + VPL + 16);
          const f16x8_t vh = __builtin_bit_cast(f16x8_t, make_uint4(a0.x, a0.y, a1.x, a1.y));
          const f16x8_t vl = __builtin_bit_cast(f16x8_t, make_uint4(b0.x, b0.y, b1.x, b1.y));
          f32x4 c = mfma16(vl, ph, ov[db]);
          c = mfma16(vh, pl, c);
          ov[db] = mfma16(vh, ph, c);
        }
      }
#pragma unroll
      for (int db = 0; db < HD / 16; ++db) ov[db] *= inv;
    }
    __syncthreads();  // every wave has read K / V^T
    WX_STAMP(7 + 6 * hp);
#pragma unroll
    for (int db = 0; db < HD / 16; ++db)
    {
      store4<PSO, OPL>(Op, qb * 16 + l15, lh * HD + db * 16 + 4 * g, ov[db]);
      rng = range_acc(rng, ov[db]);
    }
    __syncthreads();
    gemm_w<128, 2, 4, 2, PSO, OPL, false>(p.wo, C, C, hp * 128, cbo, Op, 0, acc_o, lane);
    WX_STAMP(8 + 6 * hp);
  }
  // T += O Wo^T + bo (this wave's column blocks; rows < 49)
#pragma unroll
  for (int rb = 0; rb < 4; ++rb) {
    const int tok = rb * 16 + l15;
    if (tok < NR) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        f32x4* tp = reinterpret_cast<f32x4*>(T + tok * LT + cbo[j] * 16 + 4 * g);
        *tp = *tp + acc_o[rb][j] * (1.0f / WSC);
      }
    }
  }
  __syncthreads();
  ln_planes8(T, UP, p.ln2_eps, tid);
  __syncthreads();
  WX_STAMP(15);

  // ---- MLP in two hidden chunks of 256: GELU(U2 W1c'^T + b1c') -> WR planes -> MLP2 partial in registers ----
  f32x4 acc_m[4][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const f32x4 b = ld_bias4(p.b2, cbo[j] * 16 + 4 * g);
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) acc_m[rb][j] = b;
  }
#pragma unroll 1
  for (int ck = 0; ck < 2; ++ck) {
    f32x4 ah[4][2];
    const int cb1[2] = {ck * 16 + wid, ck * 16 + wid + 8};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const f32x4 b = ld_bias4(p.b1, cb1[j] * 16 + 4 * g);
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) ah[rb][j] = b;
    }
    gemm_w<C, 2, 4, 2, PSU, UPL, true>(p.w1, HID, C, 0, cb1, UP, 0, ah, lane);
    WX_STAMP(16 + 3 * ck);
    __syncthreads();  // the previous chunk's MLP2 has read WR
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      const int tok = rb * 16 + l15;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const f32x4 a = ah[rb][j] * (1.0f / WSC);
        const f32x2 lo = gelu2_fast_(f32x2{a[0], a[1]});
        const f32x2 hi = gelu2_fast_(f32x2{a[2], a[3]});
        if (tok < NR) store4<PSU, UPL>(Hp, tok, cbo[j] * 16 + 4 * g, f32x4{lo.x, lo.y, hi.x, hi.y});
        rng = range_acc(rng, f32x4{lo.x, lo.y, hi.x, hi.y});
      }
    }
    __syncthreads();
    WX_STAMP(17 + 3 * ck);
    gemm_w<C, 2, 4, 2, PSU, UPL, true>(p.w2, C, HID, ck * 256, cbo, Hp, 0, acc_m, lane);
    WX_STAMP(18 + 3 * ck);
  }
  // final T = T + MLP -> U planes (the pw GEMM's operand); every wave has read U2 (MLP1 of the last chunk)
#pragma unroll
  for (int rb = 0; rb < 4; ++rb) {
    const int tok = rb * 16 + l15;
    if (tok < NR) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(T + tok * LT + cbo[j] * 16 + 4 * g) + acc_m[rb][j] * (1.0f / WSC);
        store4<PSU, UPL>(UP, tok, cbo[j] * 16 + 4 * g, v);
        rng = range_acc(rng, v);
      }
    }
  }
  range_report(p.range_flag, rng);
  prep_report(p.prep_flag, p.range_flag);
  // residual x and BN terms of this lane's outputs: in flight during the pw GEMM
  const __amdgpu_buffer_rsrc_t ry = rsrc_of(p.y + (long)img * C * HWi);
  unsigned vtok[4];  // byte offset of (channel wid*16 + 4g, token tb*16 + l15), or out of range
#pragma unroll
  for (int tb = 0; tb < 4; ++tb) {
    const int tok = tb * 16 + l15;
    const int iy = tok / 7, ix = tok - (tok / 7) * 7;
    const int hh = wy * 7 + iy, wc = wx_ * 7 + ix;
    vtok[tb] = (tok < NR && hh < H && wc < W) ? (unsigned)(((wid * 16 + 4 * g) * HWi + hh * W + wc) * 4) : OOB;
  }
  float xr[2][4][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int tb = 0; tb < 4; ++tb)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        xr[j][tb][r] = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(rx, vtok[tb], (128 * j + r) * HWi * 4, 0));
  f32x4 sc[2], sh[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    sc[j] = *reinterpret_cast<const f32x4*>(p.bn_scale + cbo[j] * 16 + 4 * g) * (1.0f / WSC);
    sh[j] = *reinterpret_cast<const f32x4*>(p.bn_shift + cbo[j] * 16 + 4 * g);
  }
  __syncthreads();
  WX_STAMP(22);
  f32x4 acc[4][2];
#pragma unroll
  for (int tb = 0; tb < 4; ++tb)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[tb][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  gemm_w<C, 2, 4, 2, PSU, UPL, true>(p.wpw, C, C, 0, cbo, UP, 0, acc, lane);
  WX_STAMP(23);
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int tb = 0; tb < 4; ++tb)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        __builtin_amdgcn_raw_buffer_store_b32(
            __builtin_bit_cast(unsigned, xr[j][tb][r] + silu_fast_(acc[tb][j][r] * sc[j][r] + sh[j][r])), ry,
            vtok[tb], (128 * j + r) * HWi * 4, 0);
  WX_STAMP(24);
}
}  // namespace wx


// Weight preparation: LN affine folds and the three-plane split, one wave per output row (lanes along k,
// coalesced); also the BN fold of the pw conv. Rows: [0,3C) in_proj (LN1 folded) | [3C,4C) out_proj | [4C,4C+HID)
// mlp1 (LN2 folded) | mlp2 (K = HID) | pw | C BN entries.
struct PrepArgs {
  const float *win, *bin, *ln1_w, *ln1_b, *wo, *w1, *b1, *ln2_w, *ln2_b, *w2, *wpw;
  const float *bn_w, *bn_b, *bn_m, *bn_v;
  float bn_eps;
  int C, HID;
  h16_t *pin, *po, *p1, *p2, *ppw;
  float *bin_f, *b1_f, *bn_sc, *bn_sh;
  unsigned* range_flag;  // split-range guard: 64 W' must stay finite in fp16
  unsigned* prep_flag;   // the same result kept in the prepared block (zeroed before the launch)
};

__global__ __launch_bounds__(256) void swin_x3_prep_kernel(PrepArgs a) {
  const int C = a.C, HID = a.HID;
  const int lane = threadIdx.x & 63;
  int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  const float* src;
  const float* gam = nullptr;
  const float* bet = nullptr;
  const float* bsrc = nullptr;
  float* bdst = nullptr;
  h16_t* dst;
  int N, K;
  if (n < 3 * C) {
    src = a.win; gam = a.ln1_w; bet = a.ln1_b; bsrc = a.bin; bdst = a.bin_f; dst = a.pin; N = 3 * C; K = C;
  } else if ((n -= 3 * C) < C) {
    src = a.wo; dst = a.po; N = C; K = C;
  } else if ((n -= C) < HID) {
    src = a.w1; gam = a.ln2_w; bet = a.ln2_b; bsrc = a.b1; bdst = a.b1_f; dst = a.p1; N = HID; K = C;
  } else if ((n -= HID) < C) {
    src = a.w2; dst = a.p2; N = C; K = HID;
  } else if ((n -= C) < C) {
    src = a.wpw; dst = a.ppw; N = C; K = C;
  } else if ((n -= C) < C) {
    if (lane == 0) {
      const float inv = 1.0f / sqrtf(a.bn_v[n] + a.bn_eps);
      const float sc = a.bn_w[n] * inv;
      a.bn_sc[n] = sc;
      a.bn_sh[n] = a.bn_b[n] - a.bn_m[n] * sc;
    }
    return;
  } else {
    return;
  }
  const float* row = src + (long)n * K;
  float bacc = 0.f;
  float wmax = 0.f;
  for (int k = lane; k < K; k += 64) {
    const float w = row[k];
    if (bet) bacc = fmaf(w, bet[k], bacc);
    const float v = gam ? w * gam[k] : w;
    const _Float16 h = (_Float16)(v * WSC);
    const _Float16 l = (_Float16)(v * WSC - (float)h);
    wmax = nmax_(wmax, fabsf(v * WSC));
    // fragment-major: element (n, k) at ((n/16 * K/32 + k/32) * 64 + (k%32)/8 * 16 + n%16) * 8 + k%8, so the 64
    // lanes' MFMA fragments of one (column block, 32-k step) are 1 KB contiguous
    const long fi = ((long)((n >> 4) * (K >> 5) + (k >> 5)) * 64 + (((k & 31) >> 3) << 4) + (n & 15)) * 8 + (k & 7);
    dst[fi] = __builtin_bit_cast(h16_t, h);
    dst[(long)N * K + fi] = __builtin_bit_cast(h16_t, l);
  }
  if (bdst) {
    bacc = wave_sum(bacc);
    if (lane == 0) bdst[n] = bsrc[n] + bacc;
  }
  range_report(a.range_flag, wmax);
  range_report(a.prep_flag, wmax);
}

}  // namespace x3
}  // namespace ys

using namespace ys;

// Default for C = 64 (YOLOSOD_SWIN_X3=0 routes C = 64 SwinBlocks to the exact-fp32-MFMA kernel swin_fused.hip).
static int g_swin_x3 = -1;
static bool swin_x3_env() {
  if (g_swin_x3 < 0) {
    const char* e = getenv("YOLOSOD_SWIN_X3");
    g_swin_x3 = (e && e[0] == '0') ? 0 : 1;
  }
  return g_swin_x3 != 0;
}

// Test hook: route C = 64 SwinBlocks through this kernel (1) or swin_fused.hip (0); returns the previous state.
YS_EXPORT int yolosod_debug_set_swin_x3(int on) {
  const int prev = swin_x3_env() ? 1 : 0;
  g_swin_x3 = on ? 1 : 0;
  return prev;
}

bool yolosod_swin_x3_ok(int C, int num_heads, int wh, int ww, int mlp_hidden) {
  return swin_x3_env() && wh == 7 && ww == 7 && mlp_hidden == 2 * C &&
         ((C == 64 && num_heads == 2) || (C == x3::wx::C && num_heads == C / x3::wx::HD));
}

size_t yolosod_swin_x3_workspace(int C, int mlp_hidden) {
  Sizer s;
  s.take<h16_t>((size_t)2 * 3 * C * C);            // in_proj planes
  s.take<h16_t>((size_t)2 * C * C);                // out_proj
  s.take<h16_t>((size_t)2 * mlp_hidden * C);       // mlp1
  s.take<h16_t>((size_t)2 * C * mlp_hidden);       // mlp2
  s.take<h16_t>((size_t)2 * C * C);                // pw
  s.take<float>((size_t)3 * C + mlp_hidden + 2 * C);  // folded biases, BN scale / shift
  s.take<unsigned>(1);                             // the weights' split-range result
  return s.off;
}

// scratch of one run on a prepared block: none (every fp16-split Swin kernel is one launch)
size_t yolosod_swin_x3_run_workspace(int B, int C, int H, int W) { return 0; }

// The prepared-parameter block of the fp16-split kernels (written by swin_x3_prep_kernel): weight planes of in_proj
// (LN1 folded), out_proj, mlp1 (LN2 folded), mlp2, pw; folded in_proj / mlp1 biases; BN scale / shift; the weights'
// split-range word.
struct X3Prep {
  h16_t *pin, *po, *p1, *p2, *ppw;
  float *bin_f, *b1_f, *bn_sc, *bn_sh;
  unsigned* pflag;
};
static bool x3_carve(void* buf, size_t bytes, int C, int mlp_hidden, X3Prep& q) {
  Carver cv(buf, bytes);
  q.pin = cv.take<h16_t>((size_t)2 * 3 * C * C);
  q.po = cv.take<h16_t>((size_t)2 * C * C);
  q.p1 = cv.take<h16_t>((size_t)2 * mlp_hidden * C);
  q.p2 = cv.take<h16_t>((size_t)2 * C * mlp_hidden);
  q.ppw = cv.take<h16_t>((size_t)2 * C * C);
  float* fb = cv.take<float>((size_t)3 * C + mlp_hidden + 2 * C);
  q.pflag = cv.take<unsigned>(1);
  if (!fb || !q.pflag) return false;
  q.bin_f = fb;
  q.b1_f = fb + 3 * C;
  q.bn_sc = fb + 3 * C + mlp_hidden;
  q.bn_sh = fb + 4 * C + mlp_hidden;
  return true;
}

// weight split / folds into a prepared block (C, heads, mlp_hidden must satisfy yolosod_swin_x3_ok)
int yolosod_swin_x3_prepare(int C, int mlp_hidden, const float* ln1_w, const float* ln1_b, const float* in_proj_w,
                            const float* in_proj_b, const float* out_proj_w, const float* ln2_w, const float* ln2_b,
                            const float* mlp1_w, const float* mlp1_b, const float* mlp2_w, const float* pw_w,
                            const float* bn_w, const float* bn_b, const float* bn_mean, const float* bn_var,
                            float bn_eps, void* prep, size_t prep_bytes, hipStream_t st) {
  X3Prep q;
  if (!x3_carve(prep, prep_bytes, C, mlp_hidden, q)) {
    set_error("swin_x3: prepared-parameter buffer too small (%zu)", prep_bytes);
    return -1;
  }
  if (hipMemsetAsync(q.pflag, 0, sizeof(unsigned), st) != hipSuccess) {
    set_error("swin_x3_prep: flag reset failed");
    return -1;
  }
  x3::PrepArgs pa{in_proj_w, in_proj_b, ln1_w, ln1_b, out_proj_w, mlp1_w, mlp1_b, ln2_w, ln2_b, mlp2_w, pw_w,
                  bn_w, bn_b, bn_mean, bn_var, bn_eps, C, mlp_hidden, q.pin, q.po, q.p1, q.p2, q.ppw,
                  q.bin_f, q.b1_f, q.bn_sc, q.bn_sh, range_flag_dev(), q.pflag};
  const int rows = 3 * C + C + mlp_hidden + C + C + C;
  hipLaunchKernelGGL(x3::swin_x3_prep_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, pa);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("swin_x3_prep: launch failed: %s", hipGetErrorString(e));
    return -1;
  }
  return 0;
}

// the kernels on a prepared block; returns 1 if launched, 0 if the shape is not handled, < 0 on error. `ws` is the
// scratch of yolosod_swin_x3_run_workspace (unused by the one-kernel forms)
int yolosod_swin_x3_run(const float* x, float* y, int B, int C, int H, int W, int num_heads, int wh, int ww, int nWx,
                        int nWin, const float* dw_w, float ln1_eps, const float* out_proj_b, float ln2_eps,
                        int mlp_hidden, const float* mlp2_b, const void* prep, size_t prep_bytes, void* ws,
                        size_t ws_bytes, hipStream_t st) {
  if (!yolosod_swin_x3_ok(C, num_heads, wh, ww, mlp_hidden)) return 0;
  if ((long)C * H * W >= (1L << 30) || (long)B * nWin >= (1L << 31)) return 0;
  X3Prep q;
  if (!x3_carve(const_cast<void*>(prep), prep_bytes, C, mlp_hidden, q)) {
    set_error("swin_x3: prepared-parameter buffer too small (%zu)", prep_bytes);
    return -1;
  }
  unsigned* flag = range_flag_dev();
  x3::Args a{x, y, B, H, W, nWx, nWin, dw_w, ln1_eps, ln2_eps, q.pin, q.bin_f, q.po, out_proj_b, q.p1, q.b1_f, q.p2,
             mlp2_b, q.ppw, q.bn_sc, q.bn_sh, 1.0f / sqrtf((float)(C / num_heads)), flag, q.pflag};
  const long nwin = (long)B * nWin;
  if (nwin == 0) return 1;
  if (C == 64) {
    hipLaunchKernelGGL((x3::swin_x3_kernel<64, 2>), dim3((unsigned)(8 * ((nwin + 7) / 8))), dim3(256), 0, st, a);
  } else {
    hipLaunchKernelGGL(x3::wx::swin_wx_kernel, dim3((unsigned)(8 * ((nwin + 7) / 8))), dim3(x3::wx::NT), 0, st, a);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("swin_x3: launch failed: %s", hipGetErrorString(e));
    return -1;
  }
  return 1;
}

// returns 1 if launched, 0 if the shape is not handled, < 0 on error (prep into the workspace, then the kernels on
// the run scratch carved after it)
int yolosod_swin_x3_launch(const float* x, float* y, int B, int C, int H, int W, int num_heads, int wh, int ww,
                           int nWx, int nWin,
                           const float* dw_w, const float* ln1_w, const float* ln1_b, float ln1_eps,
                           const float* in_proj_w, const float* in_proj_b, const float* out_proj_w,
                           const float* out_proj_b, const float* ln2_w, const float* ln2_b, float ln2_eps,
                           const float* mlp1_w, const float* mlp1_b, int mlp_hidden, const float* mlp2_w,
                           const float* mlp2_b, const float* pw_w, const float* bn_w, const float* bn_b,
                           const float* bn_mean, const float* bn_var, float bn_eps, void* workspace,
                           size_t workspace_bytes, hipStream_t st) {
  if (!yolosod_swin_x3_ok(C, num_heads, wh, ww, mlp_hidden)) return 0;
  if ((long)C * H * W >= (1L << 30) || (long)B * nWin >= (1L << 31)) return 0;
  const size_t pb = yolosod_swin_x3_workspace(C, mlp_hidden);
  if (workspace_bytes < pb) {
    set_error("swin_x3: workspace too small (%zu)", workspace_bytes);
    return -1;
  }
  if (yolosod_swin_x3_prepare(C, mlp_hidden, ln1_w, ln1_b, in_proj_w, in_proj_b, out_proj_w, ln2_w, ln2_b, mlp1_w,
                              mlp1_b, mlp2_w, pw_w, bn_w, bn_b, bn_mean, bn_var, bn_eps, workspace, pb, st) < 0)
    return -1;
  return yolosod_swin_x3_run(x, y, B, C, H, W, num_heads, wh, ww, nWx, nWin, dw_w, ln1_eps, out_proj_b, ln2_eps,
                             mlp_hidden, mlp2_b, workspace, pb, (char*)workspace + pb, workspace_bytes - pb, st);
}

// ---- C ABI: the prepared-parameter path (the weight split cached by the caller across calls) -----------------------
YS_EXPORT size_t yolosod_swin_prep_bytes(int C, int num_heads, int mlp_hidden) {
  return yolosod_swin_x3_ok(C, num_heads, 7, 7, mlp_hidden) ? yolosod_swin_x3_workspace(C, mlp_hidden) : 0;
}

YS_EXPORT int yolosod_swin_prepare(int C, int num_heads, int mlp_hidden, const float* ln1_w, const float* ln1_b,
                                   const float* in_proj_w, const float* in_proj_b, const float* out_proj_w,
                                   const float* ln2_w, const float* ln2_b, const float* mlp1_w, const float* mlp1_b,
                                   const float* mlp2_w, const float* pw_w, const float* bn_w, const float* bn_b,
                                   const float* bn_mean, const float* bn_var, float bn_eps, void* prep,
                                   size_t prep_bytes, void* stream) {
  YS_CHECK_ARG(ln1_w && ln1_b && in_proj_w && in_proj_b && out_proj_w && ln2_w && ln2_b && mlp1_w && mlp1_b &&
                   mlp2_w && pw_w && bn_w && bn_b && bn_mean && bn_var && prep,
               "swin_prepare: null pointer");
  YS_CHECK_ARG(yolosod_swin_x3_ok(C, num_heads, 7, 7, mlp_hidden),
               "swin_prepare: C=%d heads=%d hidden=%d has no prepared-parameter kernel", C, num_heads, mlp_hidden);
  return yolosod_swin_x3_prepare(C, mlp_hidden, ln1_w, ln1_b, in_proj_w, in_proj_b, out_proj_w, ln2_w, ln2_b, mlp1_w,
                                 mlp1_b, mlp2_w, pw_w, bn_w, bn_b, bn_mean, bn_var, bn_eps, prep, prep_bytes,
                                 (hipStream_t)stream) < 0
             ? -1
             : 0;
}

#ifdef YS_DIAG_STAMPS
YS_EXPORT int yolosod_diag_x3_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(x3::ys_x3_stamps), sizeof(x3::ys_x3_stamps)) == hipSuccess ? 0 : -1;
}
YS_EXPORT int yolosod_diag_wx_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(x3::wx::ys_wx_stamps), sizeof(x3::wx::ys_wx_stamps)) == hipSuccess ? 0 : -1;
}
#endif
