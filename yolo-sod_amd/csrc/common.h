// Shared helpers for the YOLO-SOD gfx950 kernels.
// Every entry point in this library is extern "C", takes plain device pointers + sizes and a hipStream_t
// passed as void*, never synchronises, and reports failures through an int return code plus
// yolosod_last_error() (see include/yolosod_hip.h).
#pragma once
#include <stdlib.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <stdio.h>
#include <stdarg.h>

#define YS_EXPORT extern "C" __attribute__((visibility("default")))

namespace ys {

// ---- error reporting ------------------------------------------------------------------------------
void set_error(const char* fmt, ...);

#define YS_CHECK_ARG(cond, ...)            \
  do {                                     \
    if (!(cond)) {                         \
      ::ys::set_error(__VA_ARGS__);        \
      return -1;                           \
    }                                      \
  } while (0)

#define YS_CHECK_LAUNCH(what)                                                        \
  do {                                                                               \
    hipError_t e_ = hipGetLastError();                                               \
    if (e_ != hipSuccess) {                                                          \
      ::ys::set_error("%s: launch failed: %s", what, hipGetErrorString(e_));         \
      return (int)e_;                                                                \
    }                                                                                \
  } while (0)

// ---- workspace carving (16-byte aligned bump allocator over a caller-owned buffer) ----------------
struct Carver {
  char* base;
  size_t cap;
  size_t off;
  __host__ Carver(void* b, size_t c) : base((char*)b), cap(c), off(0) {}
  template <class T>
  __host__ T* take(size_t n) {
    size_t bytes = (n * sizeof(T) + 255) & ~(size_t)255;
    if (off + bytes > cap) return nullptr;
    T* p = (T*)(base + off);
    off += bytes;
    return p;
  }
};
// Same arithmetic as Carver, used to size workspaces.
struct Sizer {
  size_t off = 0;
  template <class T>
  void take(size_t n) { off += (n * sizeof(T) + 255) & ~(size_t)255; }
};

// ---- math -----------------------------------------------------------------------------------------
__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }
__device__ __forceinline__ float siluf_(float x) { return x / (1.0f + expf(-x)); }
__device__ __forceinline__ float geluf_(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f)); }

// erf with max |error| 1.5e-7 (Abramowitz & Stegun 7.1.26) on the hardware exp2 / rcp: ~12 VALU instead of erff's 36.
// Used where the GELU sits inside an MFMA-bound fused kernel; its error is at fp32 rounding level of the output.
__device__ __forceinline__ float erf_as_(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(1.0f + 0.3275911f * ax);  // v_rcp_f32 (1 ulp): one instruction
  const float poly =
      t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  const float r = 1.0f - poly * __expf(-ax * ax);
  return copysignf(r, x);
}
__device__ __forceinline__ float gelu_fast_(float x) { return 0.5f * x * (1.0f + erf_as_(x * 0.70710678118654752440f)); }

// The same GELU on a pair of values in packed fp32 (v_pk_fma_f32 / v_pk_mul_f32 do two lanes' worth per
// instruction; rcp / exp stay scalar): ~10 VALU per value instead of ~17, for the MLP1 epilogues.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu2_fast_(f32x2 x) {
  const f32x2 xs = x * 0.70710678118654752440f;
  const f32x2 ax = {fabsf(xs.x), fabsf(xs.y)};
  const f32x2 den = __builtin_elementwise_fma(ax, f32x2{0.3275911f, 0.3275911f}, f32x2{1.0f, 1.0f});
  const f32x2 t = {__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
  f32x2 poly = __builtin_elementwise_fma(t, f32x2{1.061405429f, 1.061405429f}, f32x2{-1.453152027f, -1.453152027f});
  poly = __builtin_elementwise_fma(t, poly, f32x2{1.421413741f, 1.421413741f});
  poly = __builtin_elementwise_fma(t, poly, f32x2{-0.284496736f, -0.284496736f});
  poly = __builtin_elementwise_fma(t, poly, f32x2{0.254829592f, 0.254829592f});
  poly = poly * t;
  const f32x2 m = ax * (ax * -1.44269504088896341f);  // -x^2 log2(e)
  const f32x2 e = {__builtin_amdgcn_exp2f(m.x), __builtin_amdgcn_exp2f(m.y)};
  const f32x2 r = __builtin_elementwise_fma(-poly, e, f32x2{1.0f, 1.0f});
  const f32x2 erf = {copysignf(r.x, xs.x), copysignf(r.y, xs.y)};
  const f32x2 hx = x * 0.5f;
  return __builtin_elementwise_fma(hx, erf, hx);
}
// x / (1 + e^-x) as x * rcp(1 + e^-x): v_rcp_f32 (1 ulp) instead of the 10-instruction IEEE division sequence
// (__fdividef is a full-precision divide on this target)
__device__ __forceinline__ float silu_fast_(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ __forceinline__ float sigmoid_fast_(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }

// wave64 reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// cross-lane reductions without LDS round trips (gfx950): DPP quad permutes, v_permlane16/32_swap
__device__ __forceinline__ float quad_sum(float v) {  // sum over lanes {4k..4k+3}
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));  // quad_perm [1,0,3,2]
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, true));  // quad_perm [2,3,0,1]
  return v;
}
__device__ __forceinline__ float xor16_sum(float v) {  // v(l) + v(l ^ 16)
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xor32_sum(float v) {  // v(l) + v(l ^ 32)
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xor16_max(float v) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor32_max(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// fp32 MFMA fragment types
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

// ---- bf16 storage (the bf16 model config: activations in HBM as bf16, arithmetic in fp32) ------------------
// bf16 values cross the C ABI as their 16-bit patterns (uint16_t, torch.bfloat16's layout). Widening is exact
// (a shift); narrowing rounds to nearest even (v_cvt_pk_bf16_f32), as torch's .to(torch.bfloat16).
typedef uint16_t bf16_t;
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float((uint32_t)v << 16); }
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  const bf16x2_t v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ bf16_t f2bf(float a) { return (bf16_t)(pack_bf16x2(a, 0.f) & 0xffffu); }

// element loads / stores of either storage type, values in fp32 registers
__device__ __forceinline__ float ld1(const float* p) { return *p; }
__device__ __forceinline__ float ld1(const bf16_t* p) { return bf2f(*p); }
__device__ __forceinline__ void st1(float* p, float v) { *p = v; }
__device__ __forceinline__ void st1(bf16_t* p, float v) { *p = f2bf(v); }
// 4 consecutive elements (16 B for fp32, 8 B for bf16; 4-element aligned)
__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ f32x4 ld4(const bf16_t* p) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  return f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
               __uint_as_float(u.y & 0xffff0000u)};
}
// the values a bf16 store of v would hold, back in fp32
__device__ __forceinline__ f32x4 round_bf16(f32x4 v) {
  const uint32_t a = pack_bf16x2(v.x, v.y), b = pack_bf16x2(v.z, v.w);
  return f32x4{__uint_as_float(a << 16), __uint_as_float(a & 0xffff0000u), __uint_as_float(b << 16),
               __uint_as_float(b & 0xffff0000u)};
}
// 8 bf16 (one uint4) <-> fp32
__device__ __forceinline__ void unpack8(uint4 u, float* f) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  return make_uint4(pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3]), pack_bf16x2(f[4], f[5]), pack_bf16x2(f[6], f[7]));
}
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
__device__ __forceinline__ void st4(bf16_t* p, f32x4 v) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pack_bf16x2(v.x, v.y), pack_bf16x2(v.z, v.w));
}

// ---- fp32-accurate products on the fp16 matrix cores ------------------------------------------------------
// v = h + l with h = fp16(v), l = fp16(v - h) (round to nearest even; v - h is exact in fp32): |v - h - l| <= 2^-22 |v|
// while l is a normal fp16 number. a.b ~ ah.bh + ah.bl + al.bh (three exact fp16 products, fp32 accumulation; the
// dropped al.bl <= 2^-22 |a.b|). Used by the fp32 Swin kernels (swin_x3.hip) and the Detect head (detect.hip).
typedef uint16_t h16_t;  // fp16 bit pattern
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
// a pair: v_cvt_pk_f16_f32, two v_cvt_f32_f16, v_pk_add_f32, v_cvt_pk_f16_f32. (A 3-instruction form with the low
// terms from v_fma_mix{lo,hi}_f16 in inline asm was tried: the compiler does not model the hazards of an asm
// statement, and with MFMA results as its inputs the C = 64 Swin kernel computed nondeterministic garbage under some
// schedules; the VALU it saved was worth ~1 % of that kernel's time.)
__device__ __forceinline__ void split2(f32x2 v, uint32_t& h, uint32_t& l) {
  const f16x2_t hh = __builtin_convertvector(v, f16x2_t);
  const f32x2 r = v - __builtin_convertvector(hh, f32x2);
  h = __builtin_bit_cast(uint32_t, hh);
  l = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, f16x2_t));
}
__device__ __forceinline__ void split4(f32x4 v, uint2& h, uint2& l) {
  split2(f32x2{v.x, v.y}, h.x, l.x);
  split2(f32x2{v.z, v.w}, h.y, l.y);
}
// The same split for values loaded from memory (no producing arithmetic the compiler could contract into the
// subtraction): the low terms as v_fma_mixlo_f16 / v_fma_mixhi_f16 (fma(h, -1, v) of the fp16 half h and the fp32 v,
// rounded once to fp16), three VALU per pair instead of five, bit-identical to split2 for such values (v - h is exact
// in fp32). The compiler forms the mixed fma only from a non-constant multiplier (a constant -1 is canonicalised to a
// subtraction first), so -1 goes through an SGPR behind an empty asm statement, and a second empty statement keeps
// the SLP vectoriser from fusing the pair's two fmas into one v_pk_fma_f32 (neither statement emits an instruction).
// Not used on computed operands: there split2's `v - h` may absorb the producer's last multiply (fp-contract) and
// keep its rounding error in the low term, which the mixed form would drop.
__device__ __forceinline__ void split2x(f32x2 v, uint32_t& h, uint32_t& l) {
  const f16x2_t hh = __builtin_convertvector(v, f16x2_t);
  h = __builtin_bit_cast(uint32_t, hh);
  float m1 = -1.0f;
  asm("" : "+s"(m1));
  _Float16 l0 = (_Float16)__builtin_fmaf((float)hh.x, m1, v.x);
  asm("" : "+v"(l0));
  const _Float16 l1 = (_Float16)__builtin_fmaf((float)hh.y, m1, v.y);
  l = __builtin_bit_cast(uint32_t, f16x2_t{l0, l1});
}
__device__ __forceinline__ void split4x(f32x4 v, uint2& h, uint2& l) {
  split2x(f32x2{v.x, v.y}, h.x, l.x);
  split2x(f32x2{v.z, v.w}, h.y, l.y);
}
__device__ __forceinline__ void split8x(f32x4 a, f32x4 b, f16x8_t& h, f16x8_t& l) {
  uint2 h0, l0, h1, l1;
  split4x(a, h0, l0);
  split4x(b, h1, l1);
  h = __builtin_bit_cast(f16x8_t, make_uint4(h0.x, h0.y, h1.x, h1.y));
  l = __builtin_bit_cast(f16x8_t, make_uint4(l0.x, l0.y, l1.x, l1.y));
}
// 8 values -> the hi / lo fp16 operands of one v_mfma_f32_16x16x32_f16 k slot group
__device__ __forceinline__ void split8(f32x4 a, f32x4 b, f16x8_t& h, f16x8_t& l) {
  uint2 h0, l0, h1, l1;
  split4(a, h0, l0);
  split4(b, h1, l1);
  h = __builtin_bit_cast(f16x8_t, make_uint4(h0.x, h0.y, h1.x, h1.y));
  l = __builtin_bit_cast(f16x8_t, make_uint4(l0.x, l0.y, l1.x, l1.y));
}
// Split-range guard (fp16 holds |h| < 65520; beyond it h = inf and the products turn into inf / NaN): every split site
// folds the magnitudes it splits into a per-thread running max (max3 with |.| modifiers, ~one VALU per pair) and the
// kernel reports once at its end into a per-device flag word (range_flag_dev(); yolosod_split_range_flag reads it).
// The flag makes a launch whose operands left the method's range visible, so the caller can redo it on the exact
// fp32 kernels (DetectionPredictor does) instead of returning silent inf / NaN.
// The running max is the IEEE 754-2019 maximum (v_maximum3_f32 on gfx950), which propagates a NaN operand: fmaxf
// (maxNum) would return the non-NaN operand and lose it, so a NaN produced upstream (e.g. a Swin block fed to the Detect
// head) would go unflagged. Same instruction count as the fmaxf form.
__device__ __forceinline__ float nmax_(float a, float b) { return __builtin_elementwise_maximum(a, b); }
__device__ __forceinline__ float range_acc(float m, f32x4 v) {
  return nmax_(nmax_(m, nmax_(fabsf(v.x), fabsf(v.y))), nmax_(fabsf(v.z), fabsf(v.w)));
}
__device__ __forceinline__ float range_acc2(float m, f32x2 v) { return nmax_(m, nmax_(fabsf(v.x), fabsf(v.y))); }
constexpr float SPLIT_RANGE = 65504.0f;  // largest finite fp16
__device__ __forceinline__ void range_report(unsigned* flag, float m) {
  if (flag && !(m <= SPLIT_RANGE)) *flag = 1u;  // NaN inputs report too
}
// host: the device's flag word (allocated and zeroed on first use, one per device)
unsigned* range_flag_dev();

// c += A.B for split operands (A = (ah, al), B = (bh, bl)), smallest terms first
__device__ __forceinline__ f32x4 mfma_f16x3(f16x8_t ah, f16x8_t al, f16x8_t bh, f16x8_t bl, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, c, 0, 0, 0);
}

// Streaming passes that re-read a tensor written just before (> 256 MiB MALL) walk it back to front, so the tail the
// producer wrote last is still in the Infinity Cache when the pass starts (SE L1 0.195 -> 0.18 ms same-box). Results
// are identical either way (each workgroup's work and summation order is unchanged).
static inline int mall_reverse() { return 1; }

}  // namespace ys
