// Shared helpers for the YOLO-SOD gfx950 kernels.
// Every entry point in this library is extern "C", takes plain device pointers + sizes and a hipStream_t
// passed as void*, never synchronises, and reports failures through an int return code plus
// yolosod_last_error() (see include/yolosod_hip.h).
#pragma once
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

// fp32 MFMA fragment types
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

}  // namespace ys
