// Library-wide runtime pieces of the C ABI: error reporting and version query.
#include "common.h"
#include <string.h>
#include <mutex>

namespace ys {
static thread_local char g_err[1024] = {0};
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace ys

YS_EXPORT const char* yolosod_last_error(void) { return ys::g_err; }

namespace ys {
// the split-range flag word of each device (common.h range_report). yolosod_init(device) allocates and zeroes it
// eagerly (the Python binding calls it once per device before the first launch, so no allocation or synchronous
// memset happens inside a stream capture); a launch on a device that was never initialised allocates it here. The
// table is guarded by a mutex, so concurrent first use from two threads allocates once.
static std::mutex g_flag_mu;
static unsigned* g_flags[64] = {nullptr};
static unsigned* flag_alloc(int dev) {
  std::lock_guard<std::mutex> lk(g_flag_mu);
  unsigned* cur = __atomic_load_n(&g_flags[dev], __ATOMIC_RELAXED);  // writers hold the lock
  if (!cur) {
    unsigned* p = nullptr;
    if (hipMalloc(&p, sizeof(unsigned)) != hipSuccess) return nullptr;
    if (hipMemset(p, 0, sizeof(unsigned)) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
      (void)hipFree(p);
      return nullptr;
    }
    __atomic_store_n(&g_flags[dev], p, __ATOMIC_RELEASE);  // pairs with the lock-free acquire load below
    cur = p;
  }
  return cur;
}
unsigned* range_flag_dev() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  unsigned* p = __atomic_load_n(&g_flags[dev], __ATOMIC_ACQUIRE);
  return p ? p : flag_alloc(dev);
}
}  // namespace ys

// Per-device initialisation of the library's device state (the split-range flag word); idempotent. Returns 0, or < 0
// if the device cannot be selected or the allocation fails. The current device is restored.
YS_EXPORT int yolosod_init(int device) {
  int prev = 0;
  YS_CHECK_ARG(device >= 0 && device < 64, "yolosod_init: device %d out of range", device);
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess) {
    ys::set_error("yolosod_init: cannot select device %d", device);
    return -1;
  }
  unsigned* p = ys::flag_alloc(device);
  (void)hipSetDevice(prev);
  YS_CHECK_ARG(p, "yolosod_init: flag allocation failed on device %d", device);
  return 0;
}

// 1 if a split kernel on the current device has seen an operand outside the fp16 range (|v| > 65504 or NaN) since
// the last reset, else 0; < 0 on error. Waits for the work queued on `stream` (the flag's producers) first.
YS_EXPORT int yolosod_split_range_flag(int reset, void* stream) {
  unsigned* f = ys::range_flag_dev();
  YS_CHECK_ARG(f, "split_range_flag: no flag word on this device");
  unsigned v = 0;
  if (hipMemcpyAsync(&v, f, sizeof(unsigned), hipMemcpyDeviceToHost, (hipStream_t)stream) != hipSuccess ||
      hipStreamSynchronize((hipStream_t)stream) != hipSuccess) {
    ys::set_error("split_range_flag: copy failed");
    return -1;
  }
  if (reset && v && hipMemsetAsync(f, 0, sizeof(unsigned), (hipStream_t)stream) != hipSuccess) {
    ys::set_error("split_range_flag: reset failed");
    return -1;
  }
  return v ? 1 : 0;
}
YS_EXPORT int yolosod_abi_version(void) { return 1; }

// Test hook for the fp16 two-term split every fp32-accurate matrix kernel uses (common.h split2): h[i] / l[i] are the
// fp16 pairs of v[2i], v[2i+1]. Lets the tests check the split bit for bit against fp16(v), fp16(v - fp16(v)).
namespace ys {
__global__ void debug_split_kernel(const float* __restrict__ v, uint32_t* __restrict__ h, uint32_t* __restrict__ l,
                                   long npair) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npair) return;
  uint32_t hh, ll;
  split2(f32x2{v[2 * i], v[2 * i + 1]}, hh, ll);
  h[i] = hh;
  l[i] = ll;
}
}  // namespace ys

YS_EXPORT int yolosod_debug_split_f16(const float* v, uint32_t* h, uint32_t* l, long npair, void* stream) {
  YS_CHECK_ARG(v && h && l && npair >= 0, "yolosod_debug_split_f16: bad arguments");
  if (npair == 0) return 0;
  ys::debug_split_kernel<<<(unsigned)((npair + 255) / 256), 256, 0, (hipStream_t)stream>>>(v, h, l, npair);
  YS_CHECK_LAUNCH("yolosod_debug_split_f16");
  return 0;
}
