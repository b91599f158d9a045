// mxddp common device/host helpers (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

#define MX_HIP_CHECK(expr)                                                                     \
  do {                                                                                          \
    hipError_t mx_err_ = (expr);                                                                \
    if (mx_err_ != hipSuccess)                                                                  \
      throw std::runtime_error(std::string("HIP error '") + hipGetErrorString(mx_err_) +       \
                               "' at " __FILE__ ":" + std::to_string(__LINE__) + ": " #expr);  \
  } while (0)

#define MX_CHECK(cond, msg)                                                                    \
  do {                                                                                          \
    if (!(cond)) throw std::runtime_error(std::string("mxddp check failed: ") + (msg));        \
  } while (0)

namespace mx {

// Launch-error check after every kernel launch; with debug sync on (MXDDP_DEBUG_SYNC=1 or
// set_debug_sync(true)) the stream is also synchronised after each launch outside graph
// capture, so an asynchronous fault is reported at the kernel that caused it.
void post_launch(hipStream_t st, const char* what);
void set_debug_sync(bool on);
bool debug_sync();
// compute units of the current device (cached per device)
int device_cu_count();

#define MX_LAUNCH(kern, grid, block, shm, st, ...)                \
  do {                                                            \
    hipLaunchKernelGGL(kern, grid, block, shm, st, __VA_ARGS__);  \
    ::mx::post_launch(st, #kern);                                 \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kWave = 64;  // CDNA wavefront width
constexpr int kNumXcd = 8;  // MI355X: 8 XCDs x 32 CUs

// Unsigned division by a runtime-invariant divisor via multiply-high (Granlund-Montgomery).
// Valid for 0 <= n < 2^31 and 1 <= d < 2^31.
struct FastDiv {
  uint32_t d = 1, m = 0, s = 0;
  FastDiv() = default;
  explicit FastDiv(uint32_t div) : d(div) {
    uint32_t l = 0;
    while ((1ull << l) < div) ++l;
    s = l;
    m = static_cast<uint32_t>(((1ull << 32) * ((1ull << l) - div)) / div + 1);
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const {
    return (__umulhi(n, m) + n) >> s;
  }
};

// Bijective XCD-aware block remap: consecutive logical tiles land on the same XCD
// (same L2). Dispatch places workgroup i on XCD i % 8 (speed only, never correctness).
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  if (nwg < 2 * kNumXcd) return orig;
  const int q = nwg / kNumXcd, r = nwg % kNumXcd, xcd = orig % kNumXcd;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / kNumXcd;
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, NOT for its
// outstanding global stores.  A __syncthreads() (workgroup release fence + s_barrier) emits
// s_waitcnt vmcnt(0) whenever global stores precede it, so a block that publishes data and then
// synchronises on LDS waits for the stores' write acknowledgements (measured in F2: the slowest
// blocks spent ~7 us there).  Use only where no other wave reads the stored global data.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
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

inline int cdiv(int a, int b) { return (a + b - 1) / b; }

}  // namespace mx
