// Host-side runtime helpers shared by every op: launch checking and the debug-sync mode.
#include <atomic>
#include <cstdlib>

#include "common.h"

namespace mx {

namespace {
std::atomic<int> g_debug_sync{-1};  // -1: not yet read from the environment
}

bool debug_sync() {
  int v = g_debug_sync.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = std::getenv("MXDDP_DEBUG_SYNC");
    v = (e && *e && *e != '0') ? 1 : 0;
    g_debug_sync.store(v, std::memory_order_relaxed);
  }
  return v == 1;
}

void set_debug_sync(bool on) { g_debug_sync.store(on ? 1 : 0, std::memory_order_relaxed); }

int device_cu_count() {
  static std::atomic<int> cache[64];
  int dev = 0;
  MX_HIP_CHECK(hipGetDevice(&dev));
  int v = dev < 64 ? cache[dev].load(std::memory_order_relaxed) : 0;
  if (v <= 0) {
    MX_HIP_CHECK(hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev));
    if (dev < 64) cache[dev].store(v, std::memory_order_relaxed);
  }
  return v;
}

void post_launch(hipStream_t st, const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    throw std::runtime_error(std::string("HIP launch of ") + what + " failed: " + hipGetErrorString(e));
  if (!debug_sync()) return;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  MX_HIP_CHECK(hipStreamIsCapturing(st, &cs));
  if (cs != hipStreamCaptureStatusNone) return;
  e = hipStreamSynchronize(st);
  if (e != hipSuccess)
    throw std::runtime_error(std::string("HIP kernel ") + what + " faulted: " + hipGetErrorString(e));
}

}  // namespace mx
