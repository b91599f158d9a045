// Shared pieces of the fused MNIST kernels (mnist_kernels.hip, mnist_conv_bwd.hip).
#pragma once
#include "common.h"
#include "mnist_engine.h"
#include "mnist_kernels.h"

namespace mx {
namespace mnist {

using L = MnistLayout;
constexpr int kPack = 18432;  // 64*32*9 conv2 weights

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float sel4(const float4& v, int j) {
  return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w;
}
__device__ __forceinline__ int g1_slab_mask(const MnistFused& f) {
  return (f.g1_slabs >= 1 && f.g1_slabs <= 64 ? f.g1_slabs : 16) - 1;
}

// Phase timestamps for in-kernel profiling (MnistFused::trace, off = null): blocks 0..1023 of
// kernel `kid` record the 100 MHz wall clock at phase `ph` (<8) from thread 0.
#define MX_TRACE_B(f, kid, ph, blk)                                                                 \
  do {                                                                                              \
    if ((f).trace && threadIdx.x == 0 && (blk) < 1024)                                              \
      (f).trace[((kid) * 1024 + (blk)) * 8 + (ph)] = (uint32_t)__builtin_amdgcn_s_memrealtime();    \
  } while (0)
#define MX_TRACE(f, kid, ph) MX_TRACE_B(f, kid, ph, (int)blockIdx.x)

struct Scratch {  // carve of MnistFused::scratch (floats)
  float* wf;      // conv2 fwd B-fragments   [18 q][4 w][64 lane][4 j]
  float* wd;      // conv2 dgrad B-fragments [9 r][4 s][2 nt][64 lane][4 j]
  float* wacc;    // conv2 wgrad accumulator slabs [kWaccSlabs][9 r][64 co][32 ci], slab = image & (kWaccSlabs - 1)
  float* wu;      // conv2 dgrad Winograd filters G w' G^T (w' = w flipped) as F7W B-fragments
                  // [16 k-step][2 ci-half][64 lane][16 xi]
  float* g1;      // conv1 grad partial slabs [kG1Slabs][320] (w[32][9] then b[32]), slab = image & (g1_slabs - 1)
  float* wv;      // conv2 forward Winograd filters G w G^T as F2W B-fragments
                  // [4 w][16 xi][2 s4][64 lane][4 j]
};
constexpr int kWinoPack = 16 * 2048;  // 16 Winograd-domain values per (co, ci)
constexpr int kG1Slabs = 64;          // conv1-grad atomic slabs allocated (MnistFused::g1_slabs used)
// conv2-wgrad atomics spread over 2 slabs (image & 1): the 64 images' blocks finish together and
// same-address float atomics serialise, so one accumulator cost F6W a 3.5 us epilogue; the
// finalize (in the SGD launch at world size 1) sums the slabs in a fixed order.  Measured at
// B = 64: 1 slab 837k, 2 slabs 843k, 4 slabs 835k, 8 slabs 821k img/s (the finalize's serial
// tail grows with the slab count faster than the epilogue shrinks: 3.5 / 2.8 / - / 2.4 us).
constexpr int kWaccSlabs = 2;
__host__ __device__ inline Scratch carve(float* s) {
  Scratch c;
  c.wf = s;
  c.wd = c.wf + kPack;
  c.wu = c.wd + kPack;
  c.g1 = c.wu + kWinoPack;
  c.wv = c.g1 + kG1Slabs * 320;
  c.wacc = c.wv + kWinoPack;
  return c;
}
inline size_t scratch_floats(int) {
  return 2 * (size_t)kPack + 2 * (size_t)kWinoPack + (size_t)kG1Slabs * 320 + (size_t)kWaccSlabs * kPack;
}

}  // namespace mnist
}  // namespace mx
