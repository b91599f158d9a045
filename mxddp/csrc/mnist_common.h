// Shared pieces of the fused MNIST kernels (mnist_kernels.hip, mnist_conv_bwd.hip).
#pragma once
#include "common.h"
#include "mnist_engine.h"
#include "mnist_kernels.h"

namespace mx {
namespace mnist {

using L = MnistLayout;
constexpr int kPack = 18432;  // 64*32*9 conv2 weights

// PyTorch SGD (momentum, weight decay; DDP's 1 / world size in gscale) with every rounding
// spelled out: the fused fc1 update in F5 and the flat SGD kernel produce bit-identical results
// whichever path a step takes (left to the compiler, the contraction of g * gscale + wd * p into an
// fma differed between the two, one ulp apart).
__device__ __forceinline__ void sgd_upd(float& p, float& buf, float g, float gscale, float mom, float wd, float lr) {
  const float gg = __fmaf_rn(wd, p, __fmul_rn(g, gscale));
  buf = __fmaf_rn(mom, buf, gg);
  p = __fmaf_rn(-lr, buf, p);
}

// 16-byte vector store with agent scope (sc1): the line is not kept dirty in this XCD's L2, the
// bytes go to memory while the kernel runs (MnistFused::wt)
__device__ __forceinline__ void st4_wt(float4* p, float4 v) {
  const f32x4 q = {v.x, v.y, v.z, v.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(q) : "memory");
}
__device__ __forceinline__ void st4(float4* p, float4 v, bool wt) {
  if (wt)
    st4_wt(p, v);
  else
    *p = v;
}
__device__ __forceinline__ void st1(float* p, float v, bool wt) {
  if (wt)
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    *p = v;
}

// ReLU that keeps NaN (fmaxf(NaN, 0) is 0: a diverged value would vanish into a finite 0)
__device__ __forceinline__ float relu_nan(float x) { return x <= 0.f ? 0.f : x; }

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float sel4(const float4& v, int j) {
  return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w;
}

// Deterministic cross-block sums: partial results are added as 64-bit fixed-point integers
// (two's complement, wrapping adds are exact and associative), so the total does not depend on
// the order in which blocks arrive.  kHScale for the fc1 pre-activation (|h| << 2^31),
// kGScale for gradients (|g| << 2^23; 2^-40 absolute resolution).
constexpr float kHScale = 4294967296.f, kHInv = 1.f / 4294967296.f;                   // 2^32
constexpr float kGScale = 1099511627776.f, kGInv = 1.f / 1099511627776.f;             // 2^40
__device__ __forceinline__ unsigned long long to_fix(float v, float scale) {
  // saturate instead of wrapping if a diverged run overflows the range
  const float s = fminf(fmaxf(v * scale, -9.2e18f), 9.2e18f);
  return (unsigned long long)__float2ll_rn(s);
}
__device__ __forceinline__ float from_fix(long long v, float inv) { return (float)v * inv; }
// A non-finite partial (a diverged step) cannot be represented in the integer sum -- to_fix would
// turn NaN into a saturated finite value -- so it raises the sticky `bad` word instead, and every
// conversion back (from_fix_chk) then yields NaN: divergence stays visible in the loss and weights.
__device__ __forceinline__ void fix_add(long long* dst, float v, float scale, int* bad) {
  if (!__builtin_isfinite(v)) atomicOr(bad, 1);
  atomicAdd(reinterpret_cast<unsigned long long*>(dst), to_fix(v, scale));
}
__device__ __forceinline__ float from_fix_chk(long long v, float inv, int bad) {
  return bad ? __builtin_nanf("") : (float)v * inv;
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
  float* wu;      // conv2 dgrad Winograd filters G w' G^T (w' = w flipped) as F7W B-fragments
                  // [16 k-step][2 ci-half][64 lane][16 xi]
  long long* g1;  // conv1 grad slabs, int64 fixed point (kGScale) [kG1Slabs][320] (w[32][9] then
                  // b[32]), slab = image & (kG1Slabs - 1)
  long long* db2; // conv2 bias grad, int64 fixed point (kGScale) [64] (F5 blocks add, finalize reads)
  float* wv;      // conv2 forward Winograd filters G w G^T as F2W B-fragments
                  // [4 w][16 xi][2 s4][64 lane][4 j]
  float* wslab;   // conv2 wgrad per-image slabs [B][64 co][32 ci][9 tap] (canonical order), written
                  // by F6W, summed by the finalize in a fixed order
  int* bad;       // sticky: a non-finite value reached a fixed-point sum (fix_add); zeroed by k_init
};
constexpr int kWinoPack = 16 * 2048;  // 16 Winograd-domain values per (co, ci)
// conv1-grad slabs: the F7W blocks of image b add into slab b & 15 (integer adds, so the slab
// count only spreads same-address contention; the sum is exact either way)
constexpr int kG1Slabs = 16;
__host__ __device__ inline Scratch carve(float* s, int B) {
  Scratch c;
  c.wu = s;
  c.g1 = reinterpret_cast<long long*>(c.wu + kWinoPack);
  c.db2 = c.g1 + kG1Slabs * 320;
  c.wv = reinterpret_cast<float*>(c.db2 + 64);
  c.wslab = c.wv + kWinoPack;
  c.bad = reinterpret_cast<int*>(c.wslab + (size_t)B * kPack);  // after the slabs
  return c;
}
inline size_t scratch_floats(int B) {
  return 2 * (size_t)kWinoPack + 2 * ((size_t)kG1Slabs * 320 + 64) + (size_t)B * kPack + 64;
}


// conv2 weight gradient of pairs 4 grp .. 4 grp + 3 (36 consecutive floats of the canonical
// [co][ci][ky][kx] layout) summed over the B per-image slabs in a fixed order -> gs[36] (LDS).
// Threads t < 144: float4 q = t % 9 of the group, image subgroup sg = t / 9 sums images sg,
// sg + 16, ... (4 loads in flight per round, clamped + masked: no load behind a branch); the 16
// subgroup partials are added in order.  red: 576 floats of LDS.
constexpr int kWslabGroups = 512;  // 2048 pairs / 4
// fc1 weight-gradient column slices (F5's blocks, and the deferred update's blocks in F67)
constexpr int kFc1Cols = 48, kFc1Slices = 9216 / kFc1Cols;
__device__ __forceinline__ void wslab_group_sum(const MnistFused& f, const Scratch& sc, int grp, float* red, float* gs) {
  const int t = threadIdx.x;
  if (t < 144) {
    const int ns = f.B, q = t % 9, sg = t / 9, nb = ns / 16;
    const float4* src = reinterpret_cast<const float4*>(sc.wslab) + grp * 9 + q;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int i0 = 0; i0 < nb; i0 += 4) {
      float4 v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = src[(size_t)min(sg + 16 * (i0 + i), ns - 1) * (kPack / 4)];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool in = i0 + i < nb;
        a.x += in ? v[i].x : 0.f;
        a.y += in ? v[i].y : 0.f;
        a.z += in ? v[i].z : 0.f;
        a.w += in ? v[i].w : 0.f;
      }
    }
    reinterpret_cast<float4*>(red)[sg * 9 + q] = a;
  }
  __syncthreads();
  if (t < 36) {
    float s = red[t];
#pragma unroll
    for (int sg = 1; sg < 16; ++sg) s += red[sg * 36 + t];
    gs[t] = s;
  }
  __syncthreads();
}

}  // namespace mnist
}  // namespace mx
