// Counter-based Philox4x32-10 (Salmon et al., SC'11) shared by the data kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace mx {

__device__ __forceinline__ uint4 philox4x32(uint4 c, uint2 k) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

__device__ __forceinline__ float u01(uint32_t v) { return (v >> 8) * (1.0f / 16777216.0f); }

// Class-conditional synthetic sample (the recipe of ops_data.hip synth_batch): label and the
// 4 pixels [d, d+4) of image b for batch counter `ctr`.
__device__ __forceinline__ uint2 synth_key(uint64_t seed) {
  return make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
}
__device__ __forceinline__ int synth_label(uint32_t ctr, int b, int C, uint2 key) {
  return (int)(philox4x32(make_uint4(ctr, (uint32_t)b, 0xFFFFFFFFu, 0), key).x % (uint32_t)C);
}
__device__ __forceinline__ uint4 synth_noise4(uint32_t ctr, int b, int d, uint2 key) {
  return philox4x32(make_uint4(ctr, (uint32_t)b, (uint32_t)d, 1), key);
}

}  // namespace mx
