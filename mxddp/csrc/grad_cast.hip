// fp32 <-> bf16 casts of gradient buckets for the opt-in bf16 gradient all-reduce
// (Reducer::set_comm_dtype; the DDP bucket all-reduce of pytorch/distributed_data_parallel.py:74
// at half the bytes over xGMI, SURVEY §2.8: ResNet-50's 102 MB fp32 gradient -> 51 MB).
// Round to nearest even; 8 elements (one 16-byte bf16 vector, two 16-byte fp32 vectors) per
// thread and iteration, scalar tail.
#include "common.h"
#include "ops.h"

namespace mx {
namespace {

__device__ __forceinline__ uint32_t rne_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u) return (u >> 16) | ((u & 0xffffu) ? 0x40u : 0u);  // inf / NaN stay
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}

__global__ __launch_bounds__(256) void f32_to_bf16_k(const float* __restrict__ x, uint16_t* __restrict__ y, int64_t n) {
  const int64_t n8 = n >> 3, stride = (int64_t)gridDim.x * 256;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n8; i += stride) {
    const float4 a = reinterpret_cast<const float4*>(x)[2 * i], b = reinterpret_cast<const float4*>(x)[2 * i + 1];
    uint4 o;
    o.x = rne_bf16(a.x) | (rne_bf16(a.y) << 16);
    o.y = rne_bf16(a.z) | (rne_bf16(a.w) << 16);
    o.z = rne_bf16(b.x) | (rne_bf16(b.y) << 16);
    o.w = rne_bf16(b.z) | (rne_bf16(b.w) << 16);
    reinterpret_cast<uint4*>(y)[i] = o;
  }
  for (int64_t i = (n8 << 3) + blockIdx.x * 256 + threadIdx.x; i < n; i += stride) y[i] = (uint16_t)rne_bf16(x[i]);
}

__global__ __launch_bounds__(256) void bf16_to_f32_k(const uint16_t* __restrict__ x, float* __restrict__ y, int64_t n) {
  const int64_t n8 = n >> 3, stride = (int64_t)gridDim.x * 256;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n8; i += stride) {
    const uint4 v = reinterpret_cast<const uint4*>(x)[i];
    reinterpret_cast<float4*>(y)[2 * i] = make_float4(__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u),
                                                      __uint_as_float(v.y << 16), __uint_as_float(v.y & 0xffff0000u));
    reinterpret_cast<float4*>(y)[2 * i + 1] = make_float4(__uint_as_float(v.z << 16), __uint_as_float(v.z & 0xffff0000u),
                                                          __uint_as_float(v.w << 16), __uint_as_float(v.w & 0xffff0000u));
  }
  for (int64_t i = (n8 << 3) + blockIdx.x * 256 + threadIdx.x; i < n; i += stride) y[i] = __uint_as_float((uint32_t)x[i] << 16);
}

int cast_grid(int64_t n) {
  const int64_t g = (n / 8 + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 2048 ? 2048 : g));
}

}  // namespace

void cast_f32_bf16(const float* x, uint16_t* y, int64_t n, hipStream_t st) {
  MX_CHECK((uintptr_t)x % 16 == 0 && (uintptr_t)y % 16 == 0, "cast_f32_bf16: 16-byte aligned buffers");
  MX_LAUNCH(f32_to_bf16_k, dim3(cast_grid(n)), dim3(256), 0, st, x, y, n);
}

void cast_bf16_f32(const uint16_t* x, float* y, int64_t n, hipStream_t st) {
  MX_CHECK((uintptr_t)x % 16 == 0 && (uintptr_t)y % 16 == 0, "cast_bf16_f32: 16-byte aligned buffers");
  MX_LAUNCH(bf16_to_f32_k, dim3(cast_grid(n)), dim3(256), 0, st, x, y, n);
}

}  // namespace mx
