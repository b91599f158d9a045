// On-device data generation / augmentation / metrics.
// Replaces the reference's CPU DataLoader workers + torchvision transforms
// (pytorch/single_gpu.py:51-61, pytorch/distributed_data_parallel.py:79-91) and the
// host-synchronising metric path (pytorch/distributed_data_parallel.py:135-140):
// batches are produced in HBM by a counter-based Philox generator and accuracy is
// counted on device, so the training step never waits on the host.
#include "common.h"
#include "ops.h"
#include "rng.h"

namespace mx {
namespace {

__global__ void synth_templates_k(float* t, int C, int D, uint64_t seed) {
  const int64_t total = (int64_t)C * D;
  const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32) ^ 0x7A3Bu);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const uint4 r = philox4x32(make_uint4((uint32_t)i, 0xC1A55u, 0, 0), key);
    t[i] = u01(r.x);
  }
}

__global__ void synth_batch_k(float* __restrict__ x, int32_t* __restrict__ y, const float* __restrict__ tmpl, int B,
                              int D, int C, uint64_t seed, int32_t* counter) {
  const uint32_t ctr = (uint32_t)*counter;
  const uint2 key = synth_key(seed);
  // blockIdx.y splits an image over several blocks (a 224x224x3 image per block left the
  // ImageNet-shape batch on one block per CU); values depend only on (counter, b, d), so the
  // mapping does not change the data
  const bool vec = (D & 3) == 0;  // rows 16-byte aligned: float4 template loads / stores
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    const int label = synth_label(ctr, b, C, key);
    if (threadIdx.x == 0 && blockIdx.y == 0) y[b] = label;
    const float* tp = tmpl + (int64_t)label * D;
    float* xp = x + (int64_t)b * D;
    for (int d = (blockIdx.y * blockDim.x + threadIdx.x) * 4; d < D; d += gridDim.y * blockDim.x * 4) {
      const uint4 r = synth_noise4(ctr, b, d, key);
      if (vec) {
        const float4 t = *reinterpret_cast<const float4*>(tp + d);
        *reinterpret_cast<float4*>(xp + d) = make_float4(0.5f * t.x + 0.5f * u01(r.x), 0.5f * t.y + 0.5f * u01(r.y),
                                                         0.5f * t.z + 0.5f * u01(r.z), 0.5f * t.w + 0.5f * u01(r.w));
      } else {
        const uint32_t rv[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (d + j < D) xp[d + j] = 0.5f * tp[d + j] + 0.5f * u01(rv[j]);
      }
    }
  }
}

__global__ void bump_counter_k(int32_t* counter) { *counter += 1; }

__global__ void augment_k(const float* __restrict__ x, float* __restrict__ y, int N, int C, int H, int W, int pad,
                          const float* __restrict__ mean, const float* __restrict__ stdv, uint64_t seed,
                          const int32_t* counter) {
  const uint32_t ctr = (uint32_t)*counter;
  const uint2 key = make_uint2((uint32_t)seed ^ 0xA5A5u, (uint32_t)(seed >> 32));
  const int64_t total = (int64_t)N * C * H * W;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int w = i % W, h = (i / W) % H;
    const int c = (i / ((int64_t)H * W)) % C;
    const int n = i / ((int64_t)C * H * W);
    const uint4 r = philox4x32(make_uint4(ctr, (uint32_t)n, 0xAu, 0), key);
    const int dy = (int)(r.x % (uint32_t)(2 * pad + 1)) - pad;
    const int dx = (int)(r.y % (uint32_t)(2 * pad + 1)) - pad;
    const bool flip = r.z & 1u;
    const int sw = flip ? (W - 1 - w) : w;
    const int hh = h + dy, ww = sw + dx;
    float v = 0.f;
    if (hh >= 0 && hh < H && ww >= 0 && ww < W) v = x[(((int64_t)n * C + c) * H + hh) * W + ww];
    y[i] = (v - mean[c]) / stdv[c];
  }
}

__global__ void count_correct_k(const float* __restrict__ logits, const int32_t* __restrict__ y,
                                float* __restrict__ correct, int B, int C) {
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= B) return;
  float mx = -INFINITY;
  int am = 0;
  for (int c = lane; c < C; c += 64) {
    const float v = logits[(int64_t)row * C + c];
    if (v > mx) { mx = v; am = c; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(am, o, 64);
    if (om > mx || (om == mx && oa < am)) { mx = om; am = oa; }
  }
  if (lane == 0 && am == y[row]) atomicAdd(correct, 1.f);
}

}  // namespace

void synth_templates(float* templates, int C, int D, uint64_t seed, hipStream_t st) {
  MX_LAUNCH(synth_templates_k, dim3(cdiv(C * D, 256)), dim3(256), 0, st, templates, C, D, seed);
}

void synth_batch(float* x, int32_t* y, const float* templates, int B, int D, int C, uint64_t seed, int32_t* counter,
                 hipStream_t st, bool bump) {
  const int gy = std::max(1, std::min(64, (D + 256 * 4 * 8 - 1) / (256 * 4 * 8)));  // >= 8 float4 per thread
  MX_LAUNCH(synth_batch_k, dim3(B < 1024 ? B : 1024, gy), dim3(256), 0, st, x, y, templates, B, D, C, seed,
                     counter);
  if (bump) MX_LAUNCH(bump_counter_k, dim3(1), dim3(1), 0, st, counter);
}

void augment_crop_flip_norm(const float* x, float* y, int N, int C, int H, int W, int pad, const float* mean,
                            const float* stdv, uint64_t seed, int32_t* counter, hipStream_t st) {
  const int64_t total = (int64_t)N * C * H * W;
  int g = (int)((total + 255) / 256);
  if (g > 4096) g = 4096;
  MX_LAUNCH(augment_k, dim3(g), dim3(256), 0, st, x, y, N, C, H, W, pad, mean, stdv, seed, counter);
}

void count_correct(const float* logits, const int32_t* y, float* correct, int B, int C, hipStream_t st) {
  MX_LAUNCH(count_correct_k, dim3(cdiv(B, 4)), dim3(256), 0, st, logits, y, correct, B, C);
}

}  // namespace mx
