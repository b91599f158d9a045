// Flat multi-tensor optimizers over one contiguous fp32 parameter buffer.
// Replace per-parameter torch.optim.SGD (pytorch/distributed_data_parallel.py:94-95)
// and Keras / Chainer Adam (tensorflow2/mnist_single.py:78, chainer/train_mnist.py:69).
// The DDP 1/world_size gradient average is folded in as `gscale` (no extra pass).
#include "common.h"
#include "ops.h"

namespace mx {
namespace {

__global__ void sgd_k(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ buf,
                      const float* __restrict__ lr_ptr, float gscale, float mom, float wd, int64_t n, int first) {
  const float lr = *lr_ptr;
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  float4* p4 = reinterpret_cast<float4*>(p);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  float4* b4 = reinterpret_cast<float4*>(buf);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pv = p4[i], gv = g4[i];
    float gg[4] = {gv.x * gscale + wd * pv.x, gv.y * gscale + wd * pv.y, gv.z * gscale + wd * pv.z,
                   gv.w * gscale + wd * pv.w};
    if (mom != 0.f) {
      float4 bv = first ? make_float4(gg[0], gg[1], gg[2], gg[3]) : b4[i];
      if (!first) {
        bv.x = mom * bv.x + gg[0];
        bv.y = mom * bv.y + gg[1];
        bv.z = mom * bv.z + gg[2];
        bv.w = mom * bv.w + gg[3];
      }
      b4[i] = bv;
      gg[0] = bv.x; gg[1] = bv.y; gg[2] = bv.z; gg[3] = bv.w;
    }
    pv.x -= lr * gg[0];
    pv.y -= lr * gg[1];
    pv.z -= lr * gg[2];
    pv.w -= lr * gg[3];
    p4[i] = pv;
  }
  for (int64_t i = (n4 << 2) + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    float gg = g[i] * gscale + wd * p[i];
    if (mom != 0.f) {
      const float b = first ? gg : mom * buf[i] + gg;
      buf[i] = b;
      gg = b;
    }
    p[i] -= lr * gg;
  }
}

// Adam with the step count on the device, so a captured hipGraph replays it exactly: every
// block reads the count of completed steps state[0], t = count + 1; block 0 records t in
// state[1] and a one-block launch right after (adam_commit_k) publishes it as state[0] -- no
// block ever writes what another block of the same launch reads.  (The previous form -- every
// block arriving on a ticket so the last one publishes -- serialised up to 2,048 same-address
// atomics per step; the Keras engine's update kernel lost ~30 us to the same pattern.)
// eps_hat (Keras / Chainer): m_hat / (sqrt(v_hat) + eps)  ==  m / bc1 / (sqrt(v) / sqrt(bc2) +
// eps / sqrt(bc2)); otherwise torch.optim.Adam's m_hat / (sqrt(v_hat) + eps).
__global__ void adam_k(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                       float* __restrict__ v, const float* __restrict__ lr_ptr, int32_t* __restrict__ state,
                       float gscale, float b1, float b2, float eps, float wd, int eps_hat, int64_t n) {
  const float lr = *lr_ptr;
  const int t = __hip_atomic_load(state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  const float bc1 = 1.f - powf(b1, (float)t), bc2 = 1.f - powf(b2, (float)t);
  const float step_size = lr / bc1;
  const float bc2s = sqrtf(bc2);
  const float e = eps_hat ? eps / bc2s : eps;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float gg = g[i] * gscale + wd * p[i];
    const float mi = b1 * m[i] + (1.f - b1) * gg;
    const float vi = b2 * v[i] + (1.f - b2) * gg * gg;
    m[i] = mi;
    v[i] = vi;
    p[i] -= step_size * mi / (sqrtf(vi) / bc2s + e);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) __hip_atomic_store(state + 1, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void adam_commit_k(int32_t* __restrict__ state) {
  if (threadIdx.x == 0) state[0] = state[1];
}

int grid_for(int64_t n) {
  int64_t g = (n / 4 + 255) / 256;
  if (g > 2048) g = 2048;
  return g < 1 ? 1 : (int)g;
}

}  // namespace

void sgd_step(float* p, const float* g, float* buf, const float* lr, float gscale, float momentum, float wd,
              int64_t n, bool first_step, hipStream_t st) {
  MX_CHECK(((uintptr_t)p % 16 == 0) && ((uintptr_t)g % 16 == 0) && ((uintptr_t)buf % 16 == 0),
           "sgd_step: buffers must be 16-byte aligned");
  MX_LAUNCH(sgd_k, dim3(grid_for(n)), dim3(256), 0, st, p, g, buf, lr, gscale, momentum, wd, n,
                     first_step ? 1 : 0);
}

void adam_step(float* p, const float* g, float* m, float* v, const float* lr, int32_t* state, float gscale,
               float b1, float b2, float eps, float wd, bool eps_hat, int64_t n, hipStream_t st) {
  MX_LAUNCH(adam_k, dim3(grid_for(n * 4)), dim3(256), 0, st, p, g, m, v, lr, state, gscale, b1, b2, eps,
                     wd, eps_hat ? 1 : 0, n);
  MX_LAUNCH(adam_commit_k, dim3(1), dim3(64), 0, st, state);
}

}  // namespace mx
