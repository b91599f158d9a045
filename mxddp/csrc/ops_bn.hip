// BatchNorm2d (NCHW, fp32 statistics) for gfx950: split-reduction design that fills the chip.
//
// A block-per-channel BN launches only C workgroups (16..271 for PyramidNet, 64..2048 for
// ResNet-50) on a 256-CU part and walks each channel serially.  Here every channel's N*HW
// elements are split over S workgroups (grid = S x C, S chosen so the grid has >= ~2048
// workgroups), each reducing its slice with float4 loads and adding its two partial sums into
// per-channel accumulators with device-scope float atomics (2 atomics per workgroup).  The
// second, elementwise launch uses the same S x C grid: each block derives its channel's
// statistics from the accumulators once and applies the affine map (forward) or the dx
// formula (backward) to its slice.
//
// No inter-workgroup fences: a last-arriver scheme needs a device-scope release per workgroup,
// which on a multi-XCD part writes back the XCD's L2 and cost 2-3x the whole reduction.  The
// accumulators are double-buffered instead: call k reduces into buffer k%2 (zero), and its
// elementwise kernel re-zeroes the OTHER buffer for call k+1 (stream order makes this safe) --
// every channel up to `hiwater`, the widest C any call has used on these buffers, since an
// earlier wider call may have left channels >= C dirty.
//
// Numerics: forward partials are sums of (x - K) and (x - K)^2 with a per-channel shift
// K = x[0, c, 0, 0] (identical in every split), which keeps E[x^2] - E[x]^2 well conditioned
// when |mean| >> std.  Backward partials are sum(dy) and sum(dy * (x - mean)).
//
// Replaces (reference): cuDNN BatchNorm fwd-training / bwd reached from pytorch/model.py:27,30,
// 33,64,74 (PyramidNet) -- SURVEY §2.4.
#include "common.h"
#include "ops.h"

namespace mx {

namespace {

constexpr int kBnTB = 256;

__device__ __forceinline__ float2 block_sum2(float a, float b, float* red) {
  a = wave_sum(a);
  b = wave_sum(b);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[2 * w] = a;
    red[2 * w + 1] = b;
  }
  __syncthreads();
  float2 t = make_float2(0.f, 0.f);
#pragma unroll
  for (int k = 0; k < kBnTB / 64; ++k) {
    t.x += red[2 * k];
    t.y += red[2 * k + 1];
  }
  __syncthreads();
  return t;
}

// Slice of channel c handled by workgroup s: images [n0, n1), all HW.
struct Slice {
  int n0, n1;
};
__device__ __forceinline__ Slice slice_of(int s, int S, int N) {
  const int per = (N + S - 1) / S;
  return Slice{min(s * per, N), min((s + 1) * per, N)};
}

// ------------------------------------------------------------------ forward statistics
template <bool VEC>
__global__ __launch_bounds__(kBnTB) void bn_stats_k(const float* __restrict__ x, int N, int C, int HW, int S, FastDiv dv,
                                                    float* __restrict__ acc) {
  __shared__ float red[2 * kBnTB / 64];
  const int s = blockIdx.x, c = blockIdx.y;
  const Slice sl = slice_of(s, S, N);
  const float K = x[(size_t)c * HW];  // shift: x[0, c, 0, 0]
  float s1 = 0.f, s2 = 0.f;
  if (VEC) {
    const int hw4 = HW >> 2;
    const int total = (sl.n1 - sl.n0) * hw4;
    for (int i = threadIdx.x; i < total; i += kBnTB) {
      const int n = sl.n0 + (int)dv.div(i), j = i - (n - sl.n0) * hw4;
      const float4 v = reinterpret_cast<const float4*>(x + ((size_t)n * C + c) * HW)[j];
      const float a = v.x - K, b = v.y - K, d = v.z - K, e = v.w - K;
      s1 += (a + b) + (d + e);
      s2 = fmaf(a, a, fmaf(b, b, fmaf(d, d, fmaf(e, e, s2))));
    }
  } else {
    const int total = (sl.n1 - sl.n0) * HW;
    for (int i = threadIdx.x; i < total; i += kBnTB) {
      const int n = sl.n0 + (int)dv.div(i), j = i - (n - sl.n0) * HW;
      const float a = x[((size_t)n * C + c) * HW + j] - K;
      s1 += a;
      s2 = fmaf(a, a, s2);
    }
  }
  const float2 t = block_sum2(s1, s2, red);
  if (threadIdx.x == 0) {
    atomicAdd(acc + 2 * c, t.x);
    atomicAdd(acc + 2 * c + 1, t.y);
  }
}

// Per-channel statistic helpers shared by the elementwise kernels.
struct FwdStat {
  float mean, inv;
};
__device__ __forceinline__ FwdStat fwd_stat(const float* __restrict__ x, const float* __restrict__ acc, int c, int HW,
                                            float cnt, float eps) {
  const float K = x[(size_t)c * HW];
  const float m1 = acc[2 * c] / cnt;
  const float var = fmaxf(acc[2 * c + 1] / cnt - m1 * m1, 0.f);
  return FwdStat{K + m1, rsqrtf(var + eps)};
}

// ------------------------------------------------------------------ backward
// partial sums of g and g * (x - mean), g = dy masked by the fused ReLU (y_relu > 0).
template <bool VEC>
__global__ __launch_bounds__(kBnTB) void bn_bwd_reduce_k(const float* __restrict__ dy, const float* __restrict__ x,
                                                         const float* __restrict__ yr, const float* __restrict__ mean,
                                                         int N, int C, int HW, int S, FastDiv dv,
                                                         float* __restrict__ acc) {
  __shared__ float red[2 * kBnTB / 64];
  const int s = blockIdx.x, c = blockIdx.y;
  const Slice sl = slice_of(s, S, N);
  const float mu = mean[c];
  float s1 = 0.f, s2 = 0.f;
  if (VEC) {
    const int hw4 = HW >> 2;
    const int total = (sl.n1 - sl.n0) * hw4;
    for (int i = threadIdx.x; i < total; i += kBnTB) {
      const int n = sl.n0 + (int)dv.div(i), j = i - (n - sl.n0) * hw4;
      const size_t base = ((size_t)n * C + c) * HW;
      float4 g = reinterpret_cast<const float4*>(dy + base)[j];
      const float4 v = reinterpret_cast<const float4*>(x + base)[j];
      if (yr) {
        const float4 r = reinterpret_cast<const float4*>(yr + base)[j];
        g.x = r.x > 0.f ? g.x : 0.f;
        g.y = r.y > 0.f ? g.y : 0.f;
        g.z = r.z > 0.f ? g.z : 0.f;
        g.w = r.w > 0.f ? g.w : 0.f;
      }
      s1 += (g.x + g.y) + (g.z + g.w);
      s2 = fmaf(g.x, v.x - mu, fmaf(g.y, v.y - mu, fmaf(g.z, v.z - mu, fmaf(g.w, v.w - mu, s2))));
    }
  } else {
    const int total = (sl.n1 - sl.n0) * HW;
    for (int i = threadIdx.x; i < total; i += kBnTB) {
      const int n = sl.n0 + (int)dv.div(i), j = i - (n - sl.n0) * HW;
      const size_t o = ((size_t)n * C + c) * HW + j;
      float g = dy[o];
      if (yr && !(yr[o] > 0.f)) g = 0.f;
      s1 += g;
      s2 = fmaf(g, x[o] - mu, s2);
    }
  }
  const float2 t = block_sum2(s1, s2, red);
  if (threadIdx.x == 0) {
    atomicAdd(acc + 2 * c, t.x);
    atomicAdd(acc + 2 * c + 1, t.y);
  }
}

// Elementwise passes: grid (S, C) exactly like the reductions, so every block works on one
// channel slice and derives that channel's coefficients ONCE (uniform scalars); a flat
// grid-stride version that recomputed mean / invstd and the channel index per element was
// measured slower.  dx = k * (cnt*g - db - xhat*dg), xhat = (x - mean) * invstd,
// k = gamma * invstd / cnt, db = sum(g), dg = sum(g * xhat).  Block (0, c) publishes the
// channel's statistics / dgamma / dbeta and zeroes channel c of the next call's accumulator.
template <bool VEC>
__global__ __launch_bounds__(kBnTB) void bn_apply_slice_k(const float* __restrict__ x, const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, const float* __restrict__ acc,
                                                          float* __restrict__ acc_next, float* __restrict__ mean_out,
                                                          float* __restrict__ invstd_out, float* __restrict__ run_mean,
                                                          float* __restrict__ run_var, float* __restrict__ y, int N,
                                                          int C, int HW, int S, FastDiv dv, float cnt, float eps,
                                                          float momentum, int relu, int hiwater,
                                                          int64_t* __restrict__ num_batches) {
  const int s = blockIdx.x, c = blockIdx.y;
  if (s == 0 && c == 0) {
    for (int k = 2 * C + threadIdx.x; k < 2 * hiwater; k += kBnTB) acc_next[k] = 0.f;
    if (num_batches && threadIdx.x == 0) *num_batches += 1;
  }
  const FwdStat st = fwd_stat(x, acc, c, HW, cnt, eps);
  const float sc = st.inv * (gamma ? gamma[c] : 1.f);
  const float sh = (beta ? beta[c] : 0.f) - st.mean * sc;
  if (s == 0 && threadIdx.x == 0) {
    mean_out[c] = st.mean;
    invstd_out[c] = st.inv;
    if (run_mean) run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * st.mean;
    if (run_var) {
      const float m1 = acc[2 * c] / cnt;
      const float var = fmaxf(acc[2 * c + 1] / cnt - m1 * m1, 0.f);
      run_var[c] = (1.f - momentum) * run_var[c] + momentum * var * cnt / fmaxf(cnt - 1.f, 1.f);
    }
  }
  // every block of channel c has read acc[2c] (above) before block 0 of the NEXT call zeroes it
  // (stream order); acc_next is only zeroed here, never read
  if (s == 0 && threadIdx.x == 0) {
    acc_next[2 * c] = 0.f;
    acc_next[2 * c + 1] = 0.f;
  }
  const Slice sl = slice_of(s, S, N);
  if (VEC) {
    const int hw4 = HW >> 2;
    const int total = (sl.n1 - sl.n0) * hw4;
    for (int i = threadIdx.x; i < total; i += kBnTB) {
      const int n = sl.n0 + (int)dv.div(i), j = i - (n - sl.n0) * hw4;
      const size_t o = ((size_t)n * C + c) * hw4 + j;
      float4 v = reinterpret_cast<const float4*>(x)[o];
      v.x = fmaf(v.x, sc, sh);
      v.y = fmaf(v.y, sc, sh);
      v.z = fmaf(v.z, sc, sh);
      v.w = fmaf(v.w, sc, sh);
      if (relu) {
        v.x = fmaxf(v.x, 0.f);
        v.y = fmaxf(v.y, 0.f);
        v.z = fmaxf(v.z, 0.f);
        v.w = fmaxf(v.w, 0.f);
      }
      reinterpret_cast<float4*>(y)[o] = v;
    }
  } else {
    const int total = (sl.n1 - sl.n0) * HW;
    for (int i = threadIdx.x; i < total; i += kBnTB) {
      const int n = sl.n0 + (int)dv.div(i), j = i - (n - sl.n0) * HW;
      const size_t o = ((size_t)n * C + c) * HW + j;
      const float r = fmaf(x[o], sc, sh);
      y[o] = relu ? fmaxf(r, 0.f) : r;
    }
  }
}

template <bool VEC>
__global__ __launch_bounds__(kBnTB) void bn_bwd_apply_slice_k(
    const float* __restrict__ dy, const float* __restrict__ x, const float* __restrict__ yr,
    const float* __restrict__ gamma, const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ acc, float* __restrict__ acc_next, float* __restrict__ dgamma, float* __restrict__ dbeta,
    float* __restrict__ dx, int N, int C, int HW, int S, FastDiv dv, float cnt, int acc_params, int hiwater) {
  const int s = blockIdx.x, c = blockIdx.y;
  if (s == 0 && c == 0)
    for (int k = 2 * C + threadIdx.x; k < 2 * hiwater; k += kBnTB) acc_next[k] = 0.f;
  const float inv = invstd[c], mu = mean[c];
  const float db = acc[2 * c], dg = acc[2 * c + 1] * inv;
  const float k = (gamma ? gamma[c] : 1.f) * inv / cnt;
  const float A = k * cnt, D = -k * dg * inv, Bc = -k * db + k * dg * inv * mu;
  if (s == 0 && threadIdx.x == 0) {
    if (dgamma) dgamma[c] = acc_params ? dgamma[c] + dg : dg;
    if (dbeta) dbeta[c] = acc_params ? dbeta[c] + db : db;
    acc_next[2 * c] = 0.f;
    acc_next[2 * c + 1] = 0.f;
  }
  const Slice sl = slice_of(s, S, N);
  if (VEC) {
    const int hw4 = HW >> 2;
    const int total = (sl.n1 - sl.n0) * hw4;
    for (int i = threadIdx.x; i < total; i += kBnTB) {
      const int n = sl.n0 + (int)dv.div(i), j = i - (n - sl.n0) * hw4;
      const size_t o = ((size_t)n * C + c) * hw4 + j;
      float4 g = reinterpret_cast<const float4*>(dy)[o];
      const float4 v = reinterpret_cast<const float4*>(x)[o];
      if (yr) {
        const float4 r = reinterpret_cast<const float4*>(yr)[o];
        g.x = r.x > 0.f ? g.x : 0.f;
        g.y = r.y > 0.f ? g.y : 0.f;
        g.z = r.z > 0.f ? g.z : 0.f;
        g.w = r.w > 0.f ? g.w : 0.f;
      }
      float4 out;
      out.x = fmaf(A, g.x, fmaf(D, v.x, Bc));
      out.y = fmaf(A, g.y, fmaf(D, v.y, Bc));
      out.z = fmaf(A, g.z, fmaf(D, v.z, Bc));
      out.w = fmaf(A, g.w, fmaf(D, v.w, Bc));
      reinterpret_cast<float4*>(dx)[o] = out;
    }
  } else {
    const int total = (sl.n1 - sl.n0) * HW;
    for (int i = threadIdx.x; i < total; i += kBnTB) {
      const int n = sl.n0 + (int)dv.div(i), j = i - (n - sl.n0) * HW;
      const size_t o = ((size_t)n * C + c) * HW + j;
      float g = dy[o];
      if (yr && !(yr[o] > 0.f)) g = 0.f;
      dx[o] = fmaf(A, g, fmaf(D, x[o], Bc));
    }
  }
}


}  // namespace

int bn_splits(int N, int C, int HW) {
  int s = (2048 + C - 1) / C;                             // >= ~2048 workgroups in the grid
  const int64_t per_min = 1024;                           // >= 4 float4 per thread per slice
  const int64_t cap = ((int64_t)N * HW + per_min - 1) / per_min;
  if (s > cap) s = (int)cap;
  if (s > N) s = N;
  if (s < 1) s = 1;
  const int per = (N + s - 1) / s;  // whole images per split; no empty splits
  return (N + per - 1) / per;
}

void bn_fwd_train(const float* x, const float* gamma, const float* beta, float* y, float* mean, float* invstd,
                  float* run_mean, float* run_var, int N, int C, int HW, float momentum, float eps, bool relu,
                  float* acc, float* acc_next, int hiwater, hipStream_t st, int64_t* num_batches) {
  MX_CHECK((int64_t)N * C * HW < (1ll << 31), "bn: tensor too large for 32-bit index math");
  const int S = bn_splits(N, C, HW);
  const bool vec = HW % 4 == 0;
  const FastDiv dv(vec ? HW / 4 : HW), dc(C);
  const int64_t total = (int64_t)N * C * HW;
  const float cnt = (float)N * (float)HW;
  if (vec) {
    MX_LAUNCH(bn_stats_k<true>, dim3(S, C), dim3(kBnTB), 0, st, x, N, C, HW, S, dv, acc);
    MX_LAUNCH(bn_apply_slice_k<true>, dim3(S, C), dim3(kBnTB), 0, st, x, gamma, beta, acc, acc_next, mean, invstd,
              run_mean, run_var, y, N, C, HW, S, dv, cnt, eps, momentum, relu ? 1 : 0, hiwater, num_batches);
  } else {
    MX_LAUNCH(bn_stats_k<false>, dim3(S, C), dim3(kBnTB), 0, st, x, N, C, HW, S, dv, acc);
    MX_LAUNCH(bn_apply_slice_k<false>, dim3(S, C), dim3(kBnTB), 0, st, x, gamma, beta, acc, acc_next, mean, invstd,
              run_mean, run_var, y, N, C, HW, S, dv, cnt, eps, momentum, relu ? 1 : 0, hiwater, num_batches);
  }
}

void bn_bwd(const float* dy, const float* x, const float* y_relu, const float* gamma, const float* mean,
            const float* invstd, float* dx, float* dgamma, float* dbeta, int N, int C, int HW, bool accp, float* acc,
            float* acc_next, int hiwater, hipStream_t st) {
  MX_CHECK((int64_t)N * C * HW < (1ll << 31), "bn: tensor too large for 32-bit index math");
  const int S = bn_splits(N, C, HW);
  const bool vec = HW % 4 == 0;
  const FastDiv dv(vec ? HW / 4 : HW), dc(C);
  const int64_t total = (int64_t)N * C * HW;
  const float cnt = (float)N * (float)HW;
  if (vec) {
    MX_LAUNCH(bn_bwd_reduce_k<true>, dim3(S, C), dim3(kBnTB), 0, st, dy, x, y_relu, mean, N, C, HW, S, dv, acc);
    MX_LAUNCH(bn_bwd_apply_slice_k<true>, dim3(S, C), dim3(kBnTB), 0, st, dy, x, y_relu, gamma, mean, invstd, acc,
              acc_next, dgamma, dbeta, dx, N, C, HW, S, dv, cnt, accp ? 1 : 0, hiwater);
  } else {
    MX_LAUNCH(bn_bwd_reduce_k<false>, dim3(S, C), dim3(kBnTB), 0, st, dy, x, y_relu, mean, N, C, HW, S, dv, acc);
    MX_LAUNCH(bn_bwd_apply_slice_k<false>, dim3(S, C), dim3(kBnTB), 0, st, dy, x, y_relu, gamma, mean, invstd, acc,
              acc_next, dgamma, dbeta, dx, N, C, HW, S, dv, cnt, accp ? 1 : 0, hiwater);
  }
}

}  // namespace mx
