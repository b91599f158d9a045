// BatchNorm2d (NCHW, fp32 statistics) for gfx950: split-reduction design that fills the chip.
//
// A block-per-channel BN launches only C workgroups (16..271 for PyramidNet, 64..2048 for
// ResNet-50) on a 256-CU part and walks each channel serially.  Here every channel's N*HW
// elements are split over S workgroups (grid = S x C, S chosen so the grid has >= ~2048
// workgroups), each reducing its slice with float4 loads and WRITING its two partial sums to
// part[c][s][2].  The second, elementwise launch uses the same S x C grid: each block first sums
// its channel's S partials (a block reduction in a fixed order: deterministic, and no
// same-address float atomics, which serialise at ~50 ns per arrival across the XCDs), then
// applies the affine map (forward) or the dx formula (backward) to its slice.  The partials are
// fully rewritten by every call, so a captured graph replays with no reset.
//
// Numerics: forward partials are sums of (x - K) and (x - K)^2 with a per-channel shift
// K = x[0, c, 0, 0] (identical in every split), which keeps E[x^2] - E[x]^2 well conditioned
// when |mean| >> std.  Backward partials are sum(dy) and sum(dy * (x - mean)).
//
// Replaces (reference): cuDNN BatchNorm fwd-training / bwd reached from pytorch/model.py:27,30,
// 33,64,74 (PyramidNet) -- SURVEY §2.4.
#include <cstdlib>

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

// sum of channel c's S partial pairs (S <= 4 x kBnTB), fixed order; every thread gets the result
__device__ __forceinline__ float2 channel_sums(const float* __restrict__ part, int c, int S, float* red) {
  float a = 0.f, b = 0.f;
  for (int t = threadIdx.x; t < S; t += kBnTB) {
    const float2 v = reinterpret_cast<const float2*>(part)[(size_t)c * S + t];
    a += v.x;
    b += v.y;
  }
  return block_sum2(a, b, red);
}

// Slice of channel c handled by workgroup s: images [n0, n1), all HW.
struct Slice {
  int n0, n1;
};
__device__ __forceinline__ Slice slice_of(int s, int S, int N) {
  const int per = (N + S - 1) / S;
  return Slice{min(s * per, N), min((s + 1) * per, N)};
}

// The split kernels' vector paths walk their slice in chunks of kBnU float4s per thread with
// every load of a chunk issued before the first is used (a slice is 1..4 float4s per thread for
// the PyramidNet stage-1 BNs: one memory round trip), and the elementwise passes request their
// first chunk before reading the channel's partials, so the two round trips overlap.  Per-thread
// summation order is unchanged (i ascending).
constexpr int kBnU = 4;
struct BnChunk {
  size_t o[kBnU];  // float4 offset of (n, c, j) in an [N][C][HW / 4] tensor
  size_t so[kBnU]; // float4 offset of (n, j) in a side tensor [N][side_c][HW / 4] at channel 0
  bool ok[kBnU];
};
__device__ __forceinline__ BnChunk bn_chunk(int i0, int total, const Slice& sl, int hw4, int C, int c, int side_c,
                                            const FastDiv& dv) {
  BnChunk k;
#pragma unroll
  for (int u = 0; u < kBnU; ++u) {
    const int iu = i0 + u * kBnTB;
    k.ok[u] = iu < total;
    const int i = k.ok[u] ? iu : i0;
    const int n = sl.n0 + (int)dv.div(i), j = i - (n - sl.n0) * hw4;
    k.o[u] = ((size_t)n * C + c) * hw4 + j;
    k.so[u] = ((size_t)n * side_c) * hw4 + j;
  }
  return k;
}

// The fused ReLU's mask of a BN whose output was never stored (its apply folded into the next
// convolution's input staging, ops.bn_conv): recomputed from x with the forward's exact
// fmaf(x, sc, sh), so it is bit for bit the mask of the values the convolution consumed.
__device__ __forceinline__ float4 mask_from_x(float4 g, const float4& v, float2 t) {
  g.x = fmaf(v.x, t.x, t.y) > 0.f ? g.x : 0.f;
  g.y = fmaf(v.y, t.x, t.y) > 0.f ? g.y : 0.f;
  g.z = fmaf(v.z, t.x, t.y) > 0.f ? g.z : 0.f;
  g.w = fmaf(v.w, t.x, t.y) > 0.f ? g.w : 0.f;
  return g;
}

// ------------------------------------------------------------------ forward statistics
template <bool VEC>
__global__ __launch_bounds__(kBnTB) void bn_stats_k(const float* __restrict__ x, int N, int C, int HW, int S, FastDiv dv,
                                                    float* __restrict__ part) {
  __shared__ float red[2 * kBnTB / 64];
  const int s = blockIdx.x, c = blockIdx.y;
  const Slice sl = slice_of(s, S, N);
  const float K = x[(size_t)c * HW];  // shift: x[0, c, 0, 0]
  float s1 = 0.f, s2 = 0.f;
  if (VEC) {
    const int hw4 = HW >> 2;
    const int total = (sl.n1 - sl.n0) * hw4;
    const float4* x4 = reinterpret_cast<const float4*>(x);
    for (int i0 = threadIdx.x; i0 < total; i0 += kBnU * kBnTB) {
      const BnChunk k = bn_chunk(i0, total, sl, hw4, C, c, 0, dv);
      float4 v[kBnU];
#pragma unroll
      for (int u = 0; u < kBnU; ++u) v[u] = x4[k.o[u]];
#pragma unroll
      for (int u = 0; u < kBnU; ++u) {
        if (!k.ok[u]) continue;
        const float a = v[u].x - K, b = v[u].y - K, d = v[u].z - K, e = v[u].w - K;
        s1 += (a + b) + (d + e);
        s2 = fmaf(a, a, fmaf(b, b, fmaf(d, d, fmaf(e, e, s2))));
      }
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
  if (threadIdx.x == 0) reinterpret_cast<float2*>(part)[(size_t)c * S + s] = t;
}

// ------------------------------------------------------------------ backward
// partial sums of g and g * (x - mean), g = dy masked by the fused ReLU (y_relu > 0).
template <bool VEC>
__global__ __launch_bounds__(kBnTB) void bn_bwd_reduce_k(const float* __restrict__ dy, const float* __restrict__ x,
                                                         const float* __restrict__ yr, const float* __restrict__ mean,
                                                         int N, int C, int HW, int S, FastDiv dv,
                                                         float* __restrict__ part, const float2* __restrict__ ssm) {
  __shared__ float red[2 * kBnTB / 64];
  const int s = blockIdx.x, c = blockIdx.y;
  const Slice sl = slice_of(s, S, N);
  const float mu = mean[c];
  const float2 mt = ssm ? ssm[c] : make_float2(0.f, 0.f);  // ssm: the ReLU mask from x (mask_from_x)
  float s1 = 0.f, s2 = 0.f;
  if (VEC) {
    const int hw4 = HW >> 2;
    const int total = (sl.n1 - sl.n0) * hw4;
    const float4 *g4 = reinterpret_cast<const float4*>(dy), *x4 = reinterpret_cast<const float4*>(x),
                 *y4 = reinterpret_cast<const float4*>(yr);
    for (int i0 = threadIdx.x; i0 < total; i0 += kBnU * kBnTB) {
      const BnChunk k = bn_chunk(i0, total, sl, hw4, C, c, 0, dv);
      // the optional operand's loads under one uniform branch (a branch per load made the
      // waitcnt pass drain each load before the next: one round trip per vector)
      float4 g[kBnU], v[kBnU], r[kBnU];
#pragma unroll
      for (int u = 0; u < kBnU; ++u) {
        g[u] = g4[k.o[u]];
        v[u] = x4[k.o[u]];
      }
      if (yr) {
#pragma unroll
        for (int u = 0; u < kBnU; ++u) r[u] = y4[k.o[u]];
      }
#pragma unroll
      for (int u = 0; u < kBnU; ++u) {
        if (!k.ok[u]) continue;
        if (yr) {
          g[u].x = r[u].x > 0.f ? g[u].x : 0.f;
          g[u].y = r[u].y > 0.f ? g[u].y : 0.f;
          g[u].z = r[u].z > 0.f ? g[u].z : 0.f;
          g[u].w = r[u].w > 0.f ? g[u].w : 0.f;
        } else if (ssm) {
          g[u] = mask_from_x(g[u], v[u], mt);
        }
        s1 += (g[u].x + g[u].y) + (g[u].z + g[u].w);
        s2 = fmaf(g[u].x, v[u].x - mu,
                  fmaf(g[u].y, v[u].y - mu, fmaf(g[u].z, v[u].z - mu, fmaf(g[u].w, v[u].w - mu, s2))));
      }
    }
  } else {
    const int total = (sl.n1 - sl.n0) * HW;
    for (int i = threadIdx.x; i < total; i += kBnTB) {
      const int n = sl.n0 + (int)dv.div(i), j = i - (n - sl.n0) * HW;
      const size_t o = ((size_t)n * C + c) * HW + j;
      float g = dy[o];
      if (yr && !(yr[o] > 0.f)) g = 0.f;
      if (!yr && ssm && !(fmaf(x[o], mt.x, mt.y) > 0.f)) g = 0.f;
      s1 += g;
      s2 = fmaf(g, x[o] - mu, s2);
    }
  }
  const float2 t = block_sum2(s1, s2, red);
  if (threadIdx.x == 0) reinterpret_cast<float2*>(part)[(size_t)c * S + s] = t;
}

// Elementwise passes: grid (S, C) exactly like the reductions, so every block works on one
// channel slice and derives that channel's coefficients ONCE (uniform scalars); a flat
// grid-stride version that recomputed mean / invstd and the channel index per element was
// measured slower.  dx = k * (cnt*g - db - xhat*dg), xhat = (x - mean) * invstd,
// k = gamma * invstd / cnt, db = sum(g), dg = sum(g * xhat).  Block (0, c) publishes the
// channel's statistics / dgamma / dbeta and zeroes channel c of the next call's accumulator.
template <bool VEC>
__global__ __launch_bounds__(kBnTB) void bn_apply_slice_k(const float* __restrict__ x, const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, const float* __restrict__ part,
                                                          float* __restrict__ mean_out, float* __restrict__ invstd_out,
                                                          float* __restrict__ run_mean, float* __restrict__ run_var,
                                                          float* __restrict__ y, int N, int C, int HW, int S, FastDiv dv,
                                                          float cnt, float eps, float momentum, int relu,
                                                          int64_t* __restrict__ num_batches,
                                                          const float* __restrict__ res, int Cr,
                                                          float2* __restrict__ ss_out) {
  // y == nullptr (the apply folded into the next convolution, ops.bn_conv): a (1, C) grid that
  // only finalizes -- the statistics and the per-channel (scale, shift) into ss_out
  __shared__ float red[2 * kBnTB / 64];
  const int s = blockIdx.x, c = blockIdx.y;
  if (s == 0 && c == 0 && num_batches && threadIdx.x == 0) *num_batches += 1;
  const Slice sl = slice_of(s, S, N);
  // residual (PyramidNet identity shortcut, channels zero-padded): channel c < Cr adds res[n][c]
  const float* rc = (res && c < Cr) ? res + (size_t)c * HW : nullptr;  // uniform per block
  const int hw4 = HW >> 2, total4 = (sl.n1 - sl.n0) * hw4;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  const float4* r4 = reinterpret_cast<const float4*>(rc);
  float4* y4 = reinterpret_cast<float4*>(y);
  BnChunk k0{};
  float4 v0[kBnU], q0[kBnU];
  if (VEC && y && threadIdx.x < total4) {  // first chunk requested before the partials are read
    k0 = bn_chunk(threadIdx.x, total4, sl, hw4, C, c, Cr, dv);
#pragma unroll
    for (int u = 0; u < kBnU; ++u) {
      v0[u] = x4[k0.o[u]];
      if (r4) q0[u] = r4[k0.so[u]];
    }
  }
  const float K = x[(size_t)c * HW];  // the statistics kernel's shift
  const float2 t = channel_sums(part, c, S, red);
  const float m1 = t.x / cnt;
  const float var = fmaxf(t.y / cnt - m1 * m1, 0.f);
  const float mu = K + m1, inv = rsqrtf(var + eps);
  const float sc = inv * (gamma ? gamma[c] : 1.f);
  const float sh = (beta ? beta[c] : 0.f) - mu * sc;
  if (s == 0 && threadIdx.x == 0) {
    mean_out[c] = mu;
    invstd_out[c] = inv;
    if (run_mean) run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mu;
    if (run_var) run_var[c] = (1.f - momentum) * run_var[c] + momentum * var * cnt / fmaxf(cnt - 1.f, 1.f);
    if (ss_out) ss_out[c] = make_float2(sc, sh);
  }
  if (!y) return;
  if (VEC) {
    auto apply = [&](const BnChunk& k, const float4 (&v)[kBnU], const float4 (&q)[kBnU]) {
#pragma unroll
      for (int u = 0; u < kBnU; ++u) {
        if (!k.ok[u]) continue;
        float4 w = v[u];
        w.x = fmaf(w.x, sc, sh);
        w.y = fmaf(w.y, sc, sh);
        w.z = fmaf(w.z, sc, sh);
        w.w = fmaf(w.w, sc, sh);
        if (relu) {
          w.x = fmaxf(w.x, 0.f);
          w.y = fmaxf(w.y, 0.f);
          w.z = fmaxf(w.z, 0.f);
          w.w = fmaxf(w.w, 0.f);
        }
        if (r4) {
          w.x += q[u].x;
          w.y += q[u].y;
          w.z += q[u].z;
          w.w += q[u].w;
        }
        y4[k.o[u]] = w;
      }
    };
    if (threadIdx.x < total4) apply(k0, v0, q0);
    for (int i0 = threadIdx.x + kBnU * kBnTB; i0 < total4; i0 += kBnU * kBnTB) {
      const BnChunk k = bn_chunk(i0, total4, sl, hw4, C, c, Cr, dv);
      float4 v[kBnU], q[kBnU];
#pragma unroll
      for (int u = 0; u < kBnU; ++u) {
        v[u] = x4[k.o[u]];
        if (r4) q[u] = r4[k.so[u]];
      }
      apply(k, v, q);
    }
  } else {
    const int total = (sl.n1 - sl.n0) * HW;
    for (int i = threadIdx.x; i < total; i += kBnTB) {
      const int n = sl.n0 + (int)dv.div(i), j = i - (n - sl.n0) * HW;
      const size_t o = ((size_t)n * C + c) * HW + j;
      float r = fmaf(x[o], sc, sh);
      if (relu) r = fmaxf(r, 0.f);
      if (rc) r += rc[(size_t)n * Cr * HW + j];
      y[o] = r;
    }
  }
}

template <bool VEC>
__global__ __launch_bounds__(kBnTB) void bn_bwd_apply_slice_k(
    const float* __restrict__ dy, const float* __restrict__ x, const float* __restrict__ yr,
    const float* __restrict__ gamma, const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ part, float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ dx, int N,
    int C, int HW, int S, FastDiv dv, float cnt, int acc_params, const float* __restrict__ extra, int extC,
    const float2* __restrict__ ssm) {
  __shared__ float red[2 * kBnTB / 64];
  const int s = blockIdx.x, c = blockIdx.y;
  const Slice sl = slice_of(s, S, N);
  const float2 mt = ssm ? ssm[c] : make_float2(0.f, 0.f);  // ssm: the ReLU mask from x (mask_from_x)
  // extra: a second gradient of x added to dx (the residual branch's, read in place from the
  // block output gradient [N][extC][HW], channels 0..C-1), instead of a separate add launch
  const float* ec = extra ? extra + (size_t)c * HW : nullptr;
  const int hw4 = HW >> 2, total4 = (sl.n1 - sl.n0) * hw4;
  const float4 *g4 = reinterpret_cast<const float4*>(dy), *x4 = reinterpret_cast<const float4*>(x),
               *y4 = reinterpret_cast<const float4*>(yr), *e4 = reinterpret_cast<const float4*>(ec);
  float4* d4 = reinterpret_cast<float4*>(dx);
  BnChunk k0{};
  float4 g0[kBnU], v0[kBnU], r0[kBnU], e0[kBnU];
  if (VEC && threadIdx.x < total4) {  // first chunk requested before the partials are read
    k0 = bn_chunk(threadIdx.x, total4, sl, hw4, C, c, extC, dv);
#pragma unroll
    for (int u = 0; u < kBnU; ++u) {
      g0[u] = g4[k0.o[u]];
      v0[u] = x4[k0.o[u]];
    }
    if (yr) {  // optional operands under one uniform branch each (see bn_bwd_reduce_k)
#pragma unroll
      for (int u = 0; u < kBnU; ++u) r0[u] = y4[k0.o[u]];
    }
    if (e4) {
#pragma unroll
      for (int u = 0; u < kBnU; ++u) e0[u] = e4[k0.so[u]];
    }
  }
  const float inv = invstd[c], mu = mean[c];
  const float2 t = channel_sums(part, c, S, red);
  const float db = t.x, dg = t.y * inv;
  const float k = (gamma ? gamma[c] : 1.f) * inv / cnt;
  const float A = k * cnt, D = -k * dg * inv, Bc = -k * db + k * dg * inv * mu;
  if (s == 0 && threadIdx.x == 0) {
    if (dgamma) dgamma[c] = acc_params ? dgamma[c] + dg : dg;
    if (dbeta) dbeta[c] = acc_params ? dbeta[c] + db : db;
  }
  if (VEC) {
    auto apply = [&](const BnChunk& k, const float4 (&g)[kBnU], const float4 (&v)[kBnU], const float4 (&r)[kBnU],
                     const float4 (&e)[kBnU]) {
#pragma unroll
      for (int u = 0; u < kBnU; ++u) {
        if (!k.ok[u]) continue;
        float4 gg = g[u];
        if (yr) {
          gg.x = r[u].x > 0.f ? gg.x : 0.f;
          gg.y = r[u].y > 0.f ? gg.y : 0.f;
          gg.z = r[u].z > 0.f ? gg.z : 0.f;
          gg.w = r[u].w > 0.f ? gg.w : 0.f;
        } else if (ssm) {
          gg = mask_from_x(gg, v[u], mt);
        }
        float4 out;
        out.x = fmaf(A, gg.x, fmaf(D, v[u].x, Bc));
        out.y = fmaf(A, gg.y, fmaf(D, v[u].y, Bc));
        out.z = fmaf(A, gg.z, fmaf(D, v[u].z, Bc));
        out.w = fmaf(A, gg.w, fmaf(D, v[u].w, Bc));
        if (e4) {
          out.x += e[u].x;
          out.y += e[u].y;
          out.z += e[u].z;
          out.w += e[u].w;
        }
        d4[k.o[u]] = out;
      }
    };
    if (threadIdx.x < total4) apply(k0, g0, v0, r0, e0);
    for (int i0 = threadIdx.x + kBnU * kBnTB; i0 < total4; i0 += kBnU * kBnTB) {
      const BnChunk k = bn_chunk(i0, total4, sl, hw4, C, c, extC, dv);
      float4 g[kBnU], v[kBnU], r[kBnU], e[kBnU];
#pragma unroll
      for (int u = 0; u < kBnU; ++u) {
        g[u] = g4[k.o[u]];
        v[u] = x4[k.o[u]];
      }
      if (yr) {
#pragma unroll
        for (int u = 0; u < kBnU; ++u) r[u] = y4[k.o[u]];
      }
      if (e4) {
#pragma unroll
        for (int u = 0; u < kBnU; ++u) e[u] = e4[k.so[u]];
      }
      apply(k, g, v, r, e);
    }
  } else {
    const int total = (sl.n1 - sl.n0) * HW;
    for (int i = threadIdx.x; i < total; i += kBnTB) {
      const int n = sl.n0 + (int)dv.div(i), j = i - (n - sl.n0) * HW;
      const size_t o = ((size_t)n * C + c) * HW + j;
      float g = dy[o];
      if (yr && !(yr[o] > 0.f)) g = 0.f;
      if (!yr && ssm && !(fmaf(x[o], mt.x, mt.y) > 0.f)) g = 0.f;
      dx[o] = fmaf(A, g, fmaf(D, x[o], Bc)) + (ec ? ec[(size_t)n * extC * HW + j] : 0.f);
    }
  }
}


// ------------------------------------------------------------------ one block per channel
// For small per-channel counts the split design's two launches (statistics, then the
// elementwise pass) cost more than the work: one block of kBnF threads owns a whole channel,
// reduces it (pass 1), derives the coefficients and applies them (pass 2, the channel's bytes
// are still in L2).  No partials, no second launch; the block reduction is a fixed-shape tree
// (deterministic).  Used for the PyramidNet stage-2 / stage-3 BNs (up to 16 K values per
// channel), where the grid still has one block per channel (106..271 channels).
constexpr int kBnF = 512;

__device__ __forceinline__ float2 block_sum2_f(float a, float b, float* red) {
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
  for (int k = 0; k < kBnF / 64; ++k) {
    t.x += red[2 * k];
    t.y += red[2 * k + 1];
  }
  __syncthreads();
  return t;
}

// HW % 4 == 0 (float4 path only); element e of the channel: image e / HW4, float4 e % HW4.
// U = float4s per thread (the channel's N * HW / 4 <= U * kBnF): every operand of the channel is
// loaded ONCE, all U loads issued before the first is consumed, and kept in registers through
// the block reduction for the apply -- one memory round trip per kernel instead of a serial
// load chain per pass plus a second read of the channel (the loop form measured 7.8 / 9.4 us
// for the PyramidNet stage-2 / 3 BNs, profiles/r3_final/summary_pyr.txt).  Same per-thread
// summation order as the loop form (u ascending), so the results are unchanged.
template <int U>
__device__ __forceinline__ void bn_chan_offsets(int c, int C, int hw4, int total, const FastDiv& dv, int side_c,
                                                size_t (&o)[U], bool (&ok)[U], size_t (&so)[U]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int i0 = threadIdx.x + u * kBnF;
    ok[u] = i0 < total;
    const int i = ok[u] ? i0 : total - 1;  // clamped: every lane loads, masked after
    const int n = (int)dv.div(i), j = i - n * hw4;
    o[u] = ((size_t)n * C + c) * hw4 + j;
    so[u] = ((size_t)n * side_c) * hw4 + j;  // the side operand (residual / shortcut gradient) of image n
  }
}

template <int U>
__global__ __launch_bounds__(kBnF) void bn_fwd_fused_k(const float* __restrict__ x, const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, float* __restrict__ y,
                                                      float* __restrict__ mean_out, float* __restrict__ invstd_out,
                                                      float* __restrict__ run_mean, float* __restrict__ run_var, int N,
                                                      int C, int HW, FastDiv dv, float eps, float momentum, int relu,
                                                      int64_t* __restrict__ num_batches, const float* __restrict__ res,
                                                      int Cr, float2* __restrict__ ss_out) {
  // y == nullptr: statistics and (scale, shift) only (the apply folded into the next convolution)
  __shared__ float red[2 * kBnF / 64];
  const int c = blockIdx.x, hw4 = HW >> 2, total = N * hw4;
  if (c == 0 && num_batches && threadIdx.x == 0) *num_batches += 1;
  size_t o[U], so[U];
  bool ok[U];
  bn_chan_offsets<U>(c, C, hw4, total, dv, Cr, o, ok, so);
  const float4* x4 = reinterpret_cast<const float4*>(x);
  const float4* r4 = (res && c < Cr) ? reinterpret_cast<const float4*>(res + (size_t)c * HW) : nullptr;
  const float K = x[(size_t)c * HW];  // shift: x[0, c, 0, 0]
  float4 v[U], rr[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = x4[o[u]];
  if (r4) {  // residual channel c of image n
#pragma unroll
    for (int u = 0; u < U; ++u) rr[u] = r4[so[u]];
  }
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (!ok[u]) continue;
    const float p = v[u].x - K, q = v[u].y - K, r = v[u].z - K, t = v[u].w - K;
    s1 += (p + q) + (r + t);
    s2 = fmaf(p, p, fmaf(q, q, fmaf(r, r, fmaf(t, t, s2))));
  }
  const float2 st = block_sum2_f(s1, s2, red);
  const float cnt = (float)N * (float)HW;
  const float m1 = st.x / cnt;
  const float var = fmaxf(st.y / cnt - m1 * m1, 0.f);
  const float mu = K + m1, inv = rsqrtf(var + eps);
  const float sc = inv * (gamma ? gamma[c] : 1.f);
  const float sh = (beta ? beta[c] : 0.f) - mu * sc;
  if (threadIdx.x == 0) {
    mean_out[c] = mu;
    invstd_out[c] = inv;
    if (run_mean) run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mu;
    if (run_var) run_var[c] = (1.f - momentum) * run_var[c] + momentum * var * cnt / fmaxf(cnt - 1.f, 1.f);
    if (ss_out) ss_out[c] = make_float2(sc, sh);
  }
  if (!y) return;
  float4* y4 = reinterpret_cast<float4*>(y);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (!ok[u]) continue;
    float4 w = v[u];
    w.x = fmaf(w.x, sc, sh);
    w.y = fmaf(w.y, sc, sh);
    w.z = fmaf(w.z, sc, sh);
    w.w = fmaf(w.w, sc, sh);
    if (relu) {
      w.x = fmaxf(w.x, 0.f);
      w.y = fmaxf(w.y, 0.f);
      w.z = fmaxf(w.z, 0.f);
      w.w = fmaxf(w.w, 0.f);
    }
    if (r4) {
      w.x += rr[u].x;
      w.y += rr[u].y;
      w.z += rr[u].z;
      w.w += rr[u].w;
    }
    y4[o[u]] = w;
  }
}

template <int U>
__global__ __launch_bounds__(kBnF) void bn_bwd_fused_k(const float* __restrict__ dy, const float* __restrict__ x,
                                                      const float* __restrict__ yr, const float* __restrict__ gamma,
                                                      const float* __restrict__ mean, const float* __restrict__ invstd,
                                                      float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                      float* __restrict__ dx, int N, int C, int HW, FastDiv dv,
                                                      int acc_params, const float* __restrict__ extra, int extC,
                                                      const float2* __restrict__ ssm) {
  __shared__ float red[2 * kBnF / 64];
  const int c = blockIdx.x, hw4 = HW >> 2, total = N * hw4;
  size_t o[U], so[U];
  bool ok[U];
  bn_chan_offsets<U>(c, C, hw4, total, dv, extC, o, ok, so);
  const float4* g4 = reinterpret_cast<const float4*>(dy);
  const float4* x4 = reinterpret_cast<const float4*>(x);
  const float4* y4 = reinterpret_cast<const float4*>(yr);
  const float4* e4 = extra ? reinterpret_cast<const float4*>(extra + (size_t)c * HW) : nullptr;
  float4 g[U], v[U], e[U], r[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    g[u] = g4[o[u]];
    v[u] = x4[o[u]];
  }
  // every y load issued before the first mask select (a select right after each load drained it:
  // one round trip per vector)
  if (yr) {
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = y4[o[u]];
  }
  if (e4) {  // the shortcut's gradient (channel c of a wider tensor): issued before the reduction
#pragma unroll
    for (int u = 0; u < U; ++u) e[u] = e4[so[u]];
  }
  if (yr) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      g[u].x = r[u].x > 0.f ? g[u].x : 0.f;
      g[u].y = r[u].y > 0.f ? g[u].y : 0.f;
      g[u].z = r[u].z > 0.f ? g[u].z : 0.f;
      g[u].w = r[u].w > 0.f ? g[u].w : 0.f;
    }
  } else if (ssm) {  // the ReLU mask from x (mask_from_x)
    const float2 mt = ssm[c];
#pragma unroll
    for (int u = 0; u < U; ++u) g[u] = mask_from_x(g[u], v[u], mt);
  }
  const float mu = mean[c], inv = invstd[c];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (!ok[u]) continue;
    s1 += (g[u].x + g[u].y) + (g[u].z + g[u].w);
    s2 = fmaf(g[u].x, v[u].x - mu, fmaf(g[u].y, v[u].y - mu, fmaf(g[u].z, v[u].z - mu, fmaf(g[u].w, v[u].w - mu, s2))));
  }
  const float2 t = block_sum2_f(s1, s2, red);
  const float cnt = (float)N * (float)HW;
  const float db = t.x, dg = t.y * inv;
  const float k = (gamma ? gamma[c] : 1.f) * inv / cnt;
  const float A = k * cnt, D = -k * dg * inv, Bc = -k * db + k * dg * inv * mu;
  if (threadIdx.x == 0) {
    if (dgamma) dgamma[c] = acc_params ? dgamma[c] + dg : dg;
    if (dbeta) dbeta[c] = acc_params ? dbeta[c] + db : db;
  }
  float4* d4 = reinterpret_cast<float4*>(dx);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (!ok[u]) continue;
    float4 out;
    out.x = fmaf(A, g[u].x, fmaf(D, v[u].x, Bc));
    out.y = fmaf(A, g[u].y, fmaf(D, v[u].y, Bc));
    out.z = fmaf(A, g[u].z, fmaf(D, v[u].z, Bc));
    out.w = fmaf(A, g[u].w, fmaf(D, v[u].w, Bc));
    if (e4) {
      out.x += e[u].x;
      out.y += e[u].y;
      out.z += e[u].z;
      out.w += e[u].w;
    }
    d4[o[u]] = out;
  }
}

// float4s per thread of the one-block-per-channel kernels (a power of two, <= 8)
int bn_fused_u(int N, int HW) {
  const int per = (N * (HW / 4) + kBnF - 1) / kBnF;
  return per <= 1 ? 1 : per <= 2 ? 2 : per <= 4 ? 4 : 8;
}

// per-channel blocks when the channel is small enough for one block and there are enough
// channels to occupy the chip: at most 16,384 values per channel
bool bn_use_fused(int N, int C, int HW) {
  return HW % 4 == 0 && (int64_t)N * HW <= 16384 && C >= 64;
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

size_t bn_partial_floats(int N, int C, int HW) { return 2 * (size_t)bn_splits(N, C, HW) * C; }

void bn_fwd_train(const float* x, const float* gamma, const float* beta, float* y, float* mean, float* invstd,
                  float* run_mean, float* run_var, int N, int C, int HW, float momentum, float eps, bool relu,
                  float* part, hipStream_t st, int64_t* num_batches, const float* res, int Cr, float* ss_out) {
  MX_CHECK((int64_t)N * C * HW < (1ll << 31), "bn: tensor too large for 32-bit index math");
  MX_CHECK(y || (ss_out && !res), "bn: without an output, (scale, shift) must be requested and no residual");
  float2* ss2 = reinterpret_cast<float2*>(ss_out);
  const int S = bn_splits(N, C, HW);
  MX_CHECK(S <= 4 * kBnTB, "bn: too many splits");
  MX_CHECK(!res || (Cr > 0 && Cr <= C), "bn: residual channels must be in 1..C");
  if (bn_use_fused(N, C, HW)) {
#define MX_BN_FWD(U_)                                                                                            \
  MX_LAUNCH(bn_fwd_fused_k<U_>, dim3(C), dim3(kBnF), 0, st, x, gamma, beta, y, mean, invstd, run_mean, run_var, N, C, \
            HW, FastDiv(HW / 4), eps, momentum, relu ? 1 : 0, num_batches, res, Cr, ss2)
    switch (bn_fused_u(N, HW)) {
      case 1: MX_BN_FWD(1); break;
      case 2: MX_BN_FWD(2); break;
      case 4: MX_BN_FWD(4); break;
      default: MX_BN_FWD(8); break;
    }
#undef MX_BN_FWD
    return;
  }
  const bool vec = HW % 4 == 0;
  const FastDiv dv(vec ? HW / 4 : HW);
  const float cnt = (float)N * (float)HW;
  const dim3 ga(y ? S : 1, C);  // no output: one finalizing block per channel
  if (vec) {
    MX_LAUNCH(bn_stats_k<true>, dim3(S, C), dim3(kBnTB), 0, st, x, N, C, HW, S, dv, part);
    MX_LAUNCH(bn_apply_slice_k<true>, ga, dim3(kBnTB), 0, st, x, gamma, beta, part, mean, invstd, run_mean,
              run_var, y, N, C, HW, S, dv, cnt, eps, momentum, relu ? 1 : 0, num_batches, res, Cr, ss2);
  } else {
    MX_LAUNCH(bn_stats_k<false>, dim3(S, C), dim3(kBnTB), 0, st, x, N, C, HW, S, dv, part);
    MX_LAUNCH(bn_apply_slice_k<false>, ga, dim3(kBnTB), 0, st, x, gamma, beta, part, mean, invstd, run_mean,
              run_var, y, N, C, HW, S, dv, cnt, eps, momentum, relu ? 1 : 0, num_batches, res, Cr, ss2);
  }
}

void bn_bwd(const float* dy, const float* x, const float* y_relu, const float* gamma, const float* mean,
            const float* invstd, float* dx, float* dgamma, float* dbeta, int N, int C, int HW, bool accp, float* part,
            hipStream_t st, const float* extra, int extC, const float* ssm) {
  MX_CHECK((int64_t)N * C * HW < (1ll << 31), "bn: tensor too large for 32-bit index math");
  const int S = bn_splits(N, C, HW);
  MX_CHECK(S <= 4 * kBnTB, "bn: too many splits");
  MX_CHECK(!extra || extC >= C, "bn: extra gradient must have >= C channels");
  MX_CHECK(!(ssm && y_relu), "bn: one ReLU mask source");
  const float2* m2 = reinterpret_cast<const float2*>(ssm);
  if (bn_use_fused(N, C, HW)) {
#define MX_BN_BWD(U_)                                                                                              \
  MX_LAUNCH(bn_bwd_fused_k<U_>, dim3(C), dim3(kBnF), 0, st, dy, x, y_relu, gamma, mean, invstd, dgamma, dbeta, dx, N, \
            C, HW, FastDiv(HW / 4), accp ? 1 : 0, extra, extC, m2)
    switch (bn_fused_u(N, HW)) {
      case 1: MX_BN_BWD(1); break;
      case 2: MX_BN_BWD(2); break;
      case 4: MX_BN_BWD(4); break;
      default: MX_BN_BWD(8); break;
    }
#undef MX_BN_BWD
    return;
  }
  const bool vec = HW % 4 == 0;
  const FastDiv dv(vec ? HW / 4 : HW);
  const float cnt = (float)N * (float)HW;
  if (vec) {
    MX_LAUNCH(bn_bwd_reduce_k<true>, dim3(S, C), dim3(kBnTB), 0, st, dy, x, y_relu, mean, N, C, HW, S, dv, part, m2);
    MX_LAUNCH(bn_bwd_apply_slice_k<true>, dim3(S, C), dim3(kBnTB), 0, st, dy, x, y_relu, gamma, mean, invstd, part,
              dgamma, dbeta, dx, N, C, HW, S, dv, cnt, accp ? 1 : 0, extra, extC, m2);
  } else {
    MX_LAUNCH(bn_bwd_reduce_k<false>, dim3(S, C), dim3(kBnTB), 0, st, dy, x, y_relu, mean, N, C, HW, S, dv, part, m2);
    MX_LAUNCH(bn_bwd_apply_slice_k<false>, dim3(S, C), dim3(kBnTB), 0, st, dy, x, y_relu, gamma, mean, invstd, part,
              dgamma, dbeta, dx, N, C, HW, S, dv, cnt, accp ? 1 : 0, extra, extC, m2);
  }
}

}  // namespace mx
