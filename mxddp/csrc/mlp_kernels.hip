// Fused gfx950 kernels for the Chainer MLP training step (fp32 in / fp32 MFMA accumulate).
//
// Reference: chainer/train_mnist.py:13-26 (l1 784->1000, l2 1000->1000, l3 1000->10, ReLU),
// :69 (Adam, alpha 1e-3, eps 1e-8 in Chainer's epsilon-hat form), L.Classifier softmax cross
// entropy + accuracy; ParallelUpdater at chainer/train_mnist_gpu.py:87-93.
//
// One step = 5 launches (world size 1; with gradient collectives K4 / K5 write g and the flat
// Adam of ops_optim.hip runs after the all-reduce):
//   K1  [on-device batch] + l1 forward + bias + ReLU          (split-K over 4 waves, MFMA)
//   K2  l2 forward + bias + ReLU
//   K3  l3 forward (logits) + softmax CE + accuracy + dlogits + dh2 = (dlogits W3) * (h2 > 0)
//   K4  per (256-row slice of W2, 16-column tile): dW2 tile (MFMA) + Adam of the tile, the l2
//       data-gradient partial of the slice (MFMA, plain stores, 4 planes); db2; 4 more blocks:
//       l3 grads on MFMA + Adam, the step's metrics                      -> bucket 0 ready
//   K5  per (16 rows of W1, 112 columns): dh1 = sum of the 4 planes, ReLU-masked; dW1 tile
//       (MFMA) + Adam; db1                                               -> bucket 1 ready
//       (mlp_set_w2_defer: K4's dW2 tiles + their Adam run as 252 extra K5 blocks instead)
// Every LDS tile is staged with all of a thread's loads issued before its first store
// (stage_f4), and the update operands (moments, Adam's step / lr) load at the kernels' tops.
// Every block owns the weights it updates, so old values (needed by K4's data gradient) are
// read before the same block writes the new ones -- no cross-block hazard, no extra launch.
// All cross-block sums are fixed-order (4 data-gradient planes, per-tile loss slots): a step is
// bitwise reproducible.  The Adam step count lives on the device: K4 / K5 read state[0] + 1, K5
// publishes it in state[1], the next step's K1 commits it to state[0] (ops_optim.hip adam_k).
//
// MFMA = v_mfma_f32_16x16x4_f32 (lane l: A[l&15][k=l>>4], B[k=l>>4][l&15]; C row = 4*(l>>4) +
// reg, col = l&15).  Where operands are read as float4 along K, the K order inside a 16-wide
// chunk is permuted (k = 16c + 4g + j for lane group g, register j) identically for A and B.
#include "common.h"
#include "mlp_kernels.h"
#include "rng.h"

namespace mx {
namespace mlp {
namespace {

using L = MlpLayout;
constexpr int kNT = (L::kH + 15) / 16;  // 63 column tiles of the hidden layers (the last half used)

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

struct AdamC {
  float step_size, bc2s, e, b1, b2, wd;
};
// the constants of ops_optim.hip adam_k for step t = completed steps + 1
// the two loads behind AdamC, issued early (at a kernel's top) and consumed late by adam_consts:
// computed where it is needed, the constants cost two serial memory round trips there
struct AdamIn {
  int t;
  float lr;
};
__device__ __forceinline__ AdamIn adam_in(const MlpFused& f) {
  return AdamIn{__hip_atomic_load(f.adam_state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1, *f.lr};
}
__device__ __forceinline__ AdamC adam_consts(const MlpFused& f, const AdamIn& in) {
  const int t = in.t;
  const float bc1 = 1.f - powf(f.b1, (float)t), bc2 = 1.f - powf(f.b2, (float)t);
  AdamC c;
  c.step_size = in.lr / bc1;
  c.bc2s = sqrtf(bc2);
  c.e = f.eps_hat ? f.eps / c.bc2s : f.eps;
  c.b1 = f.b1;
  c.b2 = f.b2;
  c.wd = f.wd;
  return c;
}
__device__ __forceinline__ AdamC adam_consts(const MlpFused& f) { return adam_consts(f, adam_in(f)); }
// adam_k's update of one parameter (same operation order: identical results)
__device__ __forceinline__ void adam_upd(float& p, float& m, float& v, float grad, const AdamC& c) {
  const float gg = grad + c.wd * p;
  m = c.b1 * m + (1.f - c.b1) * gg;
  v = c.b2 * v + (1.f - c.b2) * gg * gg;
  p -= c.step_size * m / (sqrtf(v) / c.bc2s + c.e);
}
// one parameter's gradient: Adam in place (fused) or the gradient into g (all-reduced next)
__device__ __forceinline__ void apply_grad(const MlpFused& f, size_t e, float p_old, float grad, const AdamC& c) {
  if (f.fused_adam) {
    float p = p_old, m = f.m[e], v = f.v[e];
    adam_upd(p, m, v, grad, c);
    f.m[e] = m;
    f.v[e] = v;
    f.p[e] = p;
  } else {
    f.g[e] = grad;
  }
}

// Copy `rows` rows of C4 float4s (global pitch sp floats -> LDS pitch dp floats) with 256 threads:
// each thread issues U loads before its first LDS store.  A plain `load; store` loop waits for
// every load before the next one is issued (the store needs it): one memory round trip per
// float4 -- the bulk of K4's time before (profiles/r6_mlp_stage/).  Loads and stores are both
// clamped rather than predicated: predicated, the compiler sinks each load into its store's branch
// and the round trips are back.
template <int C4, int U>
__device__ __forceinline__ void stage_f4(float* dst, int dp, const float* src, size_t sp, int rows) {
  const int n = rows * C4, tid = threadIdx.x;
  for (int k0 = 0; k0 < n; k0 += 256 * U) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {  // clamped, not predicated: the loads stay branch-free
      const int k = min(k0 + tid + 256 * u, n - 1);
      v[u] = *reinterpret_cast<const float4*>(src + (size_t)(k / C4) * sp + 4 * (k % C4));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {  // past the end: element n - 1 again (the same value, harmless)
      const int k = min(k0 + tid + 256 * u, n - 1);
      *reinterpret_cast<float4*>(dst + (k / C4) * dp + 4 * (k % C4)) = v[u];
    }
  }
}

// ------------------------------------------------------------------------------------------
// K1 / K2: out = ReLU(in W^T + b) for in [B][kIn] (x, pitch 784, or h1, pitch 1024) and W
// [1000][kIn].  Block = (16-row M-tile, 16-column N-tile): (B/16) x 63 blocks; the 4 waves split
// K into 16-wide chunks (chunk c -> wave c % 4), every operand float4 issued up front, two
// accumulator chains per wave; the 4 partials are summed in LDS in a fixed order.  The N-tiles
// of one M-tile are spread over the XCDs while the blocks sharing W rows sit on one (xcd_remap).
// K1 (kSynth) forms its A operand from the on-device generator (ops_data.hip synth_batch's
// recipe: template of the label + uniform noise) instead of loading x, and the blocks of
// N-tile 0 publish x / y for the backward.  K2's h1 columns 1000.. are zero, so its last chunk
// needs no bounds (the W2 values read past a row's end are finite parameters times zero).
template <int kIn, bool kSynth>
__global__ __launch_bounds__(256) void fwd_kernel(MlpFused f) {
  constexpr int kCh = (kIn + 15) / 16, kPerW = (kCh + 3) / 4, kAP = kIn == L::kIn ? L::kIn : L::kHP;
  static_assert(!kSynth || kIn == L::kIn, "the generator feeds l1");
  __shared__ float red[4][16][17];
  const float* W = f.p + (kIn == L::kIn ? L::w1 : L::w2);
  const float* bias = f.p + (kIn == L::kIn ? L::b1 : L::b2);
  float* out = kIn == L::kIn ? f.h1 : f.h2;
  const int MT = f.Bp / 16;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int nt = bid / MT, mt = bid - nt * MT;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, m = lane & 15;
  if (blockIdx.x == 0 && tid == 0) {
    if (kIn == L::kIn) f.adam_state[0] = f.adam_state[1];  // commit the previous step's Adam count
    else if (f.synth) *f.counter += 1;                      // K1 consumed the batch counter
  }
  const int row = 16 * mt + m, n = min(16 * nt + m, L::kH - 1);
  const float* Ap = (kIn == L::kIn ? f.x : f.h1) + (size_t)row * kAP + 4 * g;
  const float* Bp = W + (size_t)n * kIn + 4 * g;
  float4 av[kPerW], bv[kPerW];
  uint2 key = make_uint2(0, 0);
  uint32_t ctr = 0;
  int label = 0;
  if constexpr (kSynth) {
    key = synth_key(f.seed);
    ctr = (uint32_t)*f.counter;
    label = synth_label(ctr, row, L::kNC, key);
  }
#pragma unroll
  for (int i = 0; i < kPerW; ++i) {
    const int c = min(w + 4 * i, kCh - 1);  // clamped: the chunk is masked below
    bv[i] = *reinterpret_cast<const float4*>(Bp + 16 * c);
    if constexpr (kSynth)
      av[i] = *reinterpret_cast<const float4*>(f.tmpl + label * L::kIn + 16 * c + 4 * g);
    else
      av[i] = *reinterpret_cast<const float4*>(Ap + 16 * c);
  }
  if constexpr (kSynth) {
#pragma unroll
    for (int i = 0; i < kPerW; ++i) {
      const int c = min(w + 4 * i, kCh - 1), d = 16 * c + 4 * g;
      const uint4 r = synth_noise4(ctr, row, d, key);
      const float4 t = av[i];
      av[i] = make_float4(0.5f * t.x + 0.5f * u01(r.x), 0.5f * t.y + 0.5f * u01(r.y), 0.5f * t.z + 0.5f * u01(r.z),
                          0.5f * t.w + 0.5f * u01(r.w));
      if (nt == 0 && w + 4 * i < kCh) *reinterpret_cast<float4*>(f.x + (size_t)row * L::kIn + d) = av[i];
    }
    if (nt == 0 && w == 0 && g == 0) f.y[row] = label;
  }
  // every operand load issued before the first MFMA (left alone, the scheduler interleaves each
  // load with its MFMAs and the wave waits on L2 once per chunk)
  __builtin_amdgcn_sched_barrier(0);
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int i = 0; i < kPerW; ++i) {
    const bool ok = w + 4 * i < kCh;
    const float4 a = ok ? av[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    acc[0] = mfma4(a.x, bv[i].x, acc[0]);
    acc[1] = mfma4(a.y, bv[i].y, acc[1]);
    acc[0] = mfma4(a.z, bv[i].z, acc[0]);
    acc[1] = mfma4(a.w, bv[i].w, acc[1]);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) red[w][4 * g + j][m] = acc[0][j] + acc[1][j];
  __syncthreads();
  const int r = tid >> 4, col = tid & 15, no = 16 * nt + col;
  const float v = ((red[0][r][col] + red[1][r][col]) + (red[2][r][col] + red[3][r][col])) + bias[min(no, L::kH - 1)];
  float* o = out + (size_t)(16 * mt + r) * L::kHP;
  o[no] = no < L::kH ? fmaxf(v, 0.f) : 0.f;
  if (nt == kNT - 1) o[16 * kNT + col] = 0.f;  // columns 1008 .. 1023 of the padded row
}

// ------------------------------------------------------------------------------------------
// K3: head.  Block = (16-row M-tile, 128-column group of h2): (B/16) x 8 blocks.  Every block
// computes the 16 rows' logits (K = 1000 split over the 4 waves, MFMA with W3's 10 rows padded to
// 16), softmax cross entropy, accuracy and dlogits = (softmax - onehot) / B, then its slice of
// dh2 = (dlogits W3) * (h2 > 0) (K = 10, VALU, W3 columns in LDS).  Column group 0 publishes
// dlogits and the tile's loss / correct sums (fixed order) for K4.
__global__ __launch_bounds__(256) void head_kernel(MlpFused f) {
  constexpr int kCh = (L::kH + 15) / 16, kPerW = (kCh + 3) / 4;
  __shared__ float red[4][16][17];
  __shared__ float dls[16][17];
  __shared__ float w3s[L::kNC][128];
  __shared__ float lc[2][16];
  const int mt = blockIdx.x >> 3, cg = blockIdx.x & 7;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, m = lane & 15;
  const int row = 16 * mt + m;
  const float* Ap = f.h2 + (size_t)row * L::kHP + 4 * g;
  const float* Bp = f.p + L::w3 + (size_t)min(m, L::kNC - 1) * L::kH + 4 * g;
  const float bm = m < L::kNC ? 1.f : 0.f;
  float4 av[kPerW], bv[kPerW];
#pragma unroll
  for (int i = 0; i < kPerW; ++i) {
    const int c = min(w + 4 * i, kCh - 1);
    av[i] = *reinterpret_cast<const float4*>(Ap + 16 * c);
    bv[i] = *reinterpret_cast<const float4*>(Bp + 16 * c);
  }
  float w3v[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) {  // W3 columns of this group: [10][128] = 1280 = 5 x 256
    const int i = tid + 256 * k, c = i >> 7, j = 128 * cg + (i & 127);
    w3v[k] = f.p[L::w3 + c * L::kH + min(j, L::kH - 1)] * (j < L::kH ? 1.f : 0.f);
  }
  // the softmax's bias and label (threads 0..15: one row each), in flight now, not after the barrier
  float b3v[L::kNC];
  int yv = 0;
  if (tid < 16) {
#pragma unroll
    for (int c = 0; c < L::kNC; ++c) b3v[c] = f.p[L::b3 + c];
    yv = f.y[16 * mt + tid];
  }
  // this thread's h2 values for the dh2 mask at the end (one column, 8 rows), also in flight now
  const int jl = tid & 127, j = 128 * cg + jl, r0 = (tid >> 7) * 8;
  float hv[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) hv[k] = f.h2[(size_t)(16 * mt + r0 + k) * L::kHP + j];
  __builtin_amdgcn_sched_barrier(0);  // all operand loads in flight first (see fwd_kernel)
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int i = 0; i < kPerW; ++i) {
    const float4 a = w + 4 * i < kCh ? av[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 b = bv[i];
    acc[0] = mfma4(a.x, b.x * bm, acc[0]);
    acc[1] = mfma4(a.y, b.y * bm, acc[1]);
    acc[0] = mfma4(a.z, b.z * bm, acc[0]);
    acc[1] = mfma4(a.w, b.w * bm, acc[1]);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) red[w][4 * g + j][m] = acc[0][j] + acc[1][j];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const int i = tid + 256 * k;
    w3s[i >> 7][i & 127] = w3v[k];
  }
  __syncthreads();
  if (tid < 16) {  // softmax cross entropy of row tid of the tile
    float l[L::kNC];
#pragma unroll
    for (int c = 0; c < L::kNC; ++c)
      l[c] = ((red[0][tid][c] + red[1][tid][c]) + (red[2][tid][c] + red[3][tid][c])) + b3v[c];
    const int y = yv;
    float mx = l[0];
    int am = 0;
#pragma unroll
    for (int c = 1; c < L::kNC; ++c)
      if (l[c] > mx) { mx = l[c]; am = c; }
    float se = 0.f;
#pragma unroll
    for (int c = 0; c < L::kNC; ++c) se += __expf(l[c] - mx);
    const float lse = mx + __logf(se);
    float ly = 0.f;
#pragma unroll
    for (int c = 0; c < L::kNC; ++c) ly = c == y ? l[c] : ly;
    // rows B.. of the last tile (batch not a multiple of 16): no loss, no accuracy, no gradient
    const float live = 16 * mt + tid < f.B ? 1.f : 0.f;
    lc[0][tid] = (lse - ly) * live;
    lc[1][tid] = am == y ? live : 0.f;
    const float inv = live / (float)f.B;
#pragma unroll
    for (int c = 0; c < L::kNC; ++c) dls[tid][c] = (__expf(l[c] - lse) - (c == y ? 1.f : 0.f)) * inv;
#pragma unroll
    for (int c = L::kNC; c < 16; ++c) dls[tid][c] = 0.f;
  }
  __syncthreads();
  if (cg == 0) {
    f.dl[(size_t)(16 * mt + (tid >> 4)) * 16 + (tid & 15)] = dls[tid >> 4][tid & 15];
    if (tid < 2) {
      float s = 0.f;
      for (int i = 0; i < 16; ++i) s += lc[tid][i];
      f.lsum[2 * mt + tid] = s;
    }
  }
  // dh2 of the 16 rows x 128 columns: thread = one column, 8 rows
  float wc[L::kNC];
#pragma unroll
  for (int c = 0; c < L::kNC; ++c) wc[c] = w3s[c][jl];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < L::kNC; ++c) s = fmaf(dls[r0 + k][c], wc[c], s);
    f.dh2[(size_t)(16 * mt + r0 + k) * L::kHP + j] = hv[k] > 0.f ? s : 0.f;  // h2 pad columns are 0
  }
}

// ------------------------------------------------------------------------------------------
// K4's l3 blocks [252, 256): wave wv (0 .. 15) owns W3 column tiles jt = wv + 16 u (u < 4) --
// dW3 tile [16 classes (10 used)][16 columns] = dl^T . h2[:, tile] (MFMA, K = B) -> Adam / g;
// wave 0 also db3 (the same MFMA against ones), and the spare tile (jt = 63) is the step's
// metrics.  Every operand and the update's values load up front (one memory round trip, not one
// per parameter).  Four blocks only: K4's dynamic LDS (the l2 blocks' 87 KB) holds each block on
// a CU of its own, and 252 + 4 fills the 256 CUs exactly.
constexpr int kK4L3 = 4;
__device__ __forceinline__ void l3_body(const MlpFused& f, int wv, const AdamIn& ain) {
  const int B = f.Bp;
  const int lane = threadIdx.x & 63, g = lane >> 4, m = lane & 15;
  constexpr int kU = 4, kS3 = 16;  // tiles per wave; k-steps of 4 rows per operand chunk
  const bool l3b = wv == 0, met = wv + 16 * (kU - 1) == kNT && f.metrics;
  float dlv[kS3], h2v[kU][kS3], p3[kU][4], m3[kU][4], v3[kU][4], pb[4], mb[4], vb[4];
  float ls_t = 0.f, cs_t = 0.f;
#pragma unroll
  for (int s = 0; s < kS3; ++s) {
    const int b = min(4 * s + g, B - 1);
    dlv[s] = f.dl[b * 16 + m];
#pragma unroll
    for (int u = 0; u < kU; ++u)
      h2v[u][s] = f.h2[(size_t)b * L::kHP + min(16 * (wv + 16 * u) + m, L::kH - 1)];
  }
#pragma unroll
  for (int u = 0; u < kU; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = min(4 * g + r, L::kNC - 1);
      const size_t e = L::w3 + (size_t)c * L::kH + min(16 * (wv + 16 * u) + m, L::kH - 1);
      p3[u][r] = f.p[e];
      if (f.fused_adam) {
        m3[u][r] = f.m[e];
        v3[u][r] = f.v[e];
      }
    }
  if (l3b)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const size_t eb = L::b3 + min(4 * g + r, L::kNC - 1);
      pb[r] = f.p[eb];
      if (f.fused_adam) {
        mb[r] = f.m[eb];
        vb[r] = f.v[eb];
      }
    }
  if (met && lane < B / 16) {  // K3's per-tile sums
    ls_t = f.lsum[2 * lane];
    cs_t = f.lsum[2 * lane + 1];
  }
  f32x4 a3[kU][2], ab = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < kU; ++u) a3[u][0] = a3[u][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int s0 = 0; s0 < B / 4; s0 += kS3) {
    if (s0)  // B > 64: the next chunk
#pragma unroll
      for (int s = 0; s < kS3; ++s) {
        const int b = min(4 * (s0 + s) + g, B - 1);
        dlv[s] = f.dl[b * 16 + m];
#pragma unroll
        for (int u = 0; u < kU; ++u)
          h2v[u][s] = f.h2[(size_t)b * L::kHP + min(16 * (wv + 16 * u) + m, L::kH - 1)];
      }
#pragma unroll
    for (int s = 0; s < kS3; ++s)
      if (s0 + s < B / 4) {
#pragma unroll
        for (int u = 0; u < kU; ++u) a3[u][s & 1] = mfma4(dlv[s], h2v[u][s], a3[u][s & 1]);
        if (l3b) ab = mfma4(dlv[s], 1.f, ab);
      }
  }
  const AdamC ac = adam_consts(f, ain);
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const int j3 = 16 * (wv + 16 * u) + m;
    if (j3 >= L::kH) continue;  // tile 62's columns 1000.. and the metrics tile
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = 4 * g + r;
      if (c >= L::kNC) continue;
      const size_t e = L::w3 + (size_t)c * L::kH + j3;
      const float gw = a3[u][0][r] + a3[u][1][r];
      if (f.fused_adam) {
        adam_upd(p3[u][r], m3[u][r], v3[u][r], gw, ac);
        f.m[e] = m3[u][r];
        f.v[e] = v3[u][r];
        f.p[e] = p3[u][r];
      } else {
        f.g[e] = gw;
      }
    }
  }
  if (l3b && m == 0)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = 4 * g + r;
      if (c >= L::kNC) continue;
      const size_t e = L::b3 + c;
      if (f.fused_adam) {
        adam_upd(pb[r], mb[r], vb[r], ab[r], ac);
        f.m[e] = mb[r];
        f.v[e] = vb[r];
        f.p[e] = pb[r];
      } else {
        f.g[e] = ab[r];
      }
    }
  if (met) {  // fixed order: tile 0, 1, ..
    float ls = 0.f, cs = 0.f;
#pragma unroll
    for (int t = 0; t < 32; ++t)
      if (t < B / 16) {
        ls += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ls_t), t));
        cs += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cs_t), t));
      }
    if (lane == 0) {
      atomicAdd(f.metrics, ls);
      atomicAdd(f.metrics + 1, cs);
    }
  }
}

// ------------------------------------------------------------------------------------------
// K4: l2 / l3 backward.  Blocks [0, 252): (row slice ri of W2: rows 256 ri .. +255, column tile
// jt: W2 columns 16 jt .. +15).  The slice's dh2 columns [B][256] (pitch 260: the data-gradient
// A reads are bank-conflict free), the W2 tile [256][16] (OLD weights) and h1's 16 columns are
// staged in LDS, then
//   dh1 partial [B][16] = dh2[:, slice] . W2[slice, tile]  (MFMA, K = 256) -> plane ri (plain stores)
//   dW2 tile [256][16]  = dh2[:, slice]^T . h1[:, tile]    (MFMA, K = B)   -> Adam / g
//   db2 (tile 0 of each slice)                                              -> Adam / g
// With f.w2_defer the dW2 tile + its update move to extra blocks of K5 (w2_update_body): K4
// keeps only what K5's l1 blocks wait for (the dh1 planes), so the chain K4 -> K5 is shorter and
// the W2 work fills K5's spare resident slots instead.
// Blocks [252, 256): l3's gradient (dW3, db3) and the step's metrics, l3_body.
constexpr int kRS = 256, kDhP = 260, kK4A = 4 * kNT;
constexpr int kBC2 = 128;  // batch rows per LDS pass of K4 (dh2 [128][260] + W2 tile + h1: 157 KB)
__global__ __launch_bounds__(256) void bwd2_kernel(MlpFused f) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int B = f.Bp;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, m = lane & 15;
  if ((int)blockIdx.x >= kK4A) {
    l3_body(f, 4 * (blockIdx.x - kK4A) + w, adam_in(f));
    return;
  }
  const int bid = xcd_remap(blockIdx.x, kK4A);  // the tiles of one row slice share an XCD's L2
  const int ri = bid / kNT, jt = bid - ri * kNT;
  const int i0 = kRS * ri;
  const int BC = min(B, kBC2);      // rows per pass (the dynamic LDS is sized for BC, bwd2_lds)
  const bool dw2 = !f.w2_defer;     // else K5's resident W2 blocks own the dW2 tile (w2_update_body)
  const AdamIn ain = adam_in(f);
  float* dh2s = sm;                 // [BC][260]
  float* w2s = dh2s + BC * kDhP;    // [256][16]
  float* h1s = w2s + kRS * 16;      // [BC][16]
  // the update's moments (and db2's operands in column tile 0) in flight behind the staging
  const int j = 16 * jt + m;
  float mv[4][4], vv[4][4], bp = 0.f, bm = 0.f, bv = 0.f;
  if (dw2 && f.fused_adam) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = min(i0 + 16 * (w + 4 * q) + 4 * g + r, L::kH - 1);
        const size_t e = L::w2 + (size_t)i * L::kH + min(j, L::kH - 1);
        mv[q][r] = f.m[e];
        vv[q][r] = f.v[e];
      }
  }
  if (jt == 0) {
    const size_t e = L::b2 + min(i0 + tid, L::kH - 1);
    bp = f.p[e];
    if (f.fused_adam) {
      bm = f.m[e];
      bv = f.v[e];
    }
  }
  // W2 tile: thread = row i0 + tid, 16 columns (zero outside the 1000 x 1000 matrix); stored to
  // LDS after the first pass's dh2 loads are issued, so all of them are one memory round trip
  float4 w2v[4];
  {
    const int i = min(i0 + tid, L::kH - 1);
    const float4* src = reinterpret_cast<const float4*>(f.p + L::w2 + (size_t)i * L::kH + 16 * jt);
#pragma unroll
    for (int q = 0; q < 4; ++q) w2v[q] = src[q];
  }
  // the batch in passes of kBC2 rows (one pass for B <= 128): the dW2 tile and the db2 sums
  // accumulate across passes in registers, in a fixed order (deterministic)
  f32x4 dw[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) dw[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  float s2[4] = {0.f, 0.f, 0.f, 0.f};
  for (int c0 = 0; c0 < B; c0 += BC) {
    const int bc = min(BC, B - c0);
    if (c0) __syncthreads();  // the previous pass's LDS reads are done
    // dh2 columns i0 .. i0 + 255 (pad columns are 0)
    stage_f4<64, 16>(dh2s, kDhP, f.dh2 + (size_t)c0 * L::kHP + i0, L::kHP, bc);
    if (dw2) stage_f4<4, 2>(h1s, 16, f.h1 + (size_t)c0 * L::kHP + 16 * jt, L::kHP, bc);
    if (c0 == 0) {
      const bool rok = i0 + tid < L::kH;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool cok = rok && 16 * jt + 4 * q < L::kH;  // 1000 % 4 == 0: whole float4s
        *reinterpret_cast<float4*>(w2s + tid * 16 + 4 * q) = cok ? w2v[q] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    __syncthreads();
    // dh1 partial: M = batch (wave w: M-tiles w, w+4, ..), N = 16 columns, K = the 256 rows
    for (int mt = w; mt < bc / 16; mt += 4) {
      f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
      const float* a = dh2s + (16 * mt + m) * kDhP + g;
      const float* bb = w2s + g * 16 + m;
#pragma unroll 16
      for (int s = 0; s < kRS / 4; ++s) acc[s & 1] = mfma4(a[4 * s], bb[64 * s], acc[s & 1]);
      float* dst = f.dh1p + ((size_t)ri * B + c0 + 16 * mt + 4 * g) * L::kHP + 16 * jt + m;
#pragma unroll
      for (int r = 0; r < 4; ++r) dst[(size_t)r * L::kHP] = acc[0][r] + acc[1][r];
    }
    // dW2 tile: M = the 256 rows (wave w: tiles w, w+4, w+8, w+12), N = 16 columns, K = batch
    if (dw2)
      for (int s = 0; s < bc / 4; ++s) {
        const float bvv = h1s[(4 * s + g) * 16 + m];
        const float* a = dh2s + (4 * s + g) * kDhP + m;
#pragma unroll
        for (int q = 0; q < 4; ++q) dw[q] = mfma4(a[16 * (w + 4 * q)], bvv, dw[q]);
      }
    if (jt == 0)  // db2 of the slice's rows: fixed-order column sums
      for (int b = 0; b < bc; b += 4)
#pragma unroll
        for (int k = 0; k < 4; ++k) s2[k] += dh2s[(b + k) * kDhP + tid];
  }
  const AdamC ac = adam_consts(f, ain);
  if (dw2 && j < L::kH) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int il = 16 * (w + 4 * q) + 4 * g + r, i = i0 + il;
        if (i < L::kH) {
          const size_t e = L::w2 + (size_t)i * L::kH + j;
          if (f.fused_adam) {
            float p = w2s[il * 16 + m];
            adam_upd(p, mv[q][r], vv[q][r], dw[q][r], ac);
            f.m[e] = mv[q][r];
            f.v[e] = vv[q][r];
            f.p[e] = p;
          } else {
            f.g[e] = dw[q][r];
          }
        }
      }
  }
  if (jt == 0 && i0 + tid < L::kH) {
    const size_t e = L::b2 + i0 + tid;
    const float gb = (s2[0] + s2[1]) + (s2[2] + s2[3]);
    if (f.fused_adam) {
      adam_upd(bp, bm, bv, gb, ac);
      f.m[e] = bm;
      f.v[e] = bv;
      f.p[e] = bp;
    } else {
      f.g[e] = gb;
    }
  }
}

// ------------------------------------------------------------------------------------------
// K5's resident W2 blocks (f.w2_defer): K4 block (ri, jt)'s dW2 tile + update, off the dgrad chain
// K4 -> K5.  dh2's slice and h1's 16 tile columns are staged in passes of kBCW rows (35 KB: four
// blocks per CU next to K5's own); the MFMA sequence is K4's (s = 0 .. B/4 - 1 in order), so the
// update is bitwise the folded one.  The tile's OLD W2 values come from global memory: nothing
// writes W2 between K4's reads of it and these blocks.
constexpr int kBCW = 32;
__device__ __forceinline__ void w2_update_body(const MlpFused& f, float* sm, int bid) {
  const int B = f.Bp;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, m = lane & 15;
  const int ri = bid / kNT, jt = bid - ri * kNT, i0 = kRS * ri;
  float* dh2s = sm;                 // [kBCW][260]
  float* h1s = dh2s + kBCW * kDhP;  // [kBCW][16]
  const int j = 16 * jt + m;
  const AdamIn ain = adam_in(f);
  float pv[4][4], mv[4][4], vv[4][4];
  if (f.fused_adam)  // the update's operands in flight behind the staging (they do not depend on it)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = min(i0 + 16 * (w + 4 * q) + 4 * g + r, L::kH - 1);
        const size_t e = L::w2 + (size_t)i * L::kH + min(j, L::kH - 1);
        pv[q][r] = f.p[e];
        mv[q][r] = f.m[e];
        vv[q][r] = f.v[e];
      }
  f32x4 dw[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) dw[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int c0 = 0; c0 < B; c0 += kBCW) {
    const int bc = min(kBCW, B - c0);
    if (c0) __syncthreads();
    stage_f4<64, 8>(dh2s, kDhP, f.dh2 + (size_t)c0 * L::kHP + i0, L::kHP, bc);
    stage_f4<4, 1>(h1s, 16, f.h1 + (size_t)c0 * L::kHP + 16 * jt, L::kHP, bc);
    __syncthreads();
    for (int s = 0; s < bc / 4; ++s) {
      const float bvv = h1s[(4 * s + g) * 16 + m];
      const float* a = dh2s + (4 * s + g) * kDhP + m;
#pragma unroll
      for (int q = 0; q < 4; ++q) dw[q] = mfma4(a[16 * (w + 4 * q)], bvv, dw[q]);
    }
  }
  if (j >= L::kH) return;
  const AdamC ac = adam_consts(f, ain);
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + 16 * (w + 4 * q) + 4 * g + r;
      if (i < L::kH) {
        const size_t e = L::w2 + (size_t)i * L::kH + j;
        if (f.fused_adam) {
          adam_upd(pv[q][r], mv[q][r], vv[q][r], dw[q][r], ac);
          f.m[e] = mv[q][r];
          f.v[e] = vv[q][r];
          f.p[e] = pv[q][r];
        } else {
          f.g[e] = dw[q][r];
        }
      }
    }
}

// ------------------------------------------------------------------------------------------
// K5: l1 backward.  Block = (16 rows of W1 = hidden units 16 nt .., 112 input columns 112 kg ..):
// 63 x 7 blocks.  dh1 [B][16] = sum of K4's 4 planes (fixed order), masked by h1 > 0, and x's
// 112 columns are staged in LDS (pitch 112: lane groups 16 banks apart); wave w computes the
// 16 x 16 dW1 tiles kt = w, w + 4 (M = rows, N = columns, K = batch) and applies Adam to them;
// db1 in the column-group-0 blocks.  Block 0 publishes the Adam step count.  With f.w2_defer
// blocks [0, 252) are the W2 blocks above (first: they are the longer ones, and blockIdx order
// spreads them over all XCDs) and the l1 blocks follow.
constexpr int kBC1 = 256;  // batch rows per LDS pass of K5 (dh1 [256][16] + x [256][112]: 128 KB)
__global__ __launch_bounds__(256) void bwd1_kernel(MlpFused f) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int B = f.Bp;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, m = lane & 15;
  if (blockIdx.x == 0 && tid == 0 && f.fused_adam)
    __hip_atomic_store(f.adam_state + 1, __hip_atomic_load(f.adam_state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int w2b = f.w2_defer ? kK4A : 0;
  if ((int)blockIdx.x < w2b) {
    w2_update_body(f, sm, xcd_remap(blockIdx.x, kK4A));
    return;
  }
  const AdamIn ain = adam_in(f);
  const int bid = xcd_remap(blockIdx.x - w2b, kNT * 7);
  const int nt = bid / 7, kg = bid - nt * 7;
  const int BC = min(B, kBC1);   // rows per pass (the dynamic LDS is sized for BC, bwd1_lds)
  float* dh1s = sm;              // [BC][16]
  float* xs = dh1s + BC * 16;    // [BC][112]
  float pv[2][4], mv[2][4], vv[2][4];  // the update's operands, in flight behind the staging
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int kt = min(w + 4 * u, 6), k = 112 * kg + 16 * kt + m;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const size_t e = L::w1 + (size_t)min(16 * nt + 4 * g + r, L::kH - 1) * L::kIn + k;
      pv[u][r] = f.p[e];
      if (f.fused_adam) {
        mv[u][r] = f.m[e];
        vv[u][r] = f.v[e];
      }
    }
  }
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  float s1[4] = {0.f, 0.f, 0.f, 0.f};
  const size_t pl = (size_t)B * L::kHP;
  for (int c0 = 0; c0 < B; c0 += BC) {  // one pass for B <= 256; fixed accumulation order
    const int bc = min(BC, B - c0);
    if (c0) __syncthreads();
    // x's 112 columns: 7 float4 per thread at B = 64, loaded with dh1's operands, stored after
    constexpr int kXU = 7;
    const int nx = bc * 28;
    float4 xv[kXU];
#pragma unroll
    for (int u = 0; u < kXU; ++u) {
      const int k = min(tid + 256 * u, nx - 1);
      xv[u] = *reinterpret_cast<const float4*>(f.x + (size_t)(c0 + k / 28) * L::kIn + 112 * kg + 4 * (k % 28));
    }
    for (int k0 = 0; k0 < bc * 16; k0 += 1024) {  // 4 elements per thread, all loads in flight
      float dv[4][4], hv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = min(k0 + tid + 256 * u, bc * 16 - 1);  // clamped: branch-free loads
        const size_t o = (size_t)(c0 + (k >> 4)) * L::kHP + 16 * nt + (k & 15);
#pragma unroll
        for (int pp = 0; pp < 4; ++pp) dv[u][pp] = f.dh1p[pp * pl + o];
        hv[u] = f.h1[o];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = k0 + tid + 256 * u;
        const float s = (dv[u][0] + dv[u][1]) + (dv[u][2] + dv[u][3]);
        dh1s[min(k, bc * 16 - 1)] = hv[u] > 0.f ? s : 0.f;  // h1 pad columns are 0: those planes' garbage is dropped
      }
    }
#pragma unroll
    for (int u = 0; u < kXU; ++u) {
      const int k = min(tid + 256 * u, nx - 1);
      *reinterpret_cast<float4*>(xs + (k / 28) * 112 + 4 * (k % 28)) = xv[u];
    }
    if (nx > 256 * kXU)  // B > 64: the rest
      stage_f4<28, 7>(xs + 64 * 112, 112, f.x + (size_t)(c0 + 64) * L::kIn + 112 * kg, L::kIn, bc - 64);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int kt = w + 4 * u;
      if (kt < 7)
        for (int s = 0; s < bc / 4; ++s)
          acc[u] = mfma4(dh1s[(4 * s + g) * 16 + m], xs[(4 * s + g) * 112 + 16 * kt + m], acc[u]);
    }
    if (kg == 0 && tid < 16)
      for (int b = 0; b < bc; b += 4)
#pragma unroll
        for (int k = 0; k < 4; ++k) s1[k] += dh1s[(b + k) * 16 + tid];
  }
  const AdamC ac = adam_consts(f, ain);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int kt = w + 4 * u;
    if (kt >= 7) continue;
    const int k = 112 * kg + 16 * kt + m;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = 16 * nt + 4 * g + r;
      if (n < L::kH) {
        const size_t e = L::w1 + (size_t)n * L::kIn + k;
        if (f.fused_adam) {
          adam_upd(pv[u][r], mv[u][r], vv[u][r], acc[u][r], ac);
          f.m[e] = mv[u][r];
          f.v[e] = vv[u][r];
          f.p[e] = pv[u][r];
        } else {
          f.g[e] = acc[u][r];
        }
      }
    }
  }
  if (kg == 0 && tid < 16 && 16 * nt + tid < L::kH) {
    const size_t e = L::b1 + 16 * nt + tid;
    apply_grad(f, e, f.p[e], (s1[0] + s1[1]) + (s1[2] + s1[3]), ac);
  }
}

size_t bwd2_lds(int Bp) {
  const size_t bc = Bp < kBC2 ? Bp : kBC2;
  return sizeof(float) * (bc * kDhP + kRS * 16 + bc * 16);
}
size_t bwd1_lds(int Bp, bool w2) {
  const size_t bc = Bp < kBC1 ? Bp : kBC1, l1 = bc * 16 + bc * 112, w2b = w2 ? kBCW * (kDhP + 16) : 0;
  return sizeof(float) * (l1 > w2b ? l1 : w2b);
}

}  // namespace
}  // namespace mlp

using namespace mlp;

static void check(const MlpFused& f) {
  MX_CHECK(f.B >= 1 && f.B <= kMlpMaxBatch && f.Bp == (f.B + 15) / 16 * 16,
           "fused MLP engine: 1 <= batch <= 512, Bp = batch rounded up to 16");
}

void mlp_fused_forward(const MlpFused& f, hipStream_t st) {
  check(f);
  const dim3 grid((f.Bp / 16) * kNT);
  if (f.synth)
    MX_LAUNCH((fwd_kernel<MlpLayout::kIn, true>), grid, dim3(256), 0, st, f);
  else
    MX_LAUNCH((fwd_kernel<MlpLayout::kIn, false>), grid, dim3(256), 0, st, f);
  MX_LAUNCH((fwd_kernel<MlpLayout::kH, false>), grid, dim3(256), 0, st, f);
  MX_LAUNCH(head_kernel, dim3((f.Bp / 16) * 8), dim3(256), 0, st, f);
}

void mlp_fused_backward2(const MlpFused& f, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    MX_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(bwd2_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  MX_LAUNCH(bwd2_kernel, dim3(kK4A + kK4L3), dim3(256), bwd2_lds(f.Bp), st, f);
}

void mlp_fused_backward1(const MlpFused& f, hipStream_t st) {
  static bool attr = false;
  if (!attr) {  // B = 512: the l1 blocks stage 256 rows (128 KB)
    MX_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(bwd1_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  MX_LAUNCH(bwd1_kernel, dim3(kNT * 7 + (f.w2_defer ? kK4A : 0)), dim3(256), bwd1_lds(f.Bp, f.w2_defer != 0), st, f);
}

static int g_w2_defer = 0;  // measured: K4 doing the dW2 tile is faster (docs/ROUND6.md)
void mlp_set_w2_defer(int on) { g_w2_defer = on ? 1 : 0; }
int mlp_w2_defer() { return g_w2_defer; }

}  // namespace mx
