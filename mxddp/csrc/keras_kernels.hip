// Fused gfx950 training step of the reference's TF2 Keras CNN (tensorflow2/mnist_single.py:16-26,
// trained with Keras Adam: :78) -- the model of the MirroredStrategy config (BASELINE config 4).
//
// Four launches per step (five with gradient collectives), every one over the whole batch:
//   KF1  on-device batch + conv1 + ReLU + max-pool (VALU, one 28x28 image per block) + conv2 as
//        an MFMA implicit GEMM whose M order puts each 2x2 pool window in one lane's four
//        accumulators, so bias, ReLU, max-pool and argmax happen in registers
//        (block = image x 16 output channels; 4B blocks)
//   KF2  conv3 + ReLU + fc1 + ReLU + fc2 + softmax-CE + accuracy, and the whole activation
//        backward of that head down to the pooled conv2 output (conv3 data gradient, ReLU mask):
//        everything per image lives in LDS (block = image)
//   KB1  the rest of the backward in ONE heterogeneous launch:
//          A  conv2 data gradient on MFMA (dY2 expanded on the fly from its compact pooled form
//             [co][window] + argmax code: 1 compare + 1 select per operand element) -> pool1 /
//             ReLU1 backward -> conv1 weight / bias gradient (block = image x 16 ci x M quarter)
//          B  conv2 weight gradient on MFMA (block = image x 16 co)
//          C  conv3 + fc1 weight gradients (block = 8 images x N quarter)
//          E  fc2 weight gradient
//        weight gradients go to per-image / per-group partial planes with plain stores: no
//        float atomics, deterministic
//   KO   finalize (each gradient = its planes summed in a fixed order) + Adam + repack of the
//        conv2 weights into the MFMA fragment orders of KF1 / KB1 for the next step
//        (with gradient collectives: finalize -> bucket all-reduce -> Adam)
//
// MFMA = v_mfma_f32_16x16x4_f32 (exact fp32): lane l supplies A[l&15][k=l>>4] and
// B[k=l>>4][l&15]; the C tile has col = l&15, row = 4*(l>>4) + reg.
//
// Replaces (reference): the TF2 / Keras graph of Conv2D / MaxPooling2D / Dense /
// sparse_categorical_crossentropy / Adam kernels run per replica by MirroredStrategy
// (tensorflow2/mnist_mirror_strategy.py:12,68-79).
#include "common.h"
#include "keras_kernels.h"
#include "peer_device.h"

#include <cstdlib>
#include "rng.h"

namespace mx {
namespace keras {

using L = KerasLayout;

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// element k of a float4 register array (k compile-time after unrolling: no address taken, so
// the array stays in registers)
__device__ __forceinline__ float f4_at(const float4* a, int k) {
  const float4 v = a[k >> 2];
  return (k & 3) == 0 ? v.x : (k & 3) == 1 ? v.y : (k & 3) == 2 ? v.z : v.w;
}

constexpr int kP1 = 169;          // 13 x 13 pooled conv1 positions
constexpr int kP1Img = 32 * kP1;  // 5408 floats per image
constexpr int kP2Img = 64 * 25;   // 1600
constexpr int kPl2 = 64 * 288;    // conv2 weights
constexpr int kPl3 = 64 * 576;    // conv3 / fc1 weights

// ------------------------------------------------------------------------------------------
// KF1: block = (image n, conv2 output channels 16*c4 .. 16*c4+15), 8 waves.
// conv2 GEMM: M = the 100 conv2 outputs that feed pool2 (rows / cols 0..9; MaxPool2D drops the
// 11th), window-major: m = 4*window + 2*dy + dx (7 M-tiles, rows 100..111 dummy); N = 16 co;
// K = 288 ordered k = r*32 + ci so the im2col LDS offset = per-lane base + compile-time
// immediate.  The 72 B fragments (pre-packed w2f) sit in registers.
__global__ __launch_bounds__(512) void kf1_kernel(KerasFused f) {
  const int n = blockIdx.x >> 2, c4 = blockIdx.x & 3;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  // commit the previous update's Adam step count (see ko_kernel): no KO runs concurrently
  if (blockIdx.x == 0 && tid == 0) {
    const int s1 = __hip_atomic_load(f.adam_state + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (s1 > __hip_atomic_load(f.adam_state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      __hip_atomic_store(f.adam_state, s1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __shared__ float xs[784];
  __shared__ float w1s[320];
  __shared__ float p1s[kP1Img];
  // Stage-1 operands in ONE round trip (counter, conv1 weights, the image row-group of all 10
  // class templates -- the label picks one arithmetically -- or the caller's x), then the 72 conv2
  // B fragments, which stay in flight through conv1 (vmcnt counts in order: they are issued
  // last so waiting for the stage-1 operands never waits for them).  Branch-free in f.synth.
  const int t196 = min(tid, 195), d = 4 * t196;
  const uint32_t ctr = (uint32_t)*f.counter;
  float4 tv[10];
#pragma unroll
  for (int c = 0; c < 10; ++c) tv[c] = *reinterpret_cast<const float4*>(f.tmpl + c * 784 + d);
  const float4 xv = *reinterpret_cast<const float4*>(f.x + (size_t)n * 784 + d);
  const float w1v = f.p[L::w1 + min(tid, 319)];
  __builtin_amdgcn_sched_barrier(0);  // issue order: stage-1 operands, then the fragments
  float breg[72];
  const float* wf = f.w2f + (size_t)c4 * 72 * 64;
#pragma unroll
  for (int s = 0; s < 72; ++s) breg[s] = wf[s * 64 + lane];
  __builtin_amdgcn_sched_barrier(0);
  {
    const uint2 key = synth_key(f.seed);
    const int label = synth_label(ctr, n, 10, key);
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);  // masked sum (a select chain becomes tv[label])
#pragma unroll
    for (int c = 0; c < 10; ++c) {
      const float mk = (float)(label == c);
      t.x = fmaf(mk, tv[c].x, t.x);
      t.y = fmaf(mk, tv[c].y, t.y);
      t.z = fmaf(mk, tv[c].z, t.z);
      t.w = fmaf(mk, tv[c].w, t.w);
    }
    const uint4 r = synth_noise4(ctr, n, d, key);
    const float4 sv = make_float4(0.5f * t.x + 0.5f * u01(r.x), 0.5f * t.y + 0.5f * u01(r.y),
                                  0.5f * t.z + 0.5f * u01(r.z), 0.5f * t.w + 0.5f * u01(r.w));
    const float4 v = f.synth ? sv : xv;
    if (tid < 196) {
      *reinterpret_cast<float4*>(xs + d) = v;
      if (f.synth && c4 == 0) *reinterpret_cast<float4*>(f.x + (size_t)n * 784 + d) = v;
    }
    if (f.synth && c4 == 0 && tid == 0) f.y[n] = label;
  }
  if (tid < 320) w1s[tid] = w1v;  // w1 [32][9] then b1 [32]
  lds_barrier();  // (x / label stores are read by later kernels only)

  // conv1 + ReLU + 2x2 max-pool (+ argmax): 32 x 169 pooled outputs, one 4x4 input patch each
  for (int o = tid; o < kP1Img; o += 512) {
    const int ci = o / kP1, pp = o - ci * kP1, py = pp / 13, px = pp - py * 13;
    const float* xp = xs + (2 * py) * 28 + 2 * px;
    float pt[16];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) pt[a * 4 + b] = xp[a * 28 + b];
    const float* wc = w1s + ci * 9;
    float wr[9];
#pragma unroll
    for (int r = 0; r < 9; ++r) wr[r] = wc[r];
    const float bias = w1s[288 + ci];
    float bz = 0.f;
    int best = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int dy = j >> 1, dx = j & 1;
      float z = bias;
#pragma unroll
      for (int r = 0; r < 9; ++r) z += wr[r] * pt[(dy + r / 3) * 4 + dx + r % 3];
      if (j == 0 || z > bz) {
        bz = z;
        best = j;
      }
    }
    const float v = fmaxf(bz, 0.f);
    p1s[o] = v;
    if (c4 == 0) {
      f.p1[(size_t)n * kP1Img + o] = v;
      f.q1[(size_t)n * kP1Img + o] = (uint8_t)best;
    }
  }
  lds_barrier();  // the published p1 / q1 are read by KB1, not by this block

  // conv2 (16 co of this block) on MFMA (B fragments in flight since the start)
  const int co = 16 * c4 + (lane & 15);
  const float bias2 = f.p[L::b2 + co];
  for (int mt = w; mt < 7; mt += 8) {  // 7 M-tiles over 8 waves
    const int ml = lane & 15, win = 4 * mt + (ml >> 2);
    int base = 0;
    if (win < 25) {
      const int wy = win / 5, wx = win - wy * 5;
      base = (2 * wy + ((ml >> 1) & 1)) * 13 + 2 * wx + (ml & 1);
    }
    const float* ap = p1s + base + g * kP1;
    // two accumulator chains (even / odd k-steps): one chain made each MFMA wait for the last
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 72; ++s) {
      const int r = s >> 3;
      const float a = ap[(4 * (s & 7)) * kP1 + (r / 3) * 13 + (r % 3)];
      if (s & 1) acc1 = mfma4(a, breg[s], acc1);
      else acc0 = mfma4(a, breg[s], acc0);
    }
    const f32x4 acc = acc0 + acc1;
    const int wo = 4 * mt + g;  // this lane's accumulators = the 4 outputs of window wo, channel co
    if (wo < 25) {
      int best = 0;
      float bz = acc[0];
#pragma unroll
      for (int j = 1; j < 4; ++j)
        if (acc[j] > bz) {
          bz = acc[j];
          best = j;
        }
      const size_t o = ((size_t)n * 64 + co) * 25 + wo;
      f.p2[o] = fmaxf(bz + bias2, 0.f);
      f.q2[o] = (uint8_t)best;
    }
  }
}

// ------------------------------------------------------------------------------------------
// KF2: block = image, 8 waves.  Head forward + backward to the pooled conv2 output; VALU,
// LDS-resident.  The phases are a dependent chain, so no phase waits on a global load of its own:
// group 1 (entry) = conv3 / fc1 slices, the pooled input, biases, the fc2 operands of the loss
// and dh1; group 2 (issued after fc1, in flight during the loss) = the fc1-transpose column(s)
// for dx3; group 3 = the conv3 data-gradient slice, one tap row ahead of its use.  vmcnt counts in order, so a phase that needed a
// group-1 value after group 2 was issued would wait for all of group 2 -- every group-1 operand
// is therefore consumed or copied to registers before group 2 starts.  Barriers that follow
// this block's global stores (x3, dl, dh1, dx3, ... for KB1) are LDS-only (no store drain).
__global__ __launch_bounds__(512) void kf2_kernel(KerasFused f) {
  const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  __shared__ float p2s[kP2Img];
  __shared__ float x3s[576];
  __shared__ float dx3s[576];
  __shared__ float hs[64];
  __shared__ float dh1s[64];
  __shared__ float dls[16];
  __shared__ float red2[8][64];  // dx3 inputs 512..575: partial sums over 8 feature groups
  __shared__ float w2s[640];     // fc2 weights [10][64]
  __shared__ float bss[138];     // conv3 bias, fc1 bias, fc2 bias
  const int hi = tid >> 3, q = tid & 7;  // (output channel / feature, eighth of the reduction)
  // ---- group 1
  // conv3 slice w3[hi][8q .. 8q+7][9] and fc1 slice fw1[hi][72q .. 72q+71]: 18 float4 each
  float4 wc[18], wf[18];
  {
    const float4* a = reinterpret_cast<const float4*>(f.p + L::w3 + ((size_t)hi * 64 + 8 * q) * 9);
    const float4* b = reinterpret_cast<const float4*>(f.p + L::fw1 + (size_t)hi * 576 + 72 * q);
#pragma unroll
    for (int k = 0; k < 18; ++k) {
      wc[k] = a[k];
      wf[k] = b[k];
    }
  }
  float p2v[4];  // 1600 floats = 3 x 512 + 64
#pragma unroll
  for (int k = 0; k < 4; ++k) p2v[k] = f.p2[(size_t)n * kP2Img + min(tid + 512 * k, kP2Img - 1)];
  // the small operands of the later phases go to LDS with the input (registers are needed by the
  // conv3 / fc1 slices): fc2 weights [10][64], biases b3 / fb1 / fb2, the label
  const float w2v0 = f.p[L::fw2 + tid], w2v1 = f.p[L::fw2 + min(512 + tid, 639)];
  const float bv = f.p[(tid < 64 ? L::b3 : tid < 128 ? L::fb1 : L::fb2) + min(tid & 63, tid < 128 ? 63 : 9)];
  const int label = f.y[n];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (tid + 512 * k < kP2Img) p2s[tid + 512 * k] = p2v[k];
  w2s[tid] = w2v0;
  if (tid < 128) w2s[512 + tid] = w2v1;
  if (tid < 138) bss[tid] = bv;  // b3 [0, 64), fb1 [64, 128), fb2 [128, 138)
  if (f.synth && n == 0 && tid == 0) *f.counter += 1;  // KF1 consumed this batch index
  __syncthreads();

  // conv3 + bias + ReLU: thread (co = hi, ci 8q..8q+7) -> all 9 outputs of co, xor-tree over q
  {
    float acc[9];
#pragma unroll
    for (int pos = 0; pos < 9; ++pos) acc[pos] = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const float* pc = p2s + (8 * q + c) * 25;
      float pt[25];
#pragma unroll
      for (int k = 0; k < 25; ++k) pt[k] = pc[k];
#pragma unroll
      for (int pos = 0; pos < 9; ++pos)
#pragma unroll
        for (int r = 0; r < 9; ++r) acc[pos] += f4_at(wc, c * 9 + r) * pt[(pos / 3 + r / 3) * 5 + pos % 3 + r % 3];
    }
#pragma unroll
    for (int pos = 0; pos < 9; ++pos)
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) acc[pos] += __shfl_xor(acc[pos], o, 64);
    if (q == 0) {
#pragma unroll
      for (int pos = 0; pos < 9; ++pos) x3s[hi * 9 + pos] = fmaxf(acc[pos] + bss[hi], 0.f);
    }
  }
  __syncthreads();

  for (int i = tid; i < 576; i += 512) f.x3[(size_t)n * 576 + i] = x3s[i];

  // fc1 + bias + ReLU: thread (j = hi, inputs 72q .. 72q+71)
  {
    const float4* xr = reinterpret_cast<const float4*>(x3s + 72 * q);
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < 18; ++k) {
      const float4 xv = xr[k];
      a += wf[k].x * xv.x + wf[k].y * xv.y + wf[k].z * xv.z + wf[k].w * xv.w;
    }
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) a += __shfl_xor(a, o, 64);
    if (q == 0) hs[hi] = fmaxf(a + bss[64 + hi], 0.f);
  }
  lds_barrier();
  // ---- group 2 (in flight during the loss): fc1-transpose column fw1[:, tid] for dx3 input
  // tid; for inputs 512..575 thread t takes input 512 + (t & 63) over features 8 (t >> 6) .. +7
  // (8 registers, not a second 64-entry column); conv3 data-gradient slice w3[8q + c][hi][9]
  float wx[64], wx2[8];
#pragma unroll
  for (int j = 0; j < 64; ++j) wx[j] = f.p[L::fw1 + (size_t)j * 576 + tid];
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) wx2[jj] = f.p[L::fw1 + (size_t)(8 * wv + jj) * 576 + 512 + lane];

  // fc2 + softmax + cross entropy + accuracy + dlogits (wave 0)
  if (wv == 0) {
    float a = 0.f;
    if (lane < 40) {
      const int c = lane >> 2, qq = lane & 3;
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) a += w2s[c * 64 + 16 * qq + jj] * hs[16 * qq + jj];
    }
    a += __shfl_xor(a, 1, 64);
    a += __shfl_xor(a, 2, 64);
    const float lg0 = __shfl(a, 4 * (lane < 10 ? lane : 0), 64);
    const float lg = lane < 10 ? lg0 + bss[128 + lane] : -INFINITY;
    const float mx = wave_max(lg);
    const float ex = lane < 10 ? __expf(lg - mx) : 0.f;
    const float se = wave_sum(ex);
    const float lbl = __shfl(lg, label, 64);
    const unsigned long long ball = __ballot(lane < 10 && lg == mx);
    const int first = __ffsll((long long)ball) - 1;
    if (lane < 10) {
      const float d = (ex / se - (lane == label ? 1.f : 0.f)) / (float)f.B;
      dls[lane] = d;
      f.dl[(size_t)n * 16 + lane] = d;
      f.sv[(size_t)n * 256 + 192 + lane] = d;
    }
    if (lane == 0) {
      atomicAdd(f.metrics, mx + __logf(se) - lbl);
      atomicAdd(f.metrics + 1, first == label ? 1.f : 0.f);
    }
  }
  lds_barrier();
  // dh1 = (fw2^T dl) * (h > 0)
  if (tid < 64) {
    float a = 0.f;
#pragma unroll
    for (int c = 0; c < 10; ++c) a += w2s[c * 64 + tid] * dls[c];
    const float d = hs[tid] > 0.f ? a : 0.f;
    dh1s[tid] = d;
    f.dh1[(size_t)n * 64 + tid] = d;
    f.h1[(size_t)n * 64 + tid] = hs[tid];
    f.sv[(size_t)n * 256 + 128 + tid] = d;
  }
  lds_barrier();
  // dx3 = (fw1^T dh1) * (x3 > 0): inputs tid (and 512 + tid for the first wave)
  {
    float a0 = 0.f, a1 = 0.f;
#pragma unroll
    for (int j = 0; j < 64; j += 2) {
      a0 += wx[j] * dh1s[j];
      a1 += wx[j + 1] * dh1s[j + 1];
    }
    const float d = x3s[tid] > 0.f ? a0 + a1 : 0.f;
    dx3s[tid] = d;
    f.dx3[(size_t)n * 576 + tid] = d;
    float b0 = 0.f;
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) b0 += wx2[jj] * dh1s[8 * wv + jj];
    red2[wv][lane] = b0;
  }
  // group 3 (the fc1 column is consumed): the first tap row of the conv3 data-gradient slice
  // w3[8q][hi][9], in flight during the remaining dx3 / bias-gradient steps; the other 7 are
  // prefetched one step ahead inside the loop (all 72 in registers spilled: 292 B/lane)
  float wn[9];
#pragma unroll
  for (int r = 0; r < 9; ++r) wn[r] = f.p[L::w3 + ((size_t)(8 * q) * 64 + hi) * 9 + r];
  lds_barrier();
  if (tid < 64) {  // inputs 512..575: the 8 feature-group partials in a fixed order
    float b0 = red2[0][tid];
#pragma unroll
    for (int k = 1; k < 8; ++k) b0 += red2[k][tid];
    const int i2 = 512 + tid;
    const float d2 = x3s[i2] > 0.f ? b0 : 0.f;
    dx3s[i2] = d2;
    f.dx3[(size_t)n * 576 + i2] = d2;
  }
  lds_barrier();
  if (tid < 64) {  // conv3 bias grad of this image
    float sb = 0.f;
#pragma unroll
    for (int pos = 0; pos < 9; ++pos) sb += dx3s[tid * 9 + pos];
    f.sv[(size_t)n * 256 + 64 + tid] = sb;
  }
  // conv3 data gradient -> dp2 (ReLU-masked with p2 > 0) + conv2 bias grad:
  // thread (ci = hi, co 8q .. 8q+7) scatters into 25 registers, xor-tree over q
  {
    float acc[25];
#pragma unroll
    for (int k = 0; k < 25; ++k) acc[k] = 0.f;
#pragma unroll 1
    for (int c = 0; c < 8; ++c) {
      const int co = 8 * q + c;
      float w[9], d[9];
#pragma unroll
      for (int r = 0; r < 9; ++r) w[r] = wn[r];
      if (c + 1 < 8) {
#pragma unroll
        for (int r = 0; r < 9; ++r) wn[r] = f.p[L::w3 + ((size_t)(co + 1) * 64 + hi) * 9 + r];
      }
#pragma unroll
      for (int pos = 0; pos < 9; ++pos) d[pos] = dx3s[co * 9 + pos];
#pragma unroll
      for (int pos = 0; pos < 9; ++pos)
#pragma unroll
        for (int r = 0; r < 9; ++r) acc[(pos / 3 + r / 3) * 5 + pos % 3 + r % 3] += d[pos] * w[r];
    }
#pragma unroll
    for (int k = 0; k < 25; ++k)
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) acc[k] += __shfl_xor(acc[k], o, 64);
    if (q == 0) {
      float sb = 0.f;
#pragma unroll
      for (int k = 0; k < 25; ++k) {
        const float v = p2s[hi * 25 + k] > 0.f ? acc[k] : 0.f;
        f.dp2[((size_t)n * 64 + hi) * 25 + k] = v;
        sb += v;
      }
      f.sv[(size_t)n * 256 + hi] = sb;
    }
  }
}

// ------------------------------------------------------------------------------------------
// KB1 role A: conv2 data gradient dP1[ci][y][x] = sum_{co,ky,kx} dY2[co][y-ky][x-kx] w2[co][ci][ky][kx]
// on MFMA: M = the 169 pooled conv1 positions (11 tiles; this block: M quarter mq = 3 tiles, the
// last 2), N = 16 ci (ci half nh), K = 576 = (tap r, co) split over the 4 waves by co (wave w:
// co 16w..16w+15, 36 k-steps: r = s/4, co = 16w + 4(s%4) + lane group).  dY2 lives compact in LDS
// as [co][8][8] pool windows (a dead ring of windows around the 5x5, so no bounds checks) + the
// argmax code; an operand element is (code == its parity) ? value : 0.  The 4 waves' partial
// tiles are summed in LDS, then each lane masks with pool1 / ReLU1 (argmax code, p1 > 0) and
// contracts with the 3x3 input patch at the argmax position: conv1 weight / bias grads, reduced
// over lanes and tiles into this block's partial plane.
struct SmemA {
  float dps[64 * 64];
  uint8_t qs[64 * 64];
  float xs[784];
  float red[4][3][4][64];
  float c1[3][16][10];
};
struct SmemB {
  float p1s[kP1Img];
};
struct SmemC {
  float dx3[8][576];
  float p2[8][16][25];
  float dh1[8][64];
  float x3[8][144];
};
struct SmemE {
  float dl[64 * 16];
  float h1[64 * 64];
};
union SmemKB1 {
  SmemA a;
  SmemB b;
  SmemC c;
  SmemE e;
};

__device__ void kb1_role_a(const KerasFused& f, SmemA& sm, int bid) {
  const int n = bid >> 3, nh = (bid >> 2) & 1, mq = bid & 3;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  // Every global operand of the block is requested up front, in one round trip: the B fragments
  // of this wave's 36 k-steps (pre-packed w2d), the input image, the compact dY2 + argmax codes,
  // and the pool1 / ReLU1 operands of the epilogue (clamped lanes, no loads behind branches).
  float breg[36];
  const float* wd = f.w2d + ((size_t)(nh * 4 + w) * 36) * 64;
#pragma unroll
  for (int s = 0; s < 36; ++s) breg[s] = wd[s * 64 + lane];
  float xv[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) xv[k] = f.x[(size_t)n * 784 + min(tid + 256 * k, 783)];
  float dv[7];
  uint8_t qv[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const int e = min(tid + 256 * k, kP2Img - 1);
    dv[k] = f.dp2[(size_t)n * kP2Img + e];
    qv[k] = f.q2[(size_t)n * kP2Img + e];
  }
  const int t0 = 3 * mq, nt = mq == 3 ? 2 : 3;
  float p1v[4];
  uint8_t q1v[4];
  {
    const int ci = 16 * nh + (lane & 15);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = min(16 * (t0 + min(w, nt - 1)) + 4 * g + j, kP1 - 1);
      const size_t pi = ((size_t)n * 32 + ci) * kP1 + m;
      p1v[j] = f.p1[pi];
      q1v[j] = f.q1[pi];
    }
  }
  // dY2 windows [co][8][8] with a dead ring: the ring is zeroed, the 5 x 5 interior scattered
  // (disjoint entries: one barrier)
  for (int i = tid; i < 64 * 64; i += 256) {
    const int wy = (i >> 3) & 7, wx = i & 7;
    if (wy < 1 || wy > 5 || wx < 1 || wx > 5) {
      sm.dps[i] = 0.f;
      sm.qs[i] = 0;
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (tid + 256 * k < 784) sm.xs[tid + 256 * k] = xv[k];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const int e = tid + 256 * k;
    if (e < kP2Img) {
      const int co = e / 25, wi = e - co * 25, wy = wi / 5, wx = wi - wy * 5;
      const int idx = co * 64 + (wy + 1) * 8 + wx + 1;
      sm.dps[idx] = dv[k];
      sm.qs[idx] = qv[k];
    }
  }
  // per tile, per tap: window offset [8x8 grid] and the argmax code dY2's position must match
  int off[3][9], code[3][9];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    int m = 16 * (t0 + t) + (lane & 15);
    if (t >= nt || m >= kP1) m = 0;
    const int y = m / 13, x = m - y * 13;
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      const int oy = y - r / 3, ox = x - r % 3;
      off[t][r] = ((oy + 2) >> 1) * 8 + ((ox + 2) >> 1);
      code[t][r] = (oy & 1) * 2 + (ox & 1);
    }
  }
  __syncthreads();
  const int lbase = (16 * w + g) * 64;
  f32x4 acc[3] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  // The (value, code) pairs of k-step s + 1 are read while k-step s's MFMAs run, both loads
  // unconditional: written as `code == c ? dps[idx] : 0` the value load sat behind the code
  // load's wait, and every MFMA behind two dependent LDS round trips (the ISA: ds_read_u8,
  // lgkmcnt(0), ds_read_b32, lgkmcnt(0), v_mfma).
  float dn[3];
  int qn[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int idx = lbase + off[t][0];
    dn[t] = sm.dps[idx];
    qn[t] = sm.qs[idx];
  }
#pragma unroll
  for (int s = 0; s < 36; ++s) {
    const int r = s >> 2;
    float dc[3];
    int qc[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      dc[t] = dn[t];
      qc[t] = qn[t];
    }
    if (s + 1 < 36) {
      const int r1 = (s + 1) >> 2, cofs1 = 4 * ((s + 1) & 3) * 64;
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const int idx = lbase + cofs1 + off[t][r1];
        dn[t] = sm.dps[idx];
        qn[t] = sm.qs[idx];
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < 3; ++t) acc[t] = mfma4(qc[t] == code[t][r] ? dc[t] : 0.f, breg[s], acc[t]);
  }
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) sm.red[w][t][j][lane] = acc[t][j];
  __syncthreads();
  if (w < nt) {  // wave w finishes tile t0 + w
    const int t = w, ci_l = lane & 15, ci = 16 * nh + ci_l;
    float cw[9], cb = 0.f;
#pragma unroll
    for (int r = 0; r < 9; ++r) cw[r] = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = 16 * (t0 + t) + 4 * g + j;
      if (m < kP1) {
        const float d = sm.red[0][t][j][lane] + sm.red[1][t][j][lane] + sm.red[2][t][j][lane] + sm.red[3][t][j][lane];
        if (p1v[j] > 0.f) {
          const int cd = q1v[j];
          const int y1 = 2 * (m / 13) + (cd >> 1), x1 = 2 * (m % 13) + (cd & 1);
#pragma unroll
          for (int r = 0; r < 9; ++r) cw[r] += d * sm.xs[(y1 + r / 3) * 28 + x1 + r % 3];
          cb += d;
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      cw[r] += __shfl_xor(cw[r], 16, 64);
      cw[r] += __shfl_xor(cw[r], 32, 64);
    }
    cb += __shfl_xor(cb, 16, 64);
    cb += __shfl_xor(cb, 32, 64);
    if (g == 0) {
#pragma unroll
      for (int r = 0; r < 9; ++r) sm.c1[t][ci_l][r] = cw[r];
      sm.c1[t][ci_l][9] = cb;
    }
  }
  __syncthreads();
  if (tid < 160) {
    const int ci_l = tid / 10, k = tid - ci_l * 10, ci = 16 * nh + ci_l;
    float s = 0.f;
    for (int t = 0; t < nt; ++t) s += sm.c1[t][ci_l][k];
    float* plane = f.pl1 + ((size_t)n * 4 + mq) * 320;
    if (k < 9) plane[ci * 9 + k] = s;
    else plane[288 + ci] = s;
  }
}

// role B: conv2 weight gradient of image n for co 16cq..16cq+15: M = 16 co, N = 288 (ci, tap) in
// 18 tiles (wave w: tiles w, w+4, ...), K = the 100 conv2 outputs that feed pool2 (25 k-steps).
// The A operand (expanded dY2) of a lane is the same for every N tile: 25 registers built once.
__device__ void kb1_role_b(const KerasFused& f, SmemB& sm, int bid) {
  const int n = bid >> 2, cq = bid & 3;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  // the pooled conv1 tile (1352 float4: 6 per thread, clamped) and the A operands below are
  // all requested before anything is stored (one round trip)
  constexpr int kP1v = kP1Img / 4, kP1n = (kP1v + 255) / 256;
  float4 pv[kP1n];
#pragma unroll
  for (int k = 0; k < kP1n; ++k)
    pv[k] = reinterpret_cast<const float4*>(f.p1 + (size_t)n * kP1Img)[min(tid + 256 * k, kP1v - 1)];
  const int co_a = 16 * cq + (lane & 15);
  float av[25];
  int poff[25];
#pragma unroll
  for (int s = 0; s < 25; ++s) {
    const int pos = 4 * s + g, oy = pos / 10, ox = pos - oy * 10;
    const size_t e = ((size_t)n * 64 + co_a) * 25 + (oy >> 1) * 5 + (ox >> 1);
    const float dv = f.dp2[e];
    av[s] = (int)f.q2[e] == (oy & 1) * 2 + (ox & 1) ? dv : 0.f;
    poff[s] = oy * 13 + ox;
  }
  // clamped, not predicated (a predicated store let the compiler sink each load into its
  // store's branch: one memory round trip per float4); past the end: element kP1v - 1 again
#pragma unroll
  for (int k = 0; k < kP1n; ++k) reinterpret_cast<float4*>(sm.p1s)[min(tid + 256 * k, kP1v - 1)] = pv[k];
  __syncthreads();
  for (int nt = w; nt < 18; nt += 4) {
    const int c = 16 * nt + (lane & 15), ci = c / 9, r = c - ci * 9;
    const float* bp = sm.p1s + ci * kP1 + (r / 3) * 13 + r % 3;
    // two accumulator chains (even / odd k-steps): one chain made each MFMA wait for the last
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 25; ++s) {
      if (s & 1) acc1 = mfma4(av[s], bp[poff[s]], acc1);
      else acc0 = mfma4(av[s], bp[poff[s]], acc0);
    }
    float* plane = f.pl2 + (size_t)n * kPl2;
#pragma unroll
    for (int j = 0; j < 4; ++j) plane[(16 * cq + 4 * g + j) * 288 + c] = acc0[j] + acc1[j];
  }
}

// role C: conv3 + fc1 weight gradients of an 8-image group gi, quarter nq of the input columns
__device__ void kb1_role_c(const KerasFused& f, SmemC& sm, int bid) {
  const int gi = bid >> 2, nq = bid & 3, tid = threadIdx.x;
  const int n0 = 8 * gi;
  // all four operand tiles requested before any LDS store (one round trip, clamped lanes)
  float vdx[18], vp2[13], vdh[2], vx3[5];
#pragma unroll
  for (int k = 0; k < 18; ++k) vdx[k] = f.dx3[(size_t)n0 * 576 + tid + 256 * k];  // 4608 = 18 x 256
#pragma unroll
  for (int k = 0; k < 13; ++k) {
    const int i = min(tid + 256 * k, 8 * 16 * 25 - 1), im = i / 400, rem = i - im * 400;
    vp2[k] = f.p2[((size_t)(n0 + im) * 64 + 16 * nq) * 25 + rem];
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) vdh[k] = f.dh1[(size_t)n0 * 64 + tid + 256 * k];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const int i = min(tid + 256 * k, 8 * 144 - 1);
    vx3[k] = f.x3[(size_t)(n0 + i / 144) * 576 + 144 * nq + i % 144];
  }
#pragma unroll
  for (int k = 0; k < 18; ++k) {
    const int i = tid + 256 * k;
    sm.dx3[i / 576][i % 576] = vdx[k];
  }
#pragma unroll
  for (int k = 0; k < 13; ++k) {
    const int i = tid + 256 * k, im = i / 400, rem = i - im * 400;
    if (i < 8 * 16 * 25) sm.p2[im][rem / 25][rem % 25] = vp2[k];
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = tid + 256 * k;
    sm.dh1[i / 64][i % 64] = vdh[k];
  }
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const int i = tid + 256 * k;
    if (i < 8 * 144) sm.x3[i / 144][i % 144] = vx3[k];
  }
  __syncthreads();
  {  // conv3: thread (co, 4 ci of the block's 16) -> 36 weights
    const int co = tid >> 2, cq = tid & 3;
    float acc[4][9];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int r = 0; r < 9; ++r) acc[c][r] = 0.f;
    for (int im = 0; im < 8; ++im) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float pt[25];
#pragma unroll
        for (int k = 0; k < 25; ++k) pt[k] = sm.p2[im][4 * cq + c][k];
#pragma unroll
        for (int pos = 0; pos < 9; ++pos) {
          const float d = sm.dx3[im][co * 9 + pos];
#pragma unroll
          for (int r = 0; r < 9; ++r) acc[c][r] += d * pt[(pos / 3 + r / 3) * 5 + pos % 3 + r % 3];
        }
      }
    }
    float* plane = f.pl3 + (size_t)gi * kPl3 + (size_t)co * 576 + (16 * nq + 4 * cq) * 9;
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int r = 0; r < 9; ++r) plane[c * 9 + r] = acc[c][r];
  }
  {  // fc1: thread (j, 36 of the block's 144 inputs)
    const int j = tid >> 2, q = tid & 3;
    float acc[36];
#pragma unroll
    for (int i = 0; i < 36; ++i) acc[i] = 0.f;
    for (int im = 0; im < 8; ++im) {
      const float h = sm.dh1[im][j];
#pragma unroll
      for (int i = 0; i < 36; ++i) acc[i] += h * sm.x3[im][36 * q + i];
    }
    float* plane = f.pf1 + (size_t)gi * kPl3 + (size_t)j * 576 + 144 * nq + 36 * q;
#pragma unroll
    for (int i = 0; i < 36; ++i) plane[i] = acc[i];
  }
}

// role E: fc2 weight gradient = sum over the batch of dl (x) h1, staged through LDS 64 images at a
// time (coalesced loads; the products then come from LDS, not from dependent global loads)
__device__ void kb1_role_e(const KerasFused& f, SmemE& sm) {
  const int tid = threadIdx.x;
  float acc[3] = {0.f, 0.f, 0.f};  // outputs tid, tid + 256, tid + 512 (< 640)
  for (int n0 = 0; n0 < f.B; n0 += 64) {
    const int nb = f.B - n0 < 64 ? f.B - n0 : 64;
    __syncthreads();
    {  // dl [nb][16] + h1 [nb][64] as float4s, all five of a thread's loads before its stores (a
       // scalar `load; store` loop was 20 serial memory round trips); clamped, not predicated:
       // past the end a thread rewrites the last float4
      const int n4d = nb * 4, n4h = nb * 16;
      const float4* dsrc = reinterpret_cast<const float4*>(f.dl + (size_t)n0 * 16);
      const float4* hsrc = reinterpret_cast<const float4*>(f.h1 + (size_t)n0 * 64);
      const int id = min(tid, n4d - 1);
      int ih[4];
      float4 hv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) ih[u] = min(tid + 256 * u, n4h - 1);
      const float4 dv = dsrc[id];
#pragma unroll
      for (int u = 0; u < 4; ++u) hv[u] = hsrc[ih[u]];
      reinterpret_cast<float4*>(sm.dl)[id] = dv;
#pragma unroll
      for (int u = 0; u < 4; ++u) reinterpret_cast<float4*>(sm.h1)[ih[u]] = hv[u];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int o = tid + 256 * k;
      if (o < 640) {
        const int c = o >> 6, j = o & 63;
        float a = 0.f;
        for (int nn = 0; nn < nb; ++nn) a += sm.dl[nn * 16 + c] * sm.h1[nn * 64 + j];
        acc[k] += a;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 3; ++k)
    if (tid + 256 * k < 640) f.gf2[tid + 256 * k] = acc[k];
}

__global__ __launch_bounds__(256) void kb1_kernel(KerasFused f) {
  __shared__ __attribute__((aligned(16))) SmemKB1 sm;
  const int b = blockIdx.x, B = f.B;
  if (b < 8 * B) {
    kb1_role_a(f, sm.a, b);
  } else if (b < 12 * B) {
    kb1_role_b(f, sm.b, b - 8 * B);
  } else if (b < 12 * B + B / 2) {
    kb1_role_c(f, sm.c, b - 12 * B);
  } else {
    kb1_role_e(f, sm.e);
  }
}

struct KoRegion {
  int blk0;          // first block of the region
  int p0, np;        // parameter range
  int T;             // 1: one thread per parameter; 4: the block's 4 waves split the planes
  int nplanes;
  long long stride;  // floats between planes
  const float* src;  // plane 0 of the region's first parameter
};
constexpr int kKoMaxRegions = 10;
struct KoPlan {
  int nreg, nblocks;
  KoRegion r[kKoMaxRegions];
};

// ------------------------------------------------------------------------------------------
// KO: finalize + Adam + repack.  The parameters are split into regions by gradient source (the
// partial planes of each weight, the per-image bias vectors).  A plane-summing region (T = 4)
// gives each block 64 consecutive parameters: wave w sums planes w, w + 4, ... with four
// independent accumulators (each plane read is one coalesced 256-byte row per wave), the four
// wave sums meet in LDS in a fixed order (deterministic), and wave 0 finishes the parameters.
// T = 1 (the all-reduced g, the single fc2 plane): one thread per parameter.
__device__ __forceinline__ void pack_w2(const KerasFused& f, int i, float val) {
  // i in [w2, b2): co, ci, tap r of conv2.weight[co][ci][ky][kx]
  const int j = i - L::w2, co = j / 288, rem = j - co * 288, ci = rem / 9, r = rem - ci * 9;
  // KF1 B: (c4, s, lane): co = 16 c4 + (lane & 15), k = 4s + (lane >> 4) = r*32 + ci
  const int k = r * 32 + ci;
  f.w2f[((co >> 4) * 72 + (k >> 2)) * 64 + (co & 15) + 16 * (k & 3)] = val;
  // KB1-A B: (nh, wave, s, lane): ci = 16 nh + (lane & 15), co = 16 wave + 4 (s%4) + (lane >> 4), r = s/4
  const int cl = co & 15;
  f.w2d[(((ci >> 4) * 4 + (co >> 4)) * 36 + r * 4 + (cl >> 2)) * 64 + (ci & 15) + 16 * (cl & 3)] = val;
}

// Adam (gradient gr already summed / averaged by gscale) + conv2 repack of parameter i
// (p, m, v, lr: the caller's values, loaded before the gradient planes -- loaded here they were
// up to three serial memory round trips after the plane sum)
__device__ __forceinline__ void adam_one(const KerasFused& f, int i, float gr, int t, float gscale, float pv, float m0,
                                         float v0, float lr) {
  gr = gr * gscale + f.wd * pv;
  const float bc1 = 1.f - powf(f.b1, (float)t), bc2 = 1.f - powf(f.b2, (float)t);
  const float bc2s = sqrtf(bc2);
  const float e = f.eps_hat ? f.eps / bc2s : f.eps;
  const float mi = f.b1 * m0 + (1.f - f.b1) * gr;
  const float vi = f.b2 * v0 + (1.f - f.b2) * gr * gr;
  f.m[i] = mi;
  f.v[i] = vi;
  pv -= (lr / bc1) * mi / (sqrtf(vi) / bc2s + e);
  f.p[i] = pv;
  if (i >= (int)L::w2 && i < (int)L::b2) pack_w2(f, i, pv);
}
__device__ __forceinline__ void adam_one(const KerasFused& f, int i, float gr, int t, float gscale) {
  adam_one(f, i, gr, t, gscale, f.p[i], f.m[i], f.v[i], *f.lr);
}

__global__ __launch_bounds__(256) void ko_kernel(KerasFused f, KoPlan plan, int mode, float gscale) {
  __shared__ float red[4][64];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int ri = 0;
#pragma unroll
  for (int k = 1; k < kKoMaxRegions; ++k)
    if (k < plan.nreg && b >= plan.r[k].blk0) ri = k;
  const KoRegion& R = plan.r[ri];
  const int T = R.T;
  const int q = T == 1 ? 0 : w;
  const int li = T == 1 ? (b - R.blk0) * 256 + tid : (b - R.blk0) * 64 + lane;  // index inside the region
  const bool live = li < R.np;
  const int i = R.p0 + li;
  const bool adam = mode == 0 || mode == 2;
  // Adam step count: state[0] = steps committed before this update (read by every block, not
  // written here), state[1] = this update's count, published by block 0 and copied to state[0]
  // by the next step's KF1.  (Each block arriving on one counter to find the last one serialised
  // ~1,450 same-address atomics: most of this kernel's 41 us.)
  int t = 0;
  if (adam) t = __hip_atomic_load(f.adam_state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  float pv = 0.f, m0 = 0.f, v0 = 0.f, lr = 0.f;
  if (adam && q == 0) {  // the update's operands, in flight with the first round of planes
    const int ic = live ? i : R.p0;
    pv = f.p[ic];
    m0 = f.m[ic];
    v0 = f.v[ic];
    lr = *f.lr;
  }
  float gr = 0.f;
  if (mode != 3) {
    // this thread's planes k = q, q + T, ... (fixed order), 8 loads in flight per round
    // (clamped + masked: no load behind a branch); np_t = planes per thread
    const float* src = R.src + (live ? li : 0);
    const long long st = R.stride;
    const int np_t = R.nplanes > q ? (R.nplanes - q + T - 1) / T : 0;
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < np_t; k0 += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = src[(size_t)(q + T * min(k0 + u, np_t - 1)) * st];
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] += k0 + u < np_t ? v[u] : 0.f;
    }
    gr = live ? ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7])) : 0.f;
    if (T > 1) {  // block-uniform branch
      red[w][lane] = gr;
      __syncthreads();
      gr = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    }
  }
  if (live && q == 0) {
    if (mode == 1) f.g[i] = gr;
    else if (adam) adam_one(f, i, gr, t, gscale, pv, m0, v0, lr);
    else if (i >= (int)L::w2 && i < (int)L::b2) pack_w2(f, i, f.p[i]);  // mode 3
  }
  if (adam && b == 0 && tid == 0) __hip_atomic_store(f.adam_state + 1, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------------------------------
// KX: the gradient exchange co-scheduled with Adam (peer transport, world size 2..8): one
// launch replaces the bucket all-reduce kernel and the Adam launch.  Block b owns parameters
// [512 b, 512 b + 512): it pushes its slice of the finalized g into every peer's exchange slot
// `rank` (one-shot: W-1 remote stores per value, all links at once), publishes its per-block
// flag, waits for the peers' flags of the same block (peer_device.h; bounded, no grid barrier),
// sums the W copies in rank order 0..W-1 (bit-identical on every rank) and applies Adam to the
// average.  Slots / flags / epochs are the PeerComm's (182 blocks fit its 256 flag sets), but the
// block partition is this kernel's own: between KX calls and the PeerComm's other exchanges every
// rank's stream must be synchronised (the trainers switch strategies only across a host sync and
// barrier, FusedTrainerBase.autotune), or a block could push into a slot region another block
// of a different partition is still reading.  Consecutive KX calls are ordered by the per-block
// flags alone.
constexpr int kKxThreads = 512;

__global__ __launch_bounds__(kKxThreads) void kx_kernel(KerasFused f, PeerArgs a) {
  __shared__ uint32_t s_ep;
  const int b = blockIdx.x, tid = threadIdx.x, r = a.rank, W = a.ws;
  const int i = b * kKxThreads + tid;
  const bool live = i < (int)L::total;
  const int t = __hip_atomic_load(f.adam_state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  if (tid == 0) s_ep = a.epoch[b] + 1;
  __syncthreads();
  const uint32_t ep = s_ep;
  const long long slot = a.slot_bytes / 4;
  const long long half = (long long)(ep & 1u) * 2 * W * slot;
  const float mine = live ? f.g[i] : 0.f;
  if (live)
    for (int j = 1; j < W; ++j) {
      const int p = (r + j) % W;
      reinterpret_cast<float*>(a.xbuf[p])[half + (long long)r * slot + i] = mine;
    }
  signal_peers(a, 0, b, ep);
  wait_peers(a, 0, b, ep);
  if (live) {
    const float* scat = reinterpret_cast<const float*>(a.xbuf[r]) + half + i;
    float acc = 0.f;
    for (int p = 0; p < W; ++p) {
      const float v = p == r ? mine : __builtin_nontemporal_load(scat + (long long)p * slot);
      acc = p == 0 ? v : acc + v;
    }
    adam_one(f, i, acc, t, a.scale);
  }
  if (tid == 0) {
    a.epoch[b] = ep;
    if (b == 0) __hip_atomic_store(f.adam_state + 1, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace keras

void keras_fused_forward(const KerasFused& f, hipStream_t st) {
  MX_CHECK(f.B > 0 && f.B % 8 == 0 && f.B <= 1024, "keras engine: batch must be a multiple of 8 (<= 1024)");
  MX_LAUNCH(keras::kf1_kernel, dim3(4 * f.B), dim3(512), 0, st, f);
  MX_LAUNCH(keras::kf2_kernel, dim3(f.B), dim3(512), 0, st, f);
}

void keras_fused_backward(const KerasFused& f, hipStream_t st) {
  MX_LAUNCH(keras::kb1_kernel, dim3(12 * f.B + f.B / 2 + 1), dim3(256), 0, st, f);
}

// Regions of the update (mode 0 / 1: the finalize reads the partial planes; mode 2: Adam from
// the all-reduced g, one thread per parameter; mode 3: only the conv2 repack)
static keras::KoPlan ko_plan(const KerasFused& f, int mode) {
  using L = KerasLayout;
  keras::KoPlan p{};
  int blk = 0;
  auto add = [&](size_t p0, size_t np, int T, int nplanes, long long stride, const float* src) {
    keras::KoRegion& r = p.r[p.nreg++];
    r.blk0 = blk;
    r.p0 = (int)p0;
    r.np = (int)np;
    r.T = T;
    r.nplanes = nplanes;
    r.stride = stride;
    r.src = src;
    const size_t per = T == 1 ? 256 : 64;
    blk += (int)((np + per - 1) / per);
  };
  const int B = f.B;
  if (mode == 2 || mode == 3) {
    add(0, L::total, 1, mode == 3 ? 0 : 1, 0, f.g);
  } else {
    add(L::w1, 320, 4, 4 * B, 320, f.pl1);
    add(L::w2, L::b2 - L::w2, 4, B, 18432, f.pl2);
    add(L::b2, 64, 4, B, 256, f.sv);
    add(L::w3, L::b3 - L::w3, 4, B / 8, 36864, f.pl3);
    add(L::b3, 64, 4, B, 256, f.sv + 64);
    add(L::fw1, L::fb1 - L::fw1, 4, B / 8, 36864, f.pf1);
    add(L::fb1, 64, 4, B, 256, f.sv + 128);
    add(L::fw2, 640, 1, 1, 0, f.gf2);
    add(L::fb2, 10, 4, B, 256, f.sv + 192);
  }
  p.nblocks = blk;
  return p;
}

int keras_exchange_blocks() { return (int)((KerasLayout::total + keras::kKxThreads - 1) / keras::kKxThreads); }

void keras_fused_exchange_adam(const KerasFused& f, const PeerArgs& a, hipStream_t st) {
  const int nb = keras_exchange_blocks();
  MX_CHECK(nb <= kPeerMaxBlocks && a.ws >= 2 && a.ws <= kPeerMaxRanks, "keras exchange: flag sets / world size");
  MX_CHECK(a.slot_bytes >= (long long)(KerasLayout::total * sizeof(float)), "keras exchange: slot too small");
  MX_LAUNCH(keras::kx_kernel, dim3(nb), dim3(keras::kKxThreads), 0, st, f, a);
}

void keras_fused_update(const KerasFused& f, int mode, float gscale, hipStream_t st) {
  MX_CHECK(mode >= 0 && mode <= 3, "keras engine: update mode 0..3");
  const keras::KoPlan plan = ko_plan(f, mode);
  MX_LAUNCH(keras::ko_kernel, dim3((unsigned)plan.nblocks), dim3(256), 0, st, f, plan, mode, gscale);
}

}  // namespace mx
