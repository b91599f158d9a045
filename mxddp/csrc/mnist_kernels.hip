// Fused gfx950 kernels for the MNIST-CNN training step (fp32 in / fp32 accumulate, exact).
//
// Step = F1 synth batch + conv1+ReLU (+ conv2 weight packing, + zeroing) | F2 conv2+bias+ReLU+
//        maxpool (MFMA) | F3 fc1 split-K (MFMA) | F4 head: fc1 bias+ReLU, fc2, log_softmax+NLL,
//        dlogits, fc2 grads, dh | F5 fc1 dgrad+wgrad (MFMA), ReLU/maxpool-masked dp
//        | [bucket 0 all-reduce on the side stream] | F6 conv2 wgrad (MFMA) | F7 conv2 dgrad
//        (MFMA) + conv1 ReLU mask + conv1 wgrad/bias grad + wgrad transpose | [bucket 1] | SGD.
//
// MFMA = v_mfma_f32_16x16x4_f32: lane l holds A[l&15][k=l>>4], B[k=l>>4][l&15]; the C/D tile
// has col = l&15, row = 4*(l>>4) + reg.  Where operands are read as float4 along K the K order
// inside a 16-wide group is permuted (k = 16*s' + 4*g + j for k-step (s', j), lane group
// g = l>>4) identically for A and B -- legal because K is a pure reduction.
//
// The grad wrt the conv2 pre-activation, dY2, is never materialised: the backward kernels
// rebuild the tiles they need in LDS from dp (B x 9216) and the uint8 argmax map written by F2.
//
// Replaces (reference): cuDNN conv/ReLU/pool + cuBLAS linear + log_softmax/NLL + per-tensor
// SGD kernels reached through the PyTorch training loop of
// pytorch/distributed_data_parallel.py:118-152 (north-star MNIST CNN variant).
#include "mnist_common.h"
#include "rng.h"

namespace mx {
namespace mnist {
namespace {

// ------------------------------------------------------------------------------------------
// F1: [synthetic batch] + conv1 (1->32, 3x3 valid) + bias + ReLU.  Block = (image b, 4 output
// channels).  With f.synth the image is generated straight into LDS (Philox, identical stream
// to ops_data.hip synth_batch) by every block of the image; block cg==0 publishes x/y for the
// backward.  Side duties (grid-stride): pack conv2 weights into the MFMA fragment orders of
// F2 / F7 and zero this step's atomic accumulators.
__global__ __launch_bounds__(256) void f1_conv1_kernel(MnistFused f, Scratch sc) {
  __shared__ float xs[784];
  __shared__ float ws[4 * 9 + 4];
  const int b = blockIdx.x >> 3, cg = (blockIdx.x & 7) * 4;
  const int tid = threadIdx.x;
  if (f.synth) {
    const uint32_t ctr = (uint32_t)*f.counter;
    const uint2 key = synth_key(f.seed);
    const int label = synth_label(ctr, b, 10, key);
    const float* tp = f.tmpl + label * 784;
    if (tid < 196) {
      const int d = tid * 4;
      const uint4 r = synth_noise4(ctr, b, d, key);
      const float4 t = *reinterpret_cast<const float4*>(tp + d);
      const float4 v = make_float4(0.5f * t.x + 0.5f * u01(r.x), 0.5f * t.y + 0.5f * u01(r.y),
                                   0.5f * t.z + 0.5f * u01(r.z), 0.5f * t.w + 0.5f * u01(r.w));
      *reinterpret_cast<float4*>(xs + d) = v;
      if (cg == 0) *reinterpret_cast<float4*>(f.x + b * 784 + d) = v;
    }
    if (cg == 0 && tid == 0) f.y[b] = label;
  } else {
    for (int i = tid; i < 784; i += 256) xs[i] = f.x[b * 784 + i];
  }
  if (tid < 36) ws[tid] = f.p[L::w1 + cg * 9 + tid];
  if (tid < 4) ws[36 + tid] = f.p[L::b1 + cg + tid];
  // ---- side duties
  const int gtid = blockIdx.x * 256 + tid, gsz = gridDim.x * 256;
  const float* w2 = f.p + L::w2;
  for (int i = gtid; i < kPack; i += gsz) {
    {  // wf: i = ((q*4 + w)*64 + l)*4 + j
      const int j = i & 3, l = (i >> 2) & 63, w = (i >> 8) & 3, q = i >> 10;
      const int s = 4 * q + j;
      const int co = 16 * w + (l & 15), ci = 4 * (s & 7) + (l >> 4), r = s >> 3;
      sc.wf[i] = w2[(co * 32 + ci) * 9 + r];
    }
    {  // wd: i = ((((r*4 + s)*2 + nt)*64 + l)*4 + j
      const int j = i & 3, l = (i >> 2) & 63, nt = (i >> 8) & 1, s = (i >> 9) & 3, r = i >> 11;
      const int co = 16 * s + 4 * (l >> 4) + j, ci = 16 * nt + (l & 15);
      sc.wd[i] = w2[(co * 32 + ci) * 9 + r];
    }
    sc.wacc[i] = 0.f;
  }
  for (int i = gtid; i < f.B * 128; i += gsz) f.h[i] = 0.f;
  for (int i = gtid; i < f.B * 320; i += gsz) sc.g1[i] = 0.f;     // conv1 grad per-image partials (F7)
  if (gtid < 64) f.g[L::b2 + gtid] = 0.f;                         // conv2 bias grad (F5 atomics)
  if (gtid < 1280 + 10) f.g[L::fw2 + gtid] = 0.f;                 // fc2 w+b grads (F4 atomics)
  if (gtid < 128) f.g[L::fb1 + gtid] = 0.f;                       // fc1 bias grad (F4 atomics)
  __syncthreads();
  // ---- conv1
  float* out = f.a1 + ((size_t)b * 32 + cg) * 676;
  for (int i = tid; i < 4 * 676; i += 256) {
    const int c = i / 676, pos = i - c * 676;
    const int oy = pos / 26, ox = pos - oy * 26;
    const float* wp = ws + c * 9;
    const float* xp = xs + oy * 28 + ox;
    float acc = ws[36 + c];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) acc = fmaf(xp[ky * 28 + kx], wp[ky * 3 + kx], acc);
    out[i] = fmaxf(acc, 0.f);
  }
}

// ------------------------------------------------------------------------------------------
// F2: conv2 (32->64, 3x3) + bias + ReLU + maxpool 2x2, implicit GEMM on MFMA.
// Block = (image b, pooled row py): 2 output rows x 24 cols = 48 positions (3 M-tiles of 16)
// x 64 channels (wave w owns N-tile w).  M is ordered window-major (m = 4*window + 2*dy + dx),
// so a lane's 4 accumulator registers are exactly one 2x2 pooling window: max-pool + argmax
// happen in registers.  K = 288 ordered k = r*32 + ci (r = ky*3+kx) so the im2col LDS offset
// splits into a per-lane base + a compile-time immediate.  The input tile [32 ci][4 rows][26]
// lives in LDS with row pitch 40 and channel pitch 176 (= 8, 16 mod 32 banks): the 32 lanes
// of each ds_read_b32 half-wave hit 32 distinct banks.  B fragments for all 72 k-steps
// (18 float4 per lane, pre-packed by F1) are loaded once into registers.
constexpr int kF2RowP = 40, kF2ChP = 176;
__global__ __launch_bounds__(256) void f2_conv2_pool_kernel(MnistFused f, Scratch sc) {
  __shared__ float tile[32 * kF2ChP];
  const int bid = xcd_remap(blockIdx.x, gridDim.x);  // an image's 12 blocks share one XCD L2
  const int b = bid / 12, py = bid - b * 12;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float* a1 = f.a1 + (size_t)b * 32 * 676 + (2 * py) * 26;
  float4 bq[18];
  const float4* wf = reinterpret_cast<const float4*>(sc.wf) + w * 64 + lane;
#pragma unroll
  for (int q = 0; q < 18; ++q) bq[q] = wf[q * 256];
  {  // 32 ci x 104 = 3328 = 13 x 256 values: issue all loads, then all LDS stores
    float v[13];
#pragma unroll
    for (int k = 0; k < 13; ++k) {
      const int i = tid + 256 * k, ci = i / 104, rem = i - ci * 104;
      v[k] = a1[ci * 676 + rem];
    }
#pragma unroll
    for (int k = 0; k < 13; ++k) {
      const int i = tid + 256 * k, ci = i / 104, rem = i - ci * 104;
      const int row = rem / 26, col = rem - row * 26;
      tile[ci * kF2ChP + row * kF2RowP + col] = v[k];
    }
  }
  __syncthreads();
  const int m = lane & 15, g = lane >> 4;
  const int base = g * kF2ChP + ((m >> 1) & 1) * kF2RowP + 2 * (m >> 2) + (m & 1);
  f32x4 acc[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 72; ++s) {
    const int r = s >> 3, ky = r / 3, kx = r - 3 * (r / 3);
    const int koff = 4 * (s & 7) * kF2ChP + ky * kF2RowP + kx;
    const float bf = sel4(bq[s >> 2], s & 3);
#pragma unroll
    for (int t = 0; t < 3; ++t) acc[t] = mfma4(tile[base + 8 * t + koff], bf, acc[t]);
  }
  // epilogue: lane holds window (4t + g) of channel co for the 4 positions j = 2*dy + dx
  const int co = 16 * w + m;
  const float bias = f.p[L::b2 + co];
  uint8_t* idx = reinterpret_cast<uint8_t*>(f.idx);
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    float best = acc[t][0];
    int q = 0;
#pragma unroll
    for (int j = 1; j < 4; ++j)
      if (acc[t][j] > best) { best = acc[t][j]; q = j; }
    const float v = best + bias;
    const int o = ((b * 64 + co) * 12 + py) * 12 + 4 * t + g;
    f.pool[o] = v > 0.f ? v : 0.f;
    idx[o] = v > 0.f ? (uint8_t)q : (uint8_t)4;
  }
}

// ------------------------------------------------------------------------------------------
// F3: fc1 forward h_pre[b][n] += pool[b][k-chunk] . W1[n][k-chunk] (split-K, MFMA, atomics).
// Block = (k-chunk of 144, 32 output features); wave w = batch rows 16w..16w+15 (loops over
// further M-tiles when B > 64).  Operands go straight to registers as float4 along K (64-byte
// row segments); the K permutation inside each 16-group is shared by A and B.
constexpr int kF3Chunk = 144, kF3Groups = kF3Chunk / 16;
__global__ __launch_bounds__(256) void f3_fc1_kernel(MnistFused f) {
  const int kc = blockIdx.x >> 2, nq = blockIdx.x & 3;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, m = lane & 15;
  if (f.synth && blockIdx.x == 0 && threadIdx.x == 0) *f.counter += 1;  // F1 consumed it
  const int k0 = kc * kF3Chunk + 4 * g;
  const float* W = f.p + L::fw1;
  float4 bw[2][kF3Groups];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int s = 0; s < kF3Groups; ++s)
      bw[nt][s] = *reinterpret_cast<const float4*>(W + (size_t)(32 * nq + 16 * nt + m) * 9216 + k0 + 16 * s);
  for (int mt = w; mt < f.B / 16; mt += 4) {
    float4 av[kF3Groups];
    const float* A = f.pool + (size_t)(16 * mt + m) * 9216 + k0;
#pragma unroll
    for (int s = 0; s < kF3Groups; ++s) av[s] = *reinterpret_cast<const float4*>(A + 16 * s);
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int s = 0; s < kF3Groups; ++s)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        acc[nt] = mfma4(av[s].x, bw[nt][s].x, acc[nt]);
        acc[nt] = mfma4(av[s].y, bw[nt][s].y, acc[nt]);
        acc[nt] = mfma4(av[s].z, bw[nt][s].z, acc[nt]);
        acc[nt] = mfma4(av[s].w, bw[nt][s].w, acc[nt]);
      }
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        atomicAdd(f.h + (16 * mt + 4 * g + j) * 128 + 32 * nq + 16 * nt + m, acc[nt][j]);
  }
}

// ------------------------------------------------------------------------------------------
// F4: head.  Block = 4 batch rows, one wave per row.  h = ReLU(h_pre + b1); logits =
// h W2^T + b2 (wave reductions); log_softmax + NLL (mean over the local batch) + argmax
// accuracy; dlogits = (softmax - onehot)/B; dh = (dlogits W2) * (h > 0).  Per-block partial
// sums of dW2 = dlogits^T h, db2, db1 = sum dh are added atomically (zeroed by F1).
__global__ __launch_bounds__(256) void f4_head_kernel(MnistFused f) {
  __shared__ float w2s[10 * 128];
  __shared__ float hs[4][128];
  __shared__ float dhs[4][128];
  __shared__ float dls[4][10];
  __shared__ float red[2];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b = blockIdx.x * 4 + w;
  for (int i = tid; i < 1280; i += 256) w2s[i] = f.p[L::fw2 + i];
  if (tid < 2) red[tid] = 0.f;
  const float h0 = fmaxf(f.h[b * 128 + lane] + f.p[L::fb1 + lane], 0.f);
  const float h1 = fmaxf(f.h[b * 128 + 64 + lane] + f.p[L::fb1 + 64 + lane], 0.f);
  hs[w][lane] = h0;
  hs[w][64 + lane] = h1;
  __syncthreads();
  float lg[10];
#pragma unroll
  for (int c = 0; c < 10; ++c) lg[c] = wave_sum(h0 * w2s[c * 128 + lane] + h1 * w2s[c * 128 + 64 + lane]) + f.p[L::fb2 + c];
  float mx = lg[0];
  int am = 0;
#pragma unroll
  for (int c = 1; c < 10; ++c)
    if (lg[c] > mx) { mx = lg[c]; am = c; }
  float se = 0.f;
#pragma unroll
  for (int c = 0; c < 10; ++c) se += __expf(lg[c] - mx);
  const float lse = mx + __logf(se);
  const int y = f.y[b];
  const float inv = 1.f / (float)f.B;
  float dl[10];
  float ly = 0.f;
#pragma unroll
  for (int c = 0; c < 10; ++c) {
    dl[c] = (__expf(lg[c] - lse) - (c == y ? 1.f : 0.f)) * inv;
    if (c == y) ly = lg[c];
  }
  if (lane == 0) {
    atomicAdd(&red[0], lse - ly);
    atomicAdd(&red[1], am == y ? 1.f : 0.f);
  }
  if (lane < 10) {
    float v = 0.f;
#pragma unroll
    for (int c = 0; c < 10; ++c) v = lane == c ? dl[c] : v;
    dls[w][lane] = v;
  }
  float d0 = 0.f, d1 = 0.f;
#pragma unroll
  for (int c = 0; c < 10; ++c) {
    d0 = fmaf(dl[c], w2s[c * 128 + lane], d0);
    d1 = fmaf(dl[c], w2s[c * 128 + 64 + lane], d1);
  }
  d0 = h0 > 0.f ? d0 : 0.f;
  d1 = h1 > 0.f ? d1 : 0.f;
  f.dh[b * 128 + lane] = d0;
  f.dh[b * 128 + 64 + lane] = d1;
  dhs[w][lane] = d0;
  dhs[w][64 + lane] = d1;
  __syncthreads();
  for (int i = tid; i < 1280; i += 256) {
    const int c = i >> 7, n = i & 127;
    atomicAdd(f.g + L::fw2 + i, dls[0][c] * hs[0][n] + dls[1][c] * hs[1][n] + dls[2][c] * hs[2][n] + dls[3][c] * hs[3][n]);
  }
  if (tid < 10) atomicAdd(f.g + L::fb2 + tid, dls[0][tid] + dls[1][tid] + dls[2][tid] + dls[3][tid]);
  if (tid >= 128) {
    const int n = tid - 128;
    atomicAdd(f.g + L::fb1 + n, dhs[0][n] + dhs[1][n] + dhs[2][n] + dhs[3][n]);
  }
  if (tid == 0 && f.metrics) {
    atomicAdd(f.metrics, red[0]);
    atomicAdd(f.metrics + 1, red[1]);
  }
}

// ------------------------------------------------------------------------------------------
// F5: fc1 backward for a 32-column slice of the 9216 inputs: dW1[:, cols] = dh^T pool[:, cols]
// (M=128, K=B) and dp[:, cols] = dh W1[:, cols] (M=B, K=128), both on MFMA from LDS.
// Epilogue masks dp with the max-pool argmax / ReLU liveness (dead windows -> 0) and
// accumulates db2.  dh is [B][132] in LDS (row pitch = 4 mod 32 words: float4 row reads and
// 4-row-strided scalar reads are both bank-conflict free).
constexpr int kF5Cols = 32, kF5DhP = 132, kF5P = 36;
template <int B>
__global__ __launch_bounds__(256) void f5_fc1_bwd_kernel(MnistFused f) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* dhs = sm;                       // [B][132]
  float* ps = dhs + B * kF5DhP;          // [B][36]
  float* wsm = ps + B * kF5P;            // [128][36]
  float* db2s = wsm + 128 * kF5P;        // [2]
  const int c0 = blockIdx.x * kF5Cols;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, m = lane & 15;
  {  // all global loads in flight at once (B/8 + B/32 + 4 float4 per thread), then LDS stores
    constexpr int ND = B * 32 / 256, NP = (B * 8 + 255) / 256, NW = 4;
    float4 vd[ND], vp[NP], vw[NW];
#pragma unroll
    for (int k = 0; k < ND; ++k) {
      const int i = tid + 256 * k;
      vd[k] = *reinterpret_cast<const float4*>(f.dh + (i >> 5) * 128 + (i & 31) * 4);
    }
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int i = min(tid + 256 * k, B * 8 - 1);
      vp[k] = *reinterpret_cast<const float4*>(f.pool + (size_t)(i >> 3) * 9216 + c0 + (i & 7) * 4);
    }
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      const int i = tid + 256 * k;
      vw[k] = *reinterpret_cast<const float4*>(f.p + L::fw1 + (size_t)(i >> 3) * 9216 + c0 + (i & 7) * 4);
    }
#pragma unroll
    for (int k = 0; k < ND; ++k) {
      const int i = tid + 256 * k;
      *reinterpret_cast<float4*>(dhs + (i >> 5) * kF5DhP + (i & 31) * 4) = vd[k];
    }
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int i = tid + 256 * k;
      if (i < B * 8) *reinterpret_cast<float4*>(ps + (i >> 3) * kF5P + (i & 7) * 4) = vp[k];
    }
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      const int i = tid + 256 * k;
      *reinterpret_cast<float4*>(wsm + (i >> 3) * kF5P + (i & 7) * 4) = vw[k];
    }
  }
  if (tid < 2) db2s[tid] = 0.f;
  __syncthreads();
  // ---- dW1 tiles: rows n (8 M-tiles, wave w takes 2w, 2w+1), cols 2 N-tiles, K = B
  {
    f32x4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < 2; ++c) acc[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < B / 16; ++s) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int b = 16 * s + 4 * g + j;
        const float a0 = dhs[b * kF5DhP + 32 * w + m], a1v = dhs[b * kF5DhP + 32 * w + 16 + m];
        const float b0 = ps[b * kF5P + m], b1v = ps[b * kF5P + 16 + m];
        acc[0][0] = mfma4(a0, b0, acc[0][0]);
        acc[0][1] = mfma4(a0, b1v, acc[0][1]);
        acc[1][0] = mfma4(a1v, b0, acc[1][0]);
        acc[1][1] = mfma4(a1v, b1v, acc[1][1]);
      }
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = 32 * w + 16 * a + 4 * g + j;
          f.g[L::fw1 + (size_t)n * 9216 + c0 + 16 * c + m] = acc[a][c][j];
        }
  }
  // ---- dp tiles: rows b (M-tiles of 16, wave-strided), cols 2 N-tiles, K = 128
  float db2_part[2] = {0.f, 0.f};
  const uint8_t* idx = reinterpret_cast<const uint8_t*>(f.idx);
  const int co_lo = c0 / 144;
  for (int mt = w; mt < B / 16; mt += 4) {
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    const float* arow = dhs + (16 * mt + m) * kF5DhP + 4 * g;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const float4 av = *reinterpret_cast<const float4*>(arow + 16 * s);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = 16 * s + 4 * g + j;
        acc[0] = mfma4(sel4(av, j), wsm[n * kF5P + m], acc[0]);
        acc[1] = mfma4(sel4(av, j), wsm[n * kF5P + 16 + m], acc[1]);
      }
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int kk = c0 + 16 * c + m;
      const int hi = (kk / 144) != co_lo;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const size_t o = (size_t)(16 * mt + 4 * g + j) * 9216 + kk;
        const bool alive = idx[o] < 4;
        const float v = alive ? acc[c][j] : 0.f;
        f.dp[o] = v;
        db2_part[hi] += v;
      }
    }
  }
  // db2: this block's 32 columns touch at most 2 channels (co_lo and co_lo + 1)
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float s = wave_sum(db2_part[k]);
    if (lane == 0 && s != 0.f) atomicAdd(&db2s[k], s);
  }
  __syncthreads();
  if (tid < 2) {
    const int co = co_lo + tid;
    if (co < 64 && db2s[tid] != 0.f) atomicAdd(f.g + L::b2 + co, db2s[tid]);
  }
}

}  // namespace
}  // namespace mnist

using namespace mnist;

size_t mnist_fused_scratch_floats(int B) { return scratch_floats(B); }

static void check(const MnistFused& f) {
  MX_CHECK(f.B % 16 == 0 && f.B >= 16 && f.B <= 128, "fused MNIST engine needs batch % 16 == 0 and 16 <= B <= 128");
}

static void set_lds_limits() {
  static bool done = false;
  if (done) return;
  const void* fns[] = {reinterpret_cast<const void*>(f5_fc1_bwd_kernel<16>),
                       reinterpret_cast<const void*>(f5_fc1_bwd_kernel<32>),
                       reinterpret_cast<const void*>(f5_fc1_bwd_kernel<48>),
                       reinterpret_cast<const void*>(f5_fc1_bwd_kernel<64>),
                       reinterpret_cast<const void*>(f5_fc1_bwd_kernel<80>),
                       reinterpret_cast<const void*>(f5_fc1_bwd_kernel<96>),
                       reinterpret_cast<const void*>(f5_fc1_bwd_kernel<112>),
                       reinterpret_cast<const void*>(f5_fc1_bwd_kernel<128>)};
  for (const void* fn : fns)
    MX_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  done = true;
}

void mnist_fused_forward(const MnistFused& f, hipStream_t st) {
  check(f);
  set_lds_limits();
  const Scratch sc = carve(f.scratch);
  hipLaunchKernelGGL(f1_conv1_kernel, dim3(f.B * 8), dim3(256), 0, st, f, sc);
  hipLaunchKernelGGL(f2_conv2_pool_kernel, dim3(f.B * 12), dim3(256), 0, st, f, sc);
  hipLaunchKernelGGL(f3_fc1_kernel, dim3((9216 / kF3Chunk) * 4), dim3(256), 0, st, f);
  MX_HIP_CHECK(hipGetLastError());
}

void mnist_fused_head(const MnistFused& f, hipStream_t st) {
  hipLaunchKernelGGL(f4_head_kernel, dim3(f.B / 4), dim3(256), 0, st, f);
  MX_HIP_CHECK(hipGetLastError());
}

void mnist_fused_fc1_bwd(const MnistFused& f, hipStream_t st) {
  const size_t lds = sizeof(float) * ((size_t)f.B * kF5DhP + f.B * kF5P + 128 * kF5P + 4);
  const dim3 grid(9216 / kF5Cols), block(256);
  switch (f.B) {
    case 16: hipLaunchKernelGGL(f5_fc1_bwd_kernel<16>, grid, block, lds, st, f); break;
    case 32: hipLaunchKernelGGL(f5_fc1_bwd_kernel<32>, grid, block, lds, st, f); break;
    case 48: hipLaunchKernelGGL(f5_fc1_bwd_kernel<48>, grid, block, lds, st, f); break;
    case 64: hipLaunchKernelGGL(f5_fc1_bwd_kernel<64>, grid, block, lds, st, f); break;
    case 80: hipLaunchKernelGGL(f5_fc1_bwd_kernel<80>, grid, block, lds, st, f); break;
    case 96: hipLaunchKernelGGL(f5_fc1_bwd_kernel<96>, grid, block, lds, st, f); break;
    case 112: hipLaunchKernelGGL(f5_fc1_bwd_kernel<112>, grid, block, lds, st, f); break;
    case 128: hipLaunchKernelGGL(f5_fc1_bwd_kernel<128>, grid, block, lds, st, f); break;
    default: MX_CHECK(false, "unsupported fused batch");
  }
  MX_HIP_CHECK(hipGetLastError());
}

}  // namespace mx
