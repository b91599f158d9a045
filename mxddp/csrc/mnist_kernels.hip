// Fused gfx950 kernels for the MNIST-CNN training step (fp32 in / fp32 accumulate, exact).
//
// Step = synth | F1 conv1+ReLU (+weight packing, +zeroing) | F2 conv2+bias+ReLU+maxpool (MFMA)
//      | F3 fc1 split-K (MFMA) | F4 head: fc1 bias+ReLU, fc2, log_softmax+NLL, dlogits, fc2
//      grads, dh | F5 fc1 dgrad+wgrad (MFMA) + maxpool/ReLU backward scatter into dY2
//      | [bucket 0 all-reduce on the side stream] | F6 conv2 wgrad (MFMA) | F7 conv2 dgrad
//      (MFMA) + ReLU mask + conv1 wgrad/bias grad + wgrad transpose | [bucket 1] | SGD.
//
// MFMA = v_mfma_f32_16x16x4_f32: lane l holds A[l&15][k=l>>4], B[k=l>>4][l&15]; the C/D tile
// has col = l&15, row = 4*(l>>4) + reg.  Where operands are loaded as float4 along K, the
// K order inside a 16-wide group is permuted (k = 16*s' + 4*g + j for k-step (s', j) and
// lane group g = l>>4) identically for A and B -- legal because K is a pure reduction.
//
// Replaces (reference): cuDNN conv/ReLU/pool + cuBLAS linear + log_softmax/NLL + per-tensor
// SGD kernels reached through the PyTorch training loop of
// pytorch/distributed_data_parallel.py:118-152 (north-star MNIST CNN variant).
#include "common.h"
#include "mnist_engine.h"
#include "mnist_kernels.h"

namespace mx {
namespace {

using L = MnistLayout;
constexpr int kPack = 18432;               // 64*32*9
constexpr int kDY2 = 64 * 24 * 24;         // per image
__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

struct Scratch {  // carve of MnistFused::scratch (floats)
  float* wf;      // conv2 fwd B-fragments   [18 q][4 w][64 lane][4 j]
  float* wd;      // conv2 dgrad B-fragments [9 r][4 s][2 nt][64 lane][4 j]
  float* wacc;    // conv2 wgrad accumulator [9 r][64 co][32 ci]
  float* dy2;     // dense grad wrt conv2 pre-activation [B][64][24][24]
};
__host__ __device__ inline Scratch carve(float* s, int B) {
  Scratch c;
  c.wf = s;
  c.wd = s + kPack;
  c.wacc = s + 2 * kPack;
  c.dy2 = s + 3 * kPack;
  (void)B;
  return c;
}

// ------------------------------------------------------------------------------------------
// F1: conv1 (1->32, 3x3 valid) + bias + ReLU.  Block = (image b, 4 output channels).
// Side duties (grid-stride over all blocks): pack conv2 weights into the MFMA fragment
// orders used by F2 and F7, zero the split-K / atomic accumulators of this step, bump the
// synthetic-data counter.
__global__ __launch_bounds__(256) void f1_conv1_kernel(MnistFused f, Scratch sc) {
  __shared__ float xs[784];
  __shared__ float ws[4 * 9 + 4];
  const int b = blockIdx.x >> 3, cg = (blockIdx.x & 7) * 4;
  const int tid = threadIdx.x;
  const float* x = f.x + b * 784;
  for (int i = tid; i < 784; i += 256) xs[i] = x[i];
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
  if (gtid < 320) f.g[L::w1 + gtid] = 0.f;       // conv1 w+b grads (atomics in F7)
  if (gtid < 64) f.g[L::b2 + gtid] = 0.f;        // conv2 bias grad (atomics in F5)
  if (gtid == 0 && f.counter) *f.counter += 1;
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
  const int b = blockIdx.x / 12, py = blockIdx.x - b * 12;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float* a1 = f.a1 + (size_t)b * 32 * 676 + (2 * py) * 26;
  for (int i = tid; i < 32 * 104; i += 256) {
    const int ci = i / 104, rem = i - ci * 104;
    const int row = rem / 26, col = rem - row * 26;
    tile[ci * kF2ChP + row * kF2RowP + col] = a1[ci * 676 + rem];
  }
  float4 bq[18];
  const float4* wf = reinterpret_cast<const float4*>(sc.wf) + w * 64 + lane;
#pragma unroll
  for (int q = 0; q < 18; ++q) bq[q] = wf[q * 256];
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
    const float4 bv = bq[s >> 2];
    const float bf = (s & 3) == 0 ? bv.x : (s & 3) == 1 ? bv.y : (s & 3) == 2 ? bv.z : bv.w;
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
// further M-tiles when B > 64).  Operands are loaded straight to registers as float4 along K
// (64-byte row segments); the K permutation inside each 16-group is shared by A and B.
constexpr int kF3Chunk = 144, kF3Groups = kF3Chunk / 16;
__global__ __launch_bounds__(256) void f3_fc1_kernel(MnistFused f) {
  const int kc = blockIdx.x >> 2, nq = blockIdx.x & 3;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, m = lane & 15;
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
// F4: head (one workgroup): h = ReLU(h_pre + b1); logits = h W2^T + b2; log_softmax + NLL
// (mean over the local batch); argmax accuracy; dlogits = (softmax - onehot)/B;
// dW2 = dlogits^T h, db2 = sum dlogits, dh = (dlogits W2) * (h > 0), db1 = sum dh.
__global__ __launch_bounds__(256) void f4_head_kernel(MnistFused f) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int B = f.B, tid = threadIdx.x;
  float* hs = sm;                 // [B][129]
  float* w2s = hs + B * 129;      // [10][129]
  float* lg = w2s + 10 * 129;     // [B][10] logits -> dlogits
  float* red = lg + B * 10;       // [8]
  for (int i = tid; i < B * 128; i += 256) {
    const int b = i >> 7, n = i & 127;
    hs[b * 129 + n] = fmaxf(f.h[i] + f.p[L::fb1 + n], 0.f);
  }
  for (int i = tid; i < 1280; i += 256) w2s[(i >> 7) * 129 + (i & 127)] = f.p[L::fw2 + i];
  if (tid < 8) red[tid] = 0.f;
  __syncthreads();
  for (int i = tid; i < B * 10; i += 256) {
    const int b = i / 10, c = i - b * 10;
    const float* hp = hs + b * 129;
    const float* wp = w2s + c * 129;
    float acc = f.p[L::fb2 + c];
#pragma unroll 8
    for (int n = 0; n < 128; ++n) acc = fmaf(hp[n], wp[n], acc);
    lg[i] = acc;
  }
  __syncthreads();
  float loss = 0.f, corr = 0.f;
  if (tid < B) {
    float* l = lg + tid * 10;
    float mx = l[0];
    int am = 0;
    for (int c = 1; c < 10; ++c)
      if (l[c] > mx) { mx = l[c]; am = c; }
    float se = 0.f;
    for (int c = 0; c < 10; ++c) se += __expf(l[c] - mx);
    const float lse = mx + __logf(se);
    const int y = f.y[tid];
    loss = lse - l[y];
    corr = am == y ? 1.f : 0.f;
    const float inv = 1.f / (float)B;
    for (int c = 0; c < 10; ++c) l[c] = (__expf(l[c] - lse) - (c == y ? 1.f : 0.f)) * inv;
  }
  loss = wave_sum(loss);
  corr = wave_sum(corr);
  if ((tid & 63) == 0) {
    atomicAdd(&red[0], loss);
    atomicAdd(&red[1], corr);
  }
  __syncthreads();
  if (tid == 0 && f.metrics) {
    atomicAdd(f.metrics, red[0]);
    atomicAdd(f.metrics + 1, red[1]);
  }
  // dW2 [10][128], db2 [10]
  for (int i = tid; i < 1280 + 10; i += 256) {
    float acc = 0.f;
    if (i < 1280) {
      const int c = i >> 7, n = i & 127;
      for (int b = 0; b < B; ++b) acc = fmaf(lg[b * 10 + c], hs[b * 129 + n], acc);
      f.g[L::fw2 + i] = acc;
    } else {
      const int c = i - 1280;
      for (int b = 0; b < B; ++b) acc += lg[b * 10 + c];
      f.g[L::fb2 + c] = acc;
    }
  }
  // dh [B][128] (grad wrt fc1 pre-activation), db1 [128]
  for (int i = tid; i < B * 128; i += 256) {
    const int b = i >> 7, n = i & 127;
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < 10; ++c) acc = fmaf(lg[b * 10 + c], w2s[c * 129 + n], acc);
    f.dh[i] = hs[b * 129 + n] > 0.f ? acc : 0.f;
  }
  __syncthreads();  // dh visible to this block
  if (tid < 128) {
    float acc = 0.f;
    for (int b = 0; b < B; ++b) acc += f.dh[b * 128 + tid];
    f.g[L::fb1 + tid] = acc;
  }
}

// ------------------------------------------------------------------------------------------
// F5: fc1 backward for a 32-column slice of the 9216 inputs: dW1[:, cols] = dh^T pool[:, cols]
// (M=128, K=B) and dp[:, cols] = dh W1[:, cols] (M=B, K=128), both on MFMA from LDS.
// Epilogue scatters dp through the max-pool argmax / ReLU mask into the dense dY2 (grad
// wrt conv2 pre-activation) and accumulates db2.  dh is [B][132] in LDS (row pitch = 4 mod 32
// words: float4 row reads and 4-row-strided scalar reads are both bank-conflict free).
constexpr int kF5Cols = 32, kF5DhP = 132, kF5P = 36;
__global__ __launch_bounds__(256) void f5_fc1_bwd_kernel(MnistFused f, Scratch sc) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int B = f.B;
  float* dhs = sm;                       // [B][132]
  float* ps = dhs + B * kF5DhP;          // [B][36]
  float* wsm = ps + B * kF5P;            // [128][36]
  float* db2s = wsm + 128 * kF5P;        // [2]
  const int c0 = blockIdx.x * kF5Cols;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, m = lane & 15;
  for (int i = tid; i < B * 32; i += 256) {  // float4 granules of dh
    const int b = i >> 5, c4 = (i & 31) * 4;
    *reinterpret_cast<float4*>(dhs + b * kF5DhP + c4) = *reinterpret_cast<const float4*>(f.dh + b * 128 + c4);
  }
  for (int i = tid; i < B * 8; i += 256) {
    const int b = i >> 3, c4 = (i & 7) * 4;
    *reinterpret_cast<float4*>(ps + b * kF5P + c4) =
        *reinterpret_cast<const float4*>(f.pool + (size_t)b * 9216 + c0 + c4);
  }
  for (int i = tid; i < 128 * 8; i += 256) {
    const int n = i >> 3, c4 = (i & 7) * 4;
    *reinterpret_cast<float4*>(wsm + n * kF5P + c4) =
        *reinterpret_cast<const float4*>(f.p + L::fw1 + (size_t)n * 9216 + c0 + c4);
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
  for (int mt = w; mt < B / 16; mt += 4) {
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    const float* arow = dhs + (16 * mt + m) * kF5DhP + 4 * g;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const float4 av = *reinterpret_cast<const float4*>(arow + 16 * s);
      const float avv[4] = {av.x, av.y, av.z, av.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = 16 * s + 4 * g + j;
        acc[0] = mfma4(avv[j], wsm[n * kF5P + m], acc[0]);
        acc[1] = mfma4(avv[j], wsm[n * kF5P + 16 + m], acc[1]);
      }
    }
    // scatter: dp[b][kk] with kk = c0 + 16c + m = (co, py, px)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int kk = c0 + 16 * c + m;
      const int co = kk / 144, win = kk - co * 144, py = win / 12, px = win - py * 12;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int b = 16 * mt + 4 * g + j;
        const int q = idx[(size_t)b * 9216 + kk];
        const float v = acc[c][j];
        float* d = sc.dy2 + (((size_t)b * 64 + co) * 24 + 2 * py) * 24 + 2 * px;
        d[0] = q == 0 ? v : 0.f;
        d[1] = q == 1 ? v : 0.f;
        d[24] = q == 2 ? v : 0.f;
        d[25] = q == 3 ? v : 0.f;
        if (q < 4) db2_part[co == c0 / 144 ? 0 : 1] += v;
      }
    }
  }
  // db2: this block's 32 columns touch at most 2 channels (c0/144 and c0/144 + 1)
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float s = wave_sum(db2_part[k]);
    if (lane == 0 && s != 0.f) atomicAdd(&db2s[k], s);
  }
  __syncthreads();
  if (tid < 2) {
    const int co = c0 / 144 + tid;
    if (co < 64 && db2s[tid] != 0.f) atomicAdd(f.g + L::b2 + co, db2s[tid]);
  }
}

// ------------------------------------------------------------------------------------------
// F6: conv2 weight grad, wacc[r][co][ci] += sum_{pos} dY2[b][co][pos] * a1[b][ci][pos + (ky,kx)].
// Block = (image group, tap r); wave w owns co tile w (16) x both ci tiles; K = positions
// (576 per image), float4 along K for dY2 (16-byte aligned rows of 24), scalar loads for the
// shifted a1 rows.  The [r][co][ci] accumulator keeps every atomic wave-instruction as 16-lane
// contiguous 64-byte segments; F7 transposes it into the canonical conv2.weight grad.
template <int IMGS>
__global__ __launch_bounds__(256) void f6_conv2_wgrad_kernel(MnistFused f, Scratch sc) {
  const int r = blockIdx.x % 9, ig = blockIdx.x / 9;
  const int ky = r / 3, kx = r - 3 * ky;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, m = lane & 15;
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  for (int ii = 0; ii < IMGS; ++ii) {
    const int b = ig * IMGS + ii;
    if (b >= f.B) break;
    const float* dy = sc.dy2 + ((size_t)b * 64 + 16 * w + m) * 576 + 4 * g;
    const float* a1a = f.a1 + ((size_t)b * 32 + m) * 676 + ky * 26 + kx;
    const float* a1b = a1a + 16 * 676;
#pragma unroll 4
    for (int s = 0; s < 36; ++s) {  // 16 positions per s: rows of 24 -> pos = 16s + 4g + j
      const int p0 = 16 * s + 4 * g;
      const int oy = p0 / 24, ox = p0 - oy * 24;
      const float4 av = *reinterpret_cast<const float4*>(dy + 16 * s);
      const float* pa = a1a + oy * 26 + ox;
      const float* pb = a1b + oy * 26 + ox;
      acc[0] = mfma4(av.x, pa[0], acc[0]);
      acc[1] = mfma4(av.x, pb[0], acc[1]);
      acc[0] = mfma4(av.y, pa[1], acc[0]);
      acc[1] = mfma4(av.y, pb[1], acc[1]);
      acc[0] = mfma4(av.z, pa[2], acc[0]);
      acc[1] = mfma4(av.z, pb[2], acc[1]);
      acc[0] = mfma4(av.w, pa[3], acc[0]);
      acc[1] = mfma4(av.w, pb[3], acc[1]);
    }
  }
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int co = 16 * w + 4 * g + j, ci = 16 * c + m;
      atomicAdd(sc.wacc + (r * 64 + co) * 32 + ci, acc[c][j]);
    }
}

// ------------------------------------------------------------------------------------------
// F7: conv2 data grad + ReLU mask of conv1 + conv1 weight/bias grad (+ wacc transpose).
// GEMM M = input positions of image b (64 per block, 4 M-tiles -> waves), N = 32 ci,
// K = (r, co) = 576; A = dY2 gathered with the (ky,kx) shift and zero halo, B = pre-packed
// conv2 weights (float4 fragments from L2).  The epilogue masks with a1 > 0 and immediately
// contracts with the 3x3 input patches of x: dW1[ci][r] and db1[ci] are reduced in
// registers -> cross-lane -> LDS -> one atomic per value per block.  dA1 never touches HBM.
__global__ __launch_bounds__(256) void f7_conv2_dgrad_kernel(MnistFused f, Scratch sc) {
  __shared__ float red[4][32][10];
  const int b = blockIdx.x / 11, chunk = blockIdx.x - b * 11;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, m = lane & 15;
  // side duty: canonical conv2.weight grad from the [r][co][ci] accumulator (F6 finished)
  for (int i = blockIdx.x * 256 + tid; i < kPack; i += gridDim.x * 256) {
    const int co = i / 288, rem = i - co * 288, ci = rem / 9, r = rem - ci * 9;
    f.g[L::w2 + i] = sc.wacc[(r * 64 + co) * 32 + ci];
  }
  const int pos = chunk * 64 + 16 * w + m;  // this lane's A row (position in 26x26)
  const bool pv = pos < 676;
  const int iy = pv ? pos / 26 : 0, ix = pv ? pos - (pos / 26) * 26 : 0;
  const float* dyb = sc.dy2 + (size_t)b * kDY2;
  const float4* wd = reinterpret_cast<const float4*>(sc.wd) + lane;
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll 1
  for (int r = 0; r < 9; ++r) {
    const int ky = r / 3, kx = r - 3 * ky;
    const int oy = iy - ky, ox = ix - kx;
    const bool ok = pv && oy >= 0 && oy < 24 && ox >= 0 && ox < 24;
    const float* ap = dyb + (ok ? oy * 24 + ox : 0) + (4 * g) * 576;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const float4 b0 = wd[((r * 4 + s) * 2 + 0) * 64];
      const float4 b1 = wd[((r * 4 + s) * 2 + 1) * 64];
      const float b0v[4] = {b0.x, b0.y, b0.z, b0.w}, b1v[4] = {b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float a = ok ? ap[(16 * s + j) * 576] : 0.f;  // co = 16s + 4g + j
        acc[0] = mfma4(a, b0v[j], acc[0]);
        acc[1] = mfma4(a, b1v[j], acc[1]);
      }
    }
  }
  // epilogue: acc[c][j] = dA1 at position p = chunk*64 + 16w + 4g + j, channel ci = 16c + m
  float part[2][10];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int k = 0; k < 10; ++k) part[c][k] = 0.f;
  const float* xb = f.x + b * 784;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int p = chunk * 64 + 16 * w + 4 * g + j;
    if (p < 676) {
      const int py = p / 26, px = p - py * 26;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int ci = 16 * c + m;
        const float a1v = f.a1[((size_t)b * 32 + ci) * 676 + p];
        const float gv = a1v > 0.f ? acc[c][j] : 0.f;
        part[c][9] += gv;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) part[c][ky * 3 + kx] = fmaf(gv, xb[(py + ky) * 28 + px + kx], part[c][ky * 3 + kx]);
      }
    }
  }
  // reduce over the 4 lane groups (g) sharing ci = 16c + m
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      float v = part[c][k];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      part[c][k] = v;
    }
  if (g == 0) {
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int k = 0; k < 10; ++k) red[w][16 * c + m][k] = part[c][k];
  }
  __syncthreads();
  for (int i = tid; i < 320; i += 256) {
    const int ci = i / 10, k = i - ci * 10;
    const float v = red[0][ci][k] + red[1][ci][k] + red[2][ci][k] + red[3][ci][k];
    // conv1.weight grad [32][9] at L::w1, conv1.bias grad [32] at L::b1
    if (k < 9) atomicAdd(f.g + L::w1 + ci * 9 + k, v);
    else atomicAdd(f.g + L::b1 + ci, v);
  }
}

}  // namespace

size_t mnist_fused_scratch_floats(int B) { return 3 * (size_t)kPack + (size_t)B * kDY2; }

static void check(const MnistFused& f) {
  MX_CHECK(f.B % 16 == 0 && f.B >= 16 && f.B <= 128, "fused MNIST engine needs batch % 16 == 0 and 16 <= B <= 128");
}

void mnist_fused_forward(const MnistFused& f, hipStream_t st) {
  check(f);
  const Scratch sc = carve(f.scratch, f.B);
  hipLaunchKernelGGL(f1_conv1_kernel, dim3(f.B * 8), dim3(256), 0, st, f, sc);
  hipLaunchKernelGGL(f2_conv2_pool_kernel, dim3(f.B * 12), dim3(256), 0, st, f, sc);
  hipLaunchKernelGGL(f3_fc1_kernel, dim3((9216 / kF3Chunk) * 4), dim3(256), 0, st, f);
  MX_HIP_CHECK(hipGetLastError());
}

void mnist_fused_head(const MnistFused& f, hipStream_t st) {
  const size_t lds = sizeof(float) * ((size_t)f.B * 129 + 10 * 129 + f.B * 10 + 8);
  hipLaunchKernelGGL(f4_head_kernel, dim3(1), dim3(256), lds, st, f);
  MX_HIP_CHECK(hipGetLastError());
}

void mnist_fused_fc1_bwd(const MnistFused& f, hipStream_t st) {
  const Scratch sc = carve(f.scratch, f.B);
  const size_t lds = sizeof(float) * ((size_t)f.B * kF5DhP + f.B * kF5P + 128 * kF5P + 4);
  hipLaunchKernelGGL(f5_fc1_bwd_kernel, dim3(9216 / kF5Cols), dim3(256), lds, st, f, sc);
  MX_HIP_CHECK(hipGetLastError());
}

void mnist_fused_conv_bwd(const MnistFused& f, hipStream_t st) {
  const Scratch sc = carve(f.scratch, f.B);
  constexpr int kImgs = 1;
  hipLaunchKernelGGL(f6_conv2_wgrad_kernel<kImgs>, dim3(9 * ((f.B + kImgs - 1) / kImgs)), dim3(256), 0, st, f, sc);
  hipLaunchKernelGGL(f7_conv2_dgrad_kernel, dim3(f.B * 11), dim3(256), 0, st, f, sc);
  MX_HIP_CHECK(hipGetLastError());
}


}  // namespace mx
