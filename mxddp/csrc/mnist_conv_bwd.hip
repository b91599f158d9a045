// Fused conv backward of the MNIST-CNN step (fp32 MFMA): F6 conv2 weight grad, F7 conv2 data
// grad + conv1 ReLU mask + conv1 weight/bias grad.  See mnist_kernels.hip for the step map.
//
// dY2 (grad wrt the conv2 pre-activation, B x 64 x 24 x 24, 75 % zeros from the 2x2 max-pool)
// is NEVER materialised.  Both kernels stage the compact pooled form -- dp (B x 64 x 144,
// already zeroed on dead windows by F5) and the uint8 argmax map q written by F2 -- into LDS
// with plain coalesced copies, and expand on the fly while forming MFMA operands:
//   dY2[co][oy][ox] = (q[co][oy/2][ox/2] == 2*(oy&1) + (ox&1)) ? dp[co][oy/2][ox/2] : 0.
// The expansion is 1 compare + 1 select per element on the VALU, which co-issues with the
// MFMA pipe; LDS traffic for the A operand drops 4x versus a dense dY2 tile.
#include <cstdlib>
#include <string>

#include "mnist_common.h"
#include "peer_device.h"

namespace mx {
namespace mnist {
namespace {

// ------------------------------------------------------------------------------------------
// F6: conv2 weight grad.  wacc[r][co][ci] += sum_pos dY2[b][co][pos] * a1[b][ci][pos + (ky,kx)]
// Block = (image b, tap r); wave w owns co tile w (16) x both ci tiles (32).  GEMM K = the 576
// output positions, walked in 16-position groups: lane group g takes positions 16s+4g .. +3,
// i.e. 4 consecutive columns of one output row = 2 pooling windows -> A = expand(dp float2,
// 2-bit argmax codes), B = a1 window row (LDS float4).  a1 is never read from HBM: each
// 2-row chunk of the shifted a1 window is recomputed from the 28x28 input image in LDS
// (conv1 + ReLU, 54 FMAs per thread per chunk, weights in registers), so F2 does not have to
// publish a1 at all.  LDS (51.3 KB -> 3 blocks per CU): dp [64][148] (pitch 148: the 16 co
// rows x 2 lane groups of a ds_read_b64 half-wave land on distinct banks), a1 chunk [32][52]
// (pitch 52 = 13 x 16 B, odd, for ds_read_b128), x [784], conv1 w/b [320], argmax codes packed
// 4 per byte [64][36] (dead windows have dp = 0, so their code is irrelevant).
constexpr int kF6DpP = 148, kF6Rows = 2, kF6Pos = kF6Rows * 24, kF6BP = 52, kF6Chunks = 24 / kF6Rows;
constexpr size_t kF6Lds = sizeof(float) * (64 * kF6DpP + 32 * kF6BP + 784 + 320) + 64 * 36;
__device__ __forceinline__ void f6_body(const MnistFused& f, const Scratch& sc, float* sm, int braw, int nblk) {
  MX_TRACE_B(f, 3, 0, braw);
  float* dps = sm;                                              // [64][148]
  float* Bs = dps + 64 * kF6DpP;                                // [32][52]
  float* xs = Bs + 32 * kF6BP;                                  // [28][28]
  float* w1s = xs + 784;                                        // conv1 w [32][9], b [32]
  uint8_t* qs = reinterpret_cast<uint8_t*>(w1s + 320);          // [64][36] packed 2-bit codes
  const int bid = xcd_remap(braw, nblk);  // an image's 9 tap blocks share one XCD L2
  const int r = bid % 9, b = bid / 9;
  const int ky = r / 3, kx = r - 3 * ky;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, m = lane & 15;
  // compact dY2 of image b: dp (float4 granules) and argmax codes (uint32 = 4 windows -> 1 byte)
  {
    const float4* src = reinterpret_cast<const float4*>(f.dp + (size_t)b * 9216);
    const uint32_t* qsrc = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(f.idx) + (size_t)b * 9216);
    float4 dv[9];
    uint32_t qv[9];
    float xv[4], wv2[2];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      dv[k] = src[tid + 256 * k];
      qv[k] = qsrc[tid + 256 * k];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) xv[k] = f.x[b * 784 + min(tid + 256 * k, 783)];
#pragma unroll
    for (int k = 0; k < 2; ++k) wv2[k] = f.p[L::w1 + min(tid + 256 * k, 319)];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int i = tid + 256 * k, co = i / 36, c4 = (i - co * 36) * 4;
      *reinterpret_cast<float4*>(dps + co * kF6DpP + c4) = dv[k];
      const uint32_t q = qv[k] & 0x03030303u;
      qs[i] = (uint8_t)(q | (q >> 6) | (q >> 12) | (q >> 18));
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (tid + 256 * k < 784) xs[tid + 256 * k] = xv[k];
#pragma unroll
    for (int k = 0; k < 2; ++k)
      if (tid + 256 * k < 320) w1s[tid + 256 * k] = wv2[k];
  }
  __syncthreads();
  MX_TRACE_B(f, 3, 1, braw);
  // conv1 role of this thread: channel cw, chunk row rr, 6 output columns from 6*cg
  const int cw = tid >> 3, rr = (tid >> 2) & 1, cg = tid & 3;
  float wk[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) wk[k] = w1s[cw * 9 + k];
  const float bk = w1s[288 + cw];
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  const float* dpr = dps + (16 * w + m) * kF6DpP;
  const uint8_t* qr = qs + (16 * w + m) * 36;
  // a1[cw][oy0 + ky + rr][kx + 6cg .. +5] = ReLU(conv1(x)) for chunk row oy0, into registers;
  // chunk c+1 is computed in the same basic block as chunk c's MFMAs so the scheduler can
  // interleave the FMAs with the (long-latency) MFMA issue
  float av1[6];
  auto conv1_chunk = [&](int oy0) {
    const float* xp = xs + (oy0 + ky + rr) * 28 + kx + 6 * cg;
    float xr[3][8];
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int c = 0; c < 8; ++c) xr[dy][c] = xp[dy * 28 + c];
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      float v = bk;
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) v = fmaf(xr[dy][c + dx], wk[dy * 3 + dx], v);
      av1[c] = fmaxf(v, 0.f);
    }
  };
  float* bo = Bs + cw * kF6BP + rr * 24 + 6 * cg;
  conv1_chunk(0);
#pragma unroll 1
  for (int ch = 0; ch < kF6Chunks; ++ch) {
    const int oy0 = ch * kF6Rows;
    if (ch > 0) __syncthreads();  // previous chunk's reads of Bs are done
#pragma unroll
    for (int c = 0; c < 6; ++c) bo[c] = av1[c];
    __syncthreads();
    // next chunk (clamped on the last iteration: branch-free, so it shares the MFMA block)
    conv1_chunk(min(oy0 + kF6Rows, 24 - kF6Rows));
    const float* br0 = Bs + m * kF6BP + 4 * g;
    const float* br1 = Bs + (16 + m) * kF6BP + 4 * g;
#pragma unroll
    for (int s = 0; s < kF6Pos / 16; ++s) {
      const int p0 = oy0 * 24 + 16 * s + 4 * g;  // absolute output position of j = 0
      const int oy = p0 / 24, ox = p0 - oy * 24;  // ox % 4 == 0 -> two whole windows
      const int w0 = (oy >> 1) * 12 + (ox >> 1);  // even
      const uint32_t t0 = (oy & 1) << 1;
      const float2 d = *reinterpret_cast<const float2*>(dpr + w0);
      const uint32_t qq = (uint32_t)qr[w0 >> 2] >> ((w0 & 3) * 2);
      const uint32_t q0 = qq & 3, q1 = (qq >> 2) & 3;
      const float a0 = q0 == t0 ? d.x : 0.f;
      const float a1 = q0 == t0 + 1 ? d.x : 0.f;
      const float a2 = q1 == t0 ? d.y : 0.f;
      const float a3 = q1 == t0 + 1 ? d.y : 0.f;
      const float4 b0 = *reinterpret_cast<const float4*>(br0 + 16 * s);
      const float4 b1 = *reinterpret_cast<const float4*>(br1 + 16 * s);
      acc[0] = mfma4(a0, b0.x, acc[0]);
      acc[1] = mfma4(a0, b1.x, acc[1]);
      acc[0] = mfma4(a1, b0.y, acc[0]);
      acc[1] = mfma4(a1, b1.y, acc[1]);
      acc[0] = mfma4(a2, b0.z, acc[0]);
      acc[1] = mfma4(a2, b1.z, acc[1]);
      acc[0] = mfma4(a3, b0.w, acc[0]);
      acc[1] = mfma4(a3, b1.w, acc[1]);
    }
  }
  MX_TRACE_B(f, 3, 2, braw);
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int co = 16 * w + 4 * g + j, ci = 16 * c + m;
      atomicAdd(sc.wacc + (b & (kWaccSlabs - 1)) * kPack + (r * 64 + co) * 32 + ci, acc[c][j]);
    }
  MX_TRACE_B(f, 3, 3, braw);
}

// ------------------------------------------------------------------------------------------
// F6W: the same conv2 weight gradient as Winograd F(2x2,3x3): 2.25x fewer MFMAs.  The 2x2 output
// tiles of conv2 are exactly the pool windows, so dY2 of tile t has ONE nonzero (value dp, argmax
// code q) and its Winograd transform A dY A^T = dp * a(qy) a(qx)^T (a(0) = (1,1,1,0),
// a(1) = (0,1,-1,-1)) is built in registers.  16 GEMMs (one per Winograd point xi) over
// K = 144 tiles: dU[xi][co][ci] = sum_t W[xi][co][t] V[xi][t][ci], V = B^T a1_t B; then
// dw = G^T dU G lane-locally (all 16 xi of a (co, ci) sit in one lane) and one atomic per
// weight per block, into the same [tap][co][ci] accumulator as F6.
// Block = (image, ci half): all 144 tiles, so the atomics per image stay 64x32x9 as in F6.
// Wave w = co 16w..16w+15.  6 chunks of 2 tile rows: (A) conv1 + ReLU of the 6 a1 rows of the
// chunk for the block's 16 ci -> LDS, (B) V of 24 tiles x 16 ci -> LDS ([t][ci][20]: conflict-free
// ds_read_b128 of the 16 xi), (C) 6 k-steps of 16 MFMAs; K inside a chunk is ordered
// t = 6g + s (lane group g) so a lane's dp / q operands are 6 contiguous windows (float2 / u16
// loads, prefetched one chunk ahead).
// kA1 (default): phase A loads the chunk's a1 rows that F2 published (one chunk ahead, 3 float4
// per thread in registers) instead of recomputing conv1: phase A was 5.4 of F6W's 25 us.  The a1
// tile pitch is then 164 (16-byte rows for the float4 stores; 36 ci mod 64 banks keeps phase B's
// reads conflict-free).
constexpr int kF6WA1P = 157, kF6WA1PL = 164, kF6WVP = 20;
constexpr size_t kF6WLds = sizeof(float) * (784 + 160 + 16 * kF6WA1PL + 24 * 16 * kF6WVP);
// kF6WSplit = blocks per (image, ci half), each 6 / kF6WSplit chunks
// kCoS = 2 (co-split): block = (image, ci half, co half) -- 2x the blocks, each wave owns one co
// tile and HALF the Winograd points (ky-side rows i = 2xh, 2xh+1: 8 accumulators, half the MFMAs);
// the wave pair sharing a co tile sums its partial G^T dU G outputs through LDS and each wave
// issues the atomics of two of its four co rows, so the atomic count per image is unchanged while
// the per-wave MFMA chain (the F67 long pole) halves and the weight gradient spreads over 2x the CUs.
template <int kF6WSplit, bool kA1, int kCoS = 1>
__device__ __forceinline__ void f6w_body(const MnistFused& f, const Scratch& sc, float* sm, int braw, int nblk) {
  MX_TRACE_B(f, 3, 0, braw);
  constexpr int kA1P = kA1 ? kF6WA1PL : kF6WA1P;
  float* xs = sm;             // [784]
  float* w1s = xs + 784;      // conv1 w [16][9] then b [16] of this ci half
  float* a1s = w1s + 160;     // [16 ci][kA1P]: 6 a1 rows x 26
  float* vs = a1s + 16 * kA1P;  // [24 t][16 ci][20]
  const int bid = xcd_remap(braw, nblk);
  static_assert(kCoS == 1 || kF6WSplit == 1, "co-split only with unsplit chunks");
  const int b = bid / (2 * kF6WSplit * kCoS), h = bid & 1, c0 = ((bid >> 1) % kF6WSplit) * (6 / kF6WSplit);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, m = lane & 15;
  // co tile of this wave and (kCoS = 2) its Winograd-row half
  const int ct = kCoS == 1 ? w : 2 * ((bid >> 1) & 1) + (w & 1), xh = kCoS == 1 ? 0 : w >> 1;
  constexpr int kNI = 4 / kCoS;  // Winograd rows i per wave
  // kA1: a1 rows 4c .. 4c+5 of the block's 16 ci = 16 x 39 float4 (624 of the 768 slots)
  // (three named registers, not an array: an array here was placed in scratch memory)
  const float* a1b = f.a1 + ((size_t)b * 32 + 16 * h) * 676;
  int a1src[3], a1dst[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int i = min(tid + 256 * k, 623), ci = i / 39, f4 = i - 39 * ci;
    a1src[k] = ci * 676 + 4 * f4;
    a1dst[k] = tid + 256 * k < 624 ? ci * kA1P + 4 * f4 : -1;
  }
  float4 pa0, pa1, pa2;
  if constexpr (kA1) {
    pa0 = *reinterpret_cast<const float4*>(a1b + a1src[0] + 104 * c0);
    pa1 = *reinterpret_cast<const float4*>(a1b + a1src[1] + 104 * c0);
    pa2 = *reinterpret_cast<const float4*>(a1b + a1src[2] + 104 * c0);
  }
  if constexpr (!kA1) {
    const float4 xv = reinterpret_cast<const float4*>(f.x + b * 784)[min(tid, 195)];
    const float wv = tid < 144 ? f.p[L::w1 + 144 * h + tid] : f.p[L::b1 + 16 * h + min(tid - 144, 15)];
    if (tid < 196) *reinterpret_cast<float4*>(xs + 4 * tid) = xv;
    if (tid < 160) w1s[tid] = wv;
  }
  const int co = 16 * ct + m;  // A row of this lane
  const float* dpl = f.dp + (size_t)b * 9216 + co * 144 + 6 * g;
  const uint16_t* qpl = reinterpret_cast<const uint16_t*>(reinterpret_cast<const uint8_t*>(f.idx) + (size_t)b * 9216 + co * 144 + 6 * g);
  float2 dn[3];
  uint16_t qn[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    dn[k] = *reinterpret_cast<const float2*>(dpl + 24 * c0 + 2 * k);
    qn[k] = qpl[12 * c0 + k];
  }
  f32x4 acc[4 * kNI];
#pragma unroll
  for (int x = 0; x < 4 * kNI; ++x) acc[x] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  MX_TRACE_B(f, 3, 1, braw);
  float w1b[3];  // conv1 B fragments: tap 4ks + g of channel m (taps 9..11 are padding)
#pragma unroll
  for (int ks = 0; ks < 3; ++ks) w1b[ks] = 4 * ks + g < 9 ? w1s[m * 9 + 4 * ks + g] : 0.f;
  const float b1v = w1s[144 + m];
  uint32_t tA = 0, tB = 0, tC = 0, tq = 0;  // phase-time sums (trace only)
  const bool trc = f.trace && threadIdx.x == 0 && braw < 1024;
#pragma unroll 1
  for (int c = c0; c < c0 + 6 / kF6WSplit; ++c) {
    if (trc) tq = (uint32_t)__builtin_amdgcn_s_memrealtime();
    if constexpr (kA1) {  // (A) published a1 rows -> LDS; next chunk's rows in flight
      *reinterpret_cast<float4*>(a1s + a1dst[0]) = pa0;
      *reinterpret_cast<float4*>(a1s + a1dst[1]) = pa1;
      if (a1dst[2] >= 0) *reinterpret_cast<float4*>(a1s + a1dst[2]) = pa2;
      if (c + 1 < c0 + 6 / kF6WSplit) {
        const float* nb = a1b + 104 * (c + 1);
        pa0 = *reinterpret_cast<const float4*>(nb + a1src[0]);
        pa1 = *reinterpret_cast<const float4*>(nb + a1src[1]);
        pa2 = *reinterpret_cast<const float4*>(nb + a1src[2]);
      }
    }
    // (A) a1 rows 4c .. 4c+5 (x rows 4c .. 4c+7 <= 27) for the 16 ci on MFMA: M = 156 positions
    // (10 tiles of 16, wave w takes tiles w, w+4, w+8), N = 16 ci, K = 9 taps padded to 12
    if constexpr (!kA1)
    for (int mt = w; mt < 10; mt += 4) {
      const int p = min(16 * mt + m, 155), r = p / 26, col = p - 26 * r;
      const float* xp = xs + (4 * c + r) * 28 + col;
      f32x4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        const int t = 4 * ks + g;
        const float av = t < 9 ? xp[(t / 3) * 28 + t % 3] : 0.f;
        a = mfma4(av, w1b[ks], a);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = 16 * mt + 4 * g + j;
        if (q < 156) a1s[m * kA1P + q] = fmaxf(a[j] + b1v, 0.f);
      }
    }
    __syncthreads();
    if (trc) {
      const uint32_t t = (uint32_t)__builtin_amdgcn_s_memrealtime();
      tA += t - tq;
      tq = t;
    }
    // (B) V = B^T d B of 24 tiles x 16 ci; tile tl: a1 rows 2(tl/12).., cols 2(tl%12)..
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = tid + 256 * k;
      if (i < 384) {
        const int ci = i & 15, tl = i >> 4, tyl = tl / 12, tx = tl - 12 * tyl;
        const float* ap = a1s + ci * kA1P + 2 * tyl * 26 + 2 * tx;
        float d[4][4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int cc = 0; cc < 4; ++cc) d[r][cc] = ap[r * 26 + cc];
        float e[4][4];
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
          e[0][cc] = d[0][cc] - d[2][cc];
          e[1][cc] = d[1][cc] + d[2][cc];
          e[2][cc] = d[2][cc] - d[1][cc];
          e[3][cc] = d[1][cc] - d[3][cc];
        }
        float4* vp = reinterpret_cast<float4*>(vs + (tl * 16 + ci) * kF6WVP);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          vp[r] = make_float4(e[r][0] - e[r][2], e[r][1] + e[r][2], e[r][2] - e[r][1], e[r][1] - e[r][3]);
      }
    }
    // this chunk's dp / q operands; prefetch the next chunk's
    float dv[6];
    uint32_t qv[6];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      dv[2 * k] = dn[k].x;
      dv[2 * k + 1] = dn[k].y;
      qv[2 * k] = qn[k] & 0xffu;
      qv[2 * k + 1] = qn[k] >> 8;
    }
    if (c + 1 < c0 + 6 / kF6WSplit) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        dn[k] = *reinterpret_cast<const float2*>(dpl + 24 * (c + 1) + 2 * k);
        qn[k] = qpl[12 * (c + 1) + k];
      }
    }
    __syncthreads();
    if (trc) {
      const uint32_t t = (uint32_t)__builtin_amdgcn_s_memrealtime();
      tB += t - tq;
      tq = t;
    }
    // (C) k-step s: tile t = 6g + s of the chunk
#pragma unroll
    for (int s = 0; s < 6; ++s) {
      const float4* vp = reinterpret_cast<const float4*>(vs + ((6 * g + s) * 16 + m) * kF6WVP) + kNI * xh;
      float4 bb[kNI];
#pragma unroll
      for (int i = 0; i < kNI; ++i) bb[i] = vp[i];
      const float v = dv[s];
      const bool qy = (qv[s] >> 1) & 1, qx = qv[s] & 1;
      const float vy4[4] = {qy ? 0.f : v, v, qy ? -v : v, qy ? -v : 0.f};
      float vy[kNI];
#pragma unroll
      for (int i = 0; i < kNI; ++i) vy[i] = kCoS == 1 ? vy4[i] : (xh ? vy4[2 + i] : vy4[i]);
#pragma unroll
      for (int i = 0; i < kNI; ++i) {
        const float w0 = qx ? 0.f : vy[i], w2 = qx ? -vy[i] : vy[i], w3 = qx ? -vy[i] : 0.f;
        acc[4 * i + 0] = mfma4(w0, bb[i].x, acc[4 * i + 0]);
        acc[4 * i + 1] = mfma4(vy[i], bb[i].y, acc[4 * i + 1]);
        acc[4 * i + 2] = mfma4(w2, bb[i].z, acc[4 * i + 2]);
        acc[4 * i + 3] = mfma4(w3, bb[i].w, acc[4 * i + 3]);
      }
    }
    if (trc) tC += (uint32_t)__builtin_amdgcn_s_memrealtime() - tq;  // issue time of (C)
  }
  MX_TRACE_B(f, 3, 2, braw);
  // dw = G^T dU G, G^T = [1 .5 .5 0; 0 .5 -.5 0; 0 .5 .5 1]; acc[4i + j'][j] = dU[i][j'] of
  // (co = 16w + 4g + j, ci = 16h + m)
  const int ci = 16 * h + m;
  float* wa = sc.wacc + (b & (kWaccSlabs - 1)) * kPack;
  if constexpr (kCoS == 2) {
    // partial G^T dU G of this wave's two Winograd rows: t[ky][jj] over rows (m0, m1) = i 0, 1 or
    // (m2, m3) = i 2, 3 of G^T = [1 .5 .5 0; 0 .5 -.5 0; 0 .5 .5 1]
    float o[4][9];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float t[3][4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const float ma = acc[jj][j], mb = acc[4 + jj][j];
        if (xh == 0) {
          t[0][jj] = ma + 0.5f * mb;
          t[1][jj] = 0.5f * mb;
          t[2][jj] = 0.5f * mb;
        } else {
          t[0][jj] = 0.5f * ma;
          t[1][jj] = -0.5f * ma;
          t[2][jj] = 0.5f * ma + mb;
        }
      }
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        o[j][ky * 3 + 0] = t[ky][0] + 0.5f * (t[ky][1] + t[ky][2]);
        o[j][ky * 3 + 1] = 0.5f * (t[ky][1] - t[ky][2]);
        o[j][ky * 3 + 2] = 0.5f * (t[ky][1] + t[ky][2]) + t[ky][3];
      }
    }
    // wave xh finalises co rows j = 2xh, 2xh+1 of its lanes; hands the other two to its partner
    // (wave w ^ 2, same co tile) through LDS over vs: [4 w][2 jl][9 tap][64 lane]
    __syncthreads();  // every wave's phase-C reads of vs are done
    float* xch = vs;
#pragma unroll
    for (int jl = 0; jl < 2; ++jl)
#pragma unroll
      for (int k = 0; k < 9; ++k) xch[((w * 2 + jl) * 9 + k) * 64 + lane] = o[xh ? jl : 2 + jl][k];
    __syncthreads();
    const int pw = w ^ 2;
    if (f.wslab) {
      // slab epilogue (as the unsplit blocks): this block's [32 co][16 ci][9] half of the image's
      // slab staged in LDS over the exchange buffer, then coalesced 16-byte stores, no atomics
      float fin[2][9];
#pragma unroll
      for (int jl = 0; jl < 2; ++jl)
#pragma unroll
        for (int k = 0; k < 9; ++k) fin[jl][k] = o[2 * xh + jl][k] + xch[((pw * 2 + jl) * 9 + k) * 64 + lane];
      __syncthreads();  // every partner read of the exchange buffer is done
      float* st = sm;   // [32 co of this half][16 ci][9]
#pragma unroll
      for (int jl = 0; jl < 2; ++jl) {
        const int cl = 16 * (w & 1) + 4 * g + 2 * xh + jl;
#pragma unroll
        for (int k = 0; k < 9; ++k) st[(cl * 16 + m) * 9 + k] = fin[jl][k];
      }
      __syncthreads();
      const int chalf = (bid >> 1) & 1;
      const float4* s4 = reinterpret_cast<const float4*>(st);
      float4* d4 = reinterpret_cast<float4*>(sc.wslab + (size_t)b * kPack + 144 * h);
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const int i = tid + 256 * k, col = i / 36, q = i - 36 * col;
        if (i < 32 * 36) d4[(32 * chalf + col) * 72 + q] = s4[i];
      }
    } else {
#pragma unroll
      for (int jl = 0; jl < 2; ++jl) {
        const int j = 2 * xh + jl, cj = 16 * ct + 4 * g + j;
#pragma unroll
        for (int k = 0; k < 9; ++k)
          atomicAdd(wa + (k * 64 + cj) * 32 + ci, o[j][k] + xch[((pw * 2 + jl) * 9 + k) * 64 + lane]);
      }
    }
  } else {
  // f.wslab (kF6WSplit == 1): this block's [64 co][16 ci][9] result is staged in LDS (over the
  // idle operand tiles) and written to the image's slab in canonical [co][ci][ky][kx] order with
  // coalesced 16-byte stores -- no atomics (the atomic epilogue was ~3 us and delayed the F7
  // blocks' own atomics behind it); the finalize sums the B slabs in a fixed order
  const bool slab = kF6WSplit == 1 && f.wslab;
  float* st = sm;  // [64 co][16 ci][9]
  if (slab) __syncthreads();  // every wave's phase-C reads of the operand tiles are done
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int cj = 16 * w + 4 * g + j;
    float t[3][4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const float m0 = acc[jj][j], m1 = acc[4 + jj][j], m2 = acc[8 + jj][j], m3 = acc[12 + jj][j];
      t[0][jj] = m0 + 0.5f * (m1 + m2);
      t[1][jj] = 0.5f * (m1 - m2);
      t[2][jj] = 0.5f * (m1 + m2) + m3;
    }
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const float o0 = t[ky][0] + 0.5f * (t[ky][1] + t[ky][2]);
      const float o1 = 0.5f * (t[ky][1] - t[ky][2]);
      const float o2 = 0.5f * (t[ky][1] + t[ky][2]) + t[ky][3];
      if (slab) {
        float* sp = st + (cj * 16 + m) * 9 + 3 * ky;
        sp[0] = o0;
        sp[1] = o1;
        sp[2] = o2;
      } else {
        atomicAdd(wa + ((ky * 3 + 0) * 64 + cj) * 32 + ci, o0);
        atomicAdd(wa + ((ky * 3 + 1) * 64 + cj) * 32 + ci, o1);
        atomicAdd(wa + ((ky * 3 + 2) * 64 + cj) * 32 + ci, o2);
      }
    }
  }
  if (slab) {
    __syncthreads();
    // per co: 16 ci x 9 taps = 144 contiguous floats (36 float4) at (co * 32 + 16 h) * 9
    const float4* s4 = reinterpret_cast<const float4*>(st);
    float4* d4 = reinterpret_cast<float4*>(sc.wslab + (size_t)b * kPack + 144 * h);
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int i = tid + 256 * k, co = i / 36, q = i - 36 * co;
      d4[co * 72 + q] = s4[i];
    }
  }
  }
  MX_TRACE_B(f, 3, 3, braw);
  if (trc) {  // phase-time sums as "time after block start" in trace slots 4..6 (A, B, C)
    const uint32_t t0 = f.trace[(3 * 1024 + braw) * 8];
    f.trace[(3 * 1024 + braw) * 8 + 4] = t0 + tA;
    f.trace[(3 * 1024 + braw) * 8 + 5] = t0 + tB;
    f.trace[(3 * 1024 + braw) * 8 + 6] = t0 + tC;
  }
}

// ------------------------------------------------------------------------------------------
// F7: conv2 data grad + conv1 ReLU mask + conv1 weight/bias grad (+ wacc -> conv2.weight grad).
// GEMM: M = 64 input positions of image b per block (4 M-tiles -> waves), N = 32 ci,
// K = (r, co) = 576.  A = dY2[co][iy-ky][ix-kx] expanded from the compact pooled tiles in LDS:
// 4 pooled rows x 14 window columns (a dead halo of one window on each side, so no bounds
// checks), channel pitch 60 words (lane groups 16 banks apart).  B = pre-packed conv2 weight
// fragments from L2, prefetched one tap ahead.  The epilogue masks with a1 > 0 (conv1
// recomputed from x and w1 in LDS: a1 is never stored) and contracts
// with the 3x3 patches of x (LDS): dW1[ci][r] and db1[ci] are reduced in registers ->
// cross-lane -> LDS -> one atomic per value per block.  dA1 never touches HBM.
constexpr int kF7WR = 4, kF7WC = 14, kF7CoP = 60;
constexpr size_t kF7Lds = sizeof(float) * (64 * kF7CoP + 784 + 320 + 1280) + 64 * kF7CoP;
__device__ __forceinline__ void f7_body(const MnistFused& f, const Scratch& sc, float* sm, int braw, int nblk) {
  MX_TRACE_B(f, 4, 0, braw);
  float* dps = sm;                                                  // [64][60] (4 x 14 used)
  float* xs = dps + 64 * kF7CoP;                                    // [784]
  float* w1s = xs + 784;                                            // conv1 w [32][9], b [32]
  float* red = w1s + 320;                                           // [4][32][10]
  uint8_t* qs = reinterpret_cast<uint8_t*>(red + 1280);             // [64][60]
  const int bid = xcd_remap(braw, nblk);  // an image's 11 blocks share one XCD L2
  const int b = bid / 11, chunk = bid - b * 11;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, m = lane & 15;
  const uint8_t* idx = reinterpret_cast<const uint8_t*>(f.idx) + (size_t)b * 9216;
  const float* dpb = f.dp + (size_t)b * 9216;
  const int p0 = chunk * 64;
  const int row0 = p0 / 26 - 2;           // first conv2-output row any tap of this chunk reads
  const int wy0 = row0 >> 1;              // first pooled row staged (arithmetic shift: -1 ok)
  {
    float dv[14];
    uint32_t qv[14];
#pragma unroll
    for (int k = 0; k < 14; ++k) {  // 64 co x 4 x 14 = 3584 = 14 x 256
      const int i = tid + 256 * k, co = i / (kF7WR * kF7WC), rem = i - co * (kF7WR * kF7WC);
      const int wyl = rem / kF7WC, wx = rem - wyl * kF7WC - 1, wy = wy0 + wyl;
      // unconditional (clamped) loads: a select around a load would make hipcc branch and
      // drain vmcnt per element; the halo is applied after all loads are in flight
      const int o = co * 144 + min(max(wy, 0), 11) * 12 + min(max(wx, 0), 11);
      dv[k] = dpb[o];
      qv[k] = idx[o];
    }
    float xv[4], wv2[2];
#pragma unroll
    for (int k = 0; k < 4; ++k) xv[k] = f.x[b * 784 + min(tid + 256 * k, 783)];
#pragma unroll
    for (int k = 0; k < 2; ++k) wv2[k] = f.p[L::w1 + min(tid + 256 * k, 319)];
#pragma unroll
    for (int k = 0; k < 14; ++k) {
      const int i = tid + 256 * k, co = i / (kF7WR * kF7WC), rem = i - co * (kF7WR * kF7WC);
      const int wyl = rem / kF7WC, wx = rem - wyl * kF7WC - 1, wy = wy0 + wyl;
      const bool ok = wy >= 0 && wy < 12 && wx >= 0 && wx < 12;
      dps[co * kF7CoP + rem] = ok ? dv[k] : 0.f;
      qs[co * kF7CoP + rem] = ok ? (uint8_t)qv[k] : (uint8_t)4;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (tid + 256 * k < 784) xs[tid + 256 * k] = xv[k];
#pragma unroll
    for (int k = 0; k < 2; ++k)
      if (tid + 256 * k < 320) w1s[tid + 256 * k] = wv2[k];
  }
  __syncthreads();
  MX_TRACE_B(f, 4, 1, braw);
  const int pos = min(p0 + 16 * w + m, 675);  // this lane's A row (clamped tail rows are discarded)
  const int iy = pos / 26, ix = pos - iy * 26;
  const float4* wd = reinterpret_cast<const float4*>(sc.wd) + lane;
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  float4 bc[8], bn[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) bc[i] = wd[i * 64];
#pragma unroll 1
  for (int r = 0; r < 9; ++r) {
    if (r < 8) {
#pragma unroll
      for (int i = 0; i < 8; ++i) bn[i] = wd[((r + 1) * 8 + i) * 64];
    }
    const int ky = r / 3, kx = r - 3 * ky;
    const int oy = iy - ky, ox = ix - kx;               // may be -2..-1 or 24..25: dead halo
    const int wb = ((oy >> 1) - wy0) * kF7WC + (ox >> 1) + 1 + 4 * g * kF7CoP;
    const uint32_t tgt = (uint32_t)(((oy & 1) << 1) | (ox & 1));
    const float* dpp = dps + wb;
    const uint8_t* qp = qs + wb;
    // All 32 LDS reads of this tap first, unconditionally; the expansion is a multiply by
    // the 0/1 match (a select around a load lets hipcc turn it into a serialised,
    // predicated read -> one LDS round trip per MFMA pair).
    float dv[16];
    uint32_t qv[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int co_off = (16 * (k >> 2) + (k & 3)) * kF7CoP;  // co = 16s + 4g + j
      dv[k] = dpp[co_off];
      qv[k] = qp[co_off];
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float a = dv[4 * s + j] * (float)(qv[4 * s + j] == tgt);
        acc[0] = mfma4(a, sel4(bc[2 * s], j), acc[0]);
        acc[1] = mfma4(a, sel4(bc[2 * s + 1], j), acc[1]);
      }
#pragma unroll
    for (int i = 0; i < 8; ++i) bc[i] = bn[i];
  }
  MX_TRACE_B(f, 4, 2, braw);
  // epilogue: acc[c][j] = dA1 at position p = p0 + 16w + 4g + j, channel ci = 16c + m
  float part[2][10];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int k = 0; k < 10; ++k) part[c][k] = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int p = p0 + 16 * w + 4 * g + j;
    if (p < 676) {
      const int py = p / 26, px = p - py * 26;
      const float* xp = xs + py * 28 + px;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int ci = 16 * c + m;
        float a1v = w1s[288 + ci];  // conv1 pre-activation at p, recomputed (a1 is not stored)
#pragma unroll
        for (int k = 0; k < 9; ++k) a1v = fmaf(xp[(k / 3) * 28 + k % 3], w1s[ci * 9 + k], a1v);
        const float gv = a1v > 0.f ? acc[c][j] : 0.f;
        part[c][9] += gv;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) part[c][ky * 3 + kx] = fmaf(gv, xp[ky * 28 + kx], part[c][ky * 3 + kx]);
      }
    }
  }
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
      for (int k = 0; k < 10; ++k) red[(w * 32 + 16 * c + m) * 10 + k] = part[c][k];
  }
  __syncthreads();
  // one of 8 partial slabs (image & 7: 88 blocks per address instead of all 704 hammering
  // the same 320 words: same-address float atomics serialise at the memory side)
  float* g1 = sc.g1 + (b & g1_slab_mask(f)) * 320;
  for (int i = tid; i < 320; i += 256) {
    const float v = red[i] + red[320 + i] + red[640 + i] + red[960 + i];
    const int ci = i / 10, k = i - ci * 10;
    if (k < 9) atomicAdd(g1 + ci * 9 + k, v);  // conv1.weight grad [32][9]
    else atomicAdd(g1 + 288 + ci, v);          // conv1.bias grad [32]
  }
  MX_TRACE_B(f, 4, 3, braw);
}

// ------------------------------------------------------------------------------------------
// F7W: the same data gradient (+ conv1 mask / weight grads) as Winograd F(2x2,3x3) on fp32 MFMA:
// 2.25x fewer MFMAs.  dA1 (26x26) = full correlation of dY2 with the flipped filter, in 13x13
// output tiles of 2x2.  Tile (ty, tx) reads the 4x4 patch of zero-padded dY2 at rows 2ty-2..2ty+1,
// cols 2tx-2..2tx+1 = exactly the 2x2 pool windows (ty-1..ty, tx-1..tx), each holding ONE nonzero
// (its argmax), so the input transform V = B^T d B is built from 4 (value, code) pairs straight
// out of the compact LDS tiles.  16 GEMMs (one per Winograd point xi, K = 64 co) share one MFMA
// fragment layout, so the output transform A^T M A of a (tile, ci) is lane-local.
// Block = (image, chunk of 32 tiles); wave w = (M-group w&1: 16 tiles, ci half w>>1: 16 ci);
// 16 k-steps of 4 co x 16 xi MFMAs.  B fragments (G w' G^T, written by F2) stream from L2 one
// k-step ahead.  Epilogue as F7: conv1 recomputed for the ReLU mask, conv1 weight/bias grads
// reduced in registers -> lanes -> LDS -> slab atomics (slab = image & 7).
constexpr int kF7WChunks = 6, kF7WRows = 5, kF7WCols = 14, kF7WCoP = 80;
constexpr size_t kF7WLds = sizeof(float) * (64 * kF7WCoP + 784 + 320 + 640) + 64 * kF7WCoP;
// kVq: the (value, code) LDS operands of k-step s + 1 are loaded during k-step s (the step's
// scheduling barrier otherwise keeps every step waiting for its own LDS reads)
template <bool kVq = false>
__device__ __forceinline__ void f7w_body(const MnistFused& f, const Scratch& sc, float* sm, int braw, int nblk) {
  MX_TRACE_B(f, 4, 0, braw);
  float* dps = sm;                                      // [64 co][80]: 5 window rows x 14 cols
  float* xs = dps + 64 * kF7WCoP;                       // [784]
  float* w1s = xs + 784;                                // conv1 w [32][9], b [32]
  float* red = w1s + 320;                               // [2 M-groups][32 ci][10]
  uint8_t* qs = reinterpret_cast<uint8_t*>(red + 640);  // [64 co][80] argmax codes
  const int bid = xcd_remap(braw, nblk);  // an image's 6 blocks share one XCD L2
  const int b = bid / kF7WChunks, chunk = bid - b * kF7WChunks;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, m = lane & 15;
  const int mg = w & 1, half = w >> 1;
  const int t0 = 32 * chunk, tyf = t0 / 13;  // first tile row of the chunk
  const int wy0 = tyf - 1;                   // first window row staged (may be -1: halo)
  {
    // per co the 5 staged window rows are 60 contiguous floats of dp (rows of 12): 15 float4 /
    // uint32 (4 argmax codes) granules; rows outside 0..11 and the halo columns become zeros
    const float4* dpb = reinterpret_cast<const float4*>(f.dp + (size_t)b * 9216);
    const uint32_t* qb = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(f.idx) + (size_t)b * 9216);
    constexpr int kN = 64 * kF7WRows * 3, kIt = (kN + 255) / 256;  // 960 granules -> 4
    float4 dv[kIt];
    uint32_t qv[kIt];
#pragma unroll
    for (int k = 0; k < kIt; ++k) {  // clamped unconditional loads, halo applied afterwards
      const int i = min(tid + 256 * k, kN - 1), co = i / (kF7WRows * 3), rem = i - co * (kF7WRows * 3);
      const int wyl = rem / 3, c4 = rem - wyl * 3, wy = min(max(wy0 + wyl, 0), 11);
      const int o = co * 36 + wy * 3 + c4;  // float4 granule index
      dv[k] = dpb[o];
      qv[k] = qb[o];
    }
    const float4 xv = reinterpret_cast<const float4*>(f.x + b * 784)[min(tid, 195)];
    const float4 wv = reinterpret_cast<const float4*>(f.p + L::w1)[min(tid, 79)];
#pragma unroll
    for (int k = 0; k < kIt; ++k) {
      const int i = tid + 256 * k;
      if (i < kN) {
        const int co = i / (kF7WRows * 3), rem = i - co * (kF7WRows * 3);
        const int wyl = rem / 3, c4 = rem - wyl * 3, wy = wy0 + wyl;
        const bool ok = wy >= 0 && wy < 12;
        float* dd = dps + co * kF7WCoP + wyl * kF7WCols + 1 + 4 * c4;  // staged column wx + 1
        uint8_t* qd = qs + co * kF7WCoP + wyl * kF7WCols + 1 + 4 * c4;
        const float4 v = dv[k];
        dd[0] = ok ? v.x : 0.f;
        dd[1] = ok ? v.y : 0.f;
        dd[2] = ok ? v.z : 0.f;
        dd[3] = ok ? v.w : 0.f;
        const uint32_t q = ok ? qv[k] : 0x04040404u;
        qd[0] = (uint8_t)q;
        qd[1] = (uint8_t)(q >> 8);
        qd[2] = (uint8_t)(q >> 16);
        qd[3] = (uint8_t)(q >> 24);
        if (c4 == 0) {  // halo columns -1 and 12
          dd[-1] = 0.f;
          qd[-1] = 4;
        } else if (c4 == 2) {
          dd[4] = 0.f;
          qd[4] = 4;
        }
      }
    }
    if (tid < 196) *reinterpret_cast<float4*>(xs + 4 * tid) = xv;
    if (tid < 80) *reinterpret_cast<float4*>(w1s + 4 * tid) = wv;
  }
  __syncthreads();
  MX_TRACE_B(f, 4, 1, braw);
  f32x4 acc[16];
#pragma unroll
  for (int x = 0; x < 16; ++x) acc[x] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (t0 + 16 * mg < 169) {  // the last chunk's second M-group has no tile
    const int tl = min(t0 + 16 * mg + m, 168);  // A row of this lane (clamped rows are discarded)
    const int ty = tl / 13, tx = tl - 13 * ty;
    // window (ty-1, tx-1) sits at staged row ty-1-wy0 = ty-tyf, column tx-1+1 = tx
    const float* dpp = dps + (ty - tyf) * kF7WCols + tx + g * kF7WCoP;
    const uint8_t* qp = qs + (ty - tyf) * kF7WCols + tx + g * kF7WCoP;
    const float4* wu = reinterpret_cast<const float4*>(sc.wu) + (half * 64 + lane) * 4;
    // fully unrolled; B fragments prefetched kF7WPf k-steps ahead (indices fold to registers)
    constexpr int kF7WPf = 2;
    constexpr bool kF7WPin = true;
    float4 bq[16][4];
#pragma unroll
    for (int s = 0; s < kF7WPf; ++s)
#pragma unroll
      for (int k = 0; k < 4; ++k) bq[s][k] = wu[s * 512 + k];
    float vn[4];
    uint32_t qn[4];
    if constexpr (kVq) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int o = (k >> 1) * kF7WCols + (k & 1);
        vn[k] = dpp[o];
        qn[k] = qp[o];
      }
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s + kF7WPf < 16) {
#pragma unroll
        for (int k = 0; k < 4; ++k) bq[s + kF7WPf][k] = wu[(s + kF7WPf) * 512 + k];
      }
      float v[4];
      uint32_t q[4];
      if constexpr (kVq) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[k] = vn[k];
          q[k] = qn[k];
        }
        if (s + 1 < 16) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int o = 4 * (s + 1) * kF7WCoP + (k >> 1) * kF7WCols + (k & 1);
            vn[k] = dpp[o];
            qn[k] = qp[o];
          }
        }
      }
      // keep the prefetch at the top of the step: left alone the scheduler sinks these loads
      // next to their use and every k-step then waits for L2 (vmcnt(0)) before its MFMAs
      if (kF7WPin) __builtin_amdgcn_sched_barrier(0);
      const float4* bc = bq[s];
      const int off = 4 * s * kF7WCoP;  // co = 4s + g
      if constexpr (!kVq) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // windows (a, c) = (k>>1, k&1) at +a*14 + c
          const int o = off + (k >> 1) * kF7WCols + (k & 1);
          v[k] = dpp[o];
          q[k] = qp[o];
        }
      }
      // d[r][c] = nonzero of window (r>>1, c>>1) if its argmax code is 2*(r&1) + (c&1)
      float d[4][4];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int k = (r >> 1) * 2 + (c >> 1);
          d[r][c] = q[k] == (uint32_t)(((r & 1) << 1) | (c & 1)) ? v[k] : 0.f;
        }
      // V = B^T d B, B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1]
      float e[4][4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        e[0][c] = d[0][c] - d[2][c];
        e[1][c] = d[1][c] + d[2][c];
        e[2][c] = d[2][c] - d[1][c];
        e[3][c] = d[1][c] - d[3][c];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v0 = e[i][0] - e[i][2], v1 = e[i][1] + e[i][2], v2 = e[i][2] - e[i][1], v3 = e[i][1] - e[i][3];
        acc[4 * i + 0] = mfma4(v0, bc[i].x, acc[4 * i + 0]);
        acc[4 * i + 1] = mfma4(v1, bc[i].y, acc[4 * i + 1]);
        acc[4 * i + 2] = mfma4(v2, bc[i].z, acc[4 * i + 2]);
        acc[4 * i + 3] = mfma4(v3, bc[i].w, acc[4 * i + 3]);
      }
    }
  }
  MX_TRACE_B(f, 4, 2, braw);
  // epilogue: acc[xi][j] = Winograd-domain dA1 of tile t0 + 16mg + 4g + j, channel ci = 16half + m
  const int ci = 16 * half + m;
  float wk[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) wk[k] = w1s[ci * 9 + k];
  const float bk = w1s[288 + ci];
  float part[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) part[k] = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int t = t0 + 16 * mg + 4 * g + j;
    if (t < 169) {
      const int ty = t / 13, tx = t - 13 * ty;
      // Y = A^T M A, A^T = [1 1 1 0; 0 1 -1 -1]
      float p0[4], p1[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        p0[c] = acc[c][j] + acc[4 + c][j] + acc[8 + c][j];
        p1[c] = acc[4 + c][j] - acc[8 + c][j] - acc[12 + c][j];
      }
      float y[2][2];
      y[0][0] = p0[0] + p0[1] + p0[2];
      y[0][1] = p0[1] - p0[2] - p0[3];
      y[1][0] = p1[0] + p1[1] + p1[2];
      y[1][1] = p1[1] - p1[2] - p1[3];
      float xp[4][4];  // x patch rows 2ty.., cols 2tx.. (the 3x3 conv1 windows of the 4 outputs)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) xp[r][c] = xs[(2 * ty + r) * 28 + 2 * tx + c];
#pragma unroll
      for (int py = 0; py < 2; ++py)
#pragma unroll
        for (int px = 0; px < 2; ++px) {
          float a1v = bk;  // conv1 pre-activation (a1 is not stored)
#pragma unroll
          for (int k = 0; k < 9; ++k) a1v = fmaf(xp[py + k / 3][px + k % 3], wk[k], a1v);
          const float gv = a1v > 0.f ? y[py][px] : 0.f;
          part[9] += gv;
#pragma unroll
          for (int k = 0; k < 9; ++k) part[k] = fmaf(gv, xp[py + k / 3][px + k % 3], part[k]);
        }
    }
  }
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    float v = part[k];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    part[k] = v;
  }
  if (g == 0) {
#pragma unroll
    for (int k = 0; k < 10; ++k) red[(mg * 32 + ci) * 10 + k] = part[k];
  }
  __syncthreads();
  float* g1 = sc.g1 + (b & g1_slab_mask(f)) * 320;
  for (int i = tid; i < 320; i += 256) {
    const float v = red[i] + red[320 + i];
    const int c = i / 10, k = i - c * 10;
    if (k < 9) atomicAdd(g1 + c * 9 + k, v);
    else atomicAdd(g1 + 288 + c, v);
  }
  MX_TRACE_B(f, 4, 3, braw);
}

// ------------------------------------------------------------------------------------------
// F6 + F7 in ONE launch: blocks [0, 9B) run the weight gradient, the rest the data gradient.
// The two are independent; sharing a grid lets the dispatcher backfill CUs as blocks retire
// (576 + 704 blocks over 256 CUs at 3 per CU), so one kernel's prologue/epilogue latency and
// the 2-vs-3-blocks-per-CU imbalance of each kernel alone are covered by the other's MFMA work.
// 9B is a multiple of 8, so the F7 part keeps its XCD-aware block mapping.
//
// Co-scheduled gradient exchange (f.co_blocks > 0): the first co_blocks blocks run the two-shot
// peer all-reduce of the fc bucket (complete since F5) instead -- dispatched first, they wait on
// the peers' matching blocks while the remaining blocks do the conv backward, so the 4.7 MB
// exchange overlaps it inside ONE launch (no side stream, no cross-queue fence).  co_blocks is
// a multiple of 8, so the conv part keeps its XCD-aware block mapping.
template <bool kWino, int kF6WSplit = 1, bool kA1 = false, int kCoS = 1, bool kVq = false>
__global__ __launch_bounds__(256, 3) void f67_conv2_bwd_kernel(MnistFused f, Scratch sc) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  if ((int)blockIdx.x < f.co_blocks) {
    MX_TRACE_B(f, 5, 0, (int)blockIdx.x);  // trace: exchange blocks vs conv blocks of this launch
    peer_two_shot_f32_block(f.co_args, f.co_part, blockIdx.x, reinterpret_cast<uint32_t*>(sm));
    MX_TRACE_B(f, 5, 1, (int)blockIdx.x);
    return;
  }
  const int bid = (int)blockIdx.x - f.co_blocks;
  const int n6 = (kWino ? 2 * kF6WSplit * kCoS : 9) * f.B;
  if (bid < n6) {
    if (kWino)
      f6w_body<kF6WSplit, kA1, kCoS>(f, sc, sm, bid, n6);
    else
      f6_body(f, sc, sm, bid, n6);
  } else if (kWino) {
    f7w_body<kVq>(f, sc, sm, bid - n6, kF7WChunks * f.B);
  } else {
    f7_body(f, sc, sm, bid - n6, 11 * f.B);
  }
}

// ------------------------------------------------------------------------------------------
// F8: finalize bucket 1: conv2.weight grad = transpose of the [r][co][ci] accumulator into
// the canonical [co][ci][ky][kx] layout; conv1 weight/bias grads = sum over the per-image
// partial slabs (and the conv2 accumulator slabs).  The accumulators g1 and the fc1 split-K h
// are reset here for the next step (the wacc slabs by the next F3): no memset launches.
// Blocks 0..71: wacc transpose (256 outputs each).  Blocks 72..73: the 8-slab sum, one output
// per thread.  Blocks 74..: zero h.
constexpr int kF8Wacc = kPack / 256, kF8G1 = 2;
__global__ __launch_bounds__(256) void f8_finalize_kernel(MnistFused f, Scratch sc) {
  __shared__ float red[576 + 36];
  const int tid = threadIdx.x;
  int blk = blockIdx.x;
  if (f.wslab) {  // blocks 0 .. 511: the fixed-order slab sum, 4 (co, ci) pairs each
    if (blk < kWslabGroups) {
      wslab_group_sum(f, sc, blk, red, red + 576);
      if (tid < 36) f.g[L::w2 + 36 * blk + tid] = red[576 + tid];
      return;
    }
    blk += kF8Wacc - kWslabGroups;  // the remaining blocks as in the atomic layout
  }
  if (blk < kF8Wacc) {
    const int i = blk * 256 + tid;
    const int co = i / 288, rem = i - co * 288, ci = rem / 9, rr = rem - ci * 9;
    float* a = sc.wacc + (rr * 64 + co) * 32 + ci;
    float v[kWaccSlabs];
#pragma unroll
    for (int k = 0; k < kWaccSlabs; ++k) v[k] = a[k * kPack];
    float s = v[0];
#pragma unroll
    for (int k = 1; k < kWaccSlabs; ++k) s += v[k];
    f.g[L::w2 + i] = s;  // (F3 of the next step zeroes the slabs)
  } else if (blk < kF8Wacc + kF8G1) {
    const int j = (blk - kF8Wacc) * 256 + tid;  // conv1 w/b grads: fixed-order sum of the slabs
    if (j < 320) {
      const int ns = g1_slab_mask(f) + 1;
      float s = 0.f;
      for (int k0 = 0; k0 < ns; k0 += 16) {  // 16 loads in flight, fixed order
        float v[16];  // clamped loads, masked adds: no load behind a branch
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = sc.g1[min(k0 + k, ns - 1) * 320 + j];
#pragma unroll
        for (int k = 0; k < 16; ++k) s += k0 + k < ns ? v[k] : 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k)
          if (k0 + k < ns) sc.g1[(k0 + k) * 320 + j] = 0.f;
      }
      f.g[L::w1 + j] = s;
    }
  } else {
    for (int i = (blk - kF8Wacc - kF8G1) * 256 + tid; i < f.B * 128; i += 8 * 256) f.h[i] = 0.f;
  }
}

}  // namespace
}  // namespace mnist

using namespace mnist;

// F7 variant: Winograd (default) or direct implicit GEMM (MXDDP_MNIST_F7=direct); Winograd
// weight-gradient blocks per (image, ci half): MXDDP_F6W_SPLIT = 1 (default: 748k img/s; 2: 725k,
// 3: 695k -- more blocks double the weight-gradient atomics and slow the F7W blocks).
bool mnist_a1_publish() {
  static const int v = [] {
    const char* e = std::getenv("MXDDP_MNIST_A1");
    return (e && std::string(e) == "recompute") ? 0 : 1;
  }();
  return v == 1;
}
bool mnist_f5_sgd() {
  static const int v = [] {
    const char* e = std::getenv("MXDDP_F5_SGD");
    return (e && std::string(e) == "0") ? 0 : 1;
  }();
  return v == 1;
}
bool mnist_f7_wino() {
  static const int v = [] {
    const char* e = std::getenv("MXDDP_MNIST_F7");
    return (e && std::string(e) == "direct") ? 0 : 1;
  }();
  return v == 1;
}
static int f6w_split();
static int f6w_cos();
bool mnist_wslab() {
  static const int v = [] {
    const char* e = std::getenv("MXDDP_WSLAB");
    return (e && std::string(e) == "0") ? 0 : 1;
  }();
  // the slab epilogue exists in the unsplit Winograd weight-gradient blocks (co-split or not)
  return v == 1 && mnist_f7_wino() && f6w_split() == 1;
}
static int f6w_split() {
  static const int v = [] {
    const char* e = std::getenv("MXDDP_F6W_SPLIT");
    const int s = e ? std::atoi(e) : 1;
    return (s == 2 || s == 3) ? s : 1;
  }();
  return v;
}
// weight-gradient blocks split over output channels (MXDDP_F6W_COS = 1 | 2)
static int f6w_cos() {
  static const int v = [] {
    const char* e = std::getenv("MXDDP_F6W_COS");
    return (e && std::atoi(e) == 2) ? 2 : 1;
  }();
  return v;
}

// F7W operand prefetch one k-step ahead (default; MXDDP_F7W_VQ=0 turns it off): 931k -> 939k
// img/s, 3 A/B pairs (profiles/r3_f5f2)
static bool f7w_vq() {
  static const int v = [] {
    const char* e = std::getenv("MXDDP_F7W_VQ");
    return (e && std::string(e) == "0") ? 0 : 1;
  }();
  return v == 1;
}

template <int kSplit>
static void launch_f67_wino(const MnistFused& f, const Scratch& sc, hipStream_t st) {
  constexpr size_t lds = kF6WLds > kF7WLds ? kF6WLds : kF7WLds;
  const int cos = kSplit == 1 && f.a1_pub ? f6w_cos() : 1;
  const dim3 grid(f.co_blocks + 2 * kSplit * cos * f.B + kF7WChunks * f.B);
  if (kSplit == 1 && f.a1_pub && cos == 2 && f7w_vq())
    MX_LAUNCH((f67_conv2_bwd_kernel<true, 1, true, 2, true>), grid, dim3(256), lds, st, f, sc);
  else if (kSplit == 1 && f.a1_pub && cos == 2)
    MX_LAUNCH((f67_conv2_bwd_kernel<true, 1, true, 2>), grid, dim3(256), lds, st, f, sc);
  else if (kSplit == 1 && f.a1_pub && f7w_vq())
    MX_LAUNCH((f67_conv2_bwd_kernel<true, 1, true, 1, true>), grid, dim3(256), lds, st, f, sc);
  else if (kSplit == 1 && f.a1_pub)
    MX_LAUNCH((f67_conv2_bwd_kernel<true, 1, true>), grid, dim3(256), lds, st, f, sc);
  else
    MX_LAUNCH((f67_conv2_bwd_kernel<true, kSplit>), grid, dim3(256), lds, st, f, sc);
}

void mnist_fused_conv_bwd(const MnistFused& f, hipStream_t st, bool finalize_in_sgd) {
  static bool attr = false;
  if (!attr) {
    for (const void* fn : {reinterpret_cast<const void*>(f67_conv2_bwd_kernel<true, 1>),
                           reinterpret_cast<const void*>(f67_conv2_bwd_kernel<true, 1, true>),
                           reinterpret_cast<const void*>(f67_conv2_bwd_kernel<true, 1, true, 1, true>),
                           reinterpret_cast<const void*>(f67_conv2_bwd_kernel<true, 1, true, 2>),
                           reinterpret_cast<const void*>(f67_conv2_bwd_kernel<true, 1, true, 2, true>),
                           reinterpret_cast<const void*>(f67_conv2_bwd_kernel<true, 2>),
                           reinterpret_cast<const void*>(f67_conv2_bwd_kernel<true, 3>),
                           reinterpret_cast<const void*>(f67_conv2_bwd_kernel<false>)})
      MX_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  const Scratch sc = carve(f.scratch);
  if (mnist_f7_wino()) {
    switch (f6w_split()) {
      case 2: launch_f67_wino<2>(f, sc, st); break;
      case 3: launch_f67_wino<3>(f, sc, st); break;
      default: launch_f67_wino<1>(f, sc, st); break;
    }
  } else {
    constexpr size_t lds = kF6Lds > kF7Lds ? kF6Lds : kF7Lds;
    MX_LAUNCH(f67_conv2_bwd_kernel<false>, dim3(f.co_blocks + 9 * f.B + 11 * f.B), dim3(256), lds, st, f, sc);
  }
  if (!finalize_in_sgd)
    MX_LAUNCH(f8_finalize_kernel, dim3((f.wslab ? kWslabGroups : kF8Wacc) + kF8G1 + 8), dim3(256), 0, st, f, sc);
  MX_HIP_CHECK(hipGetLastError());
}

}  // namespace mx
