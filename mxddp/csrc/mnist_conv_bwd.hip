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
#include "mnist_common.h"
#include "peer_device.h"

namespace mx {
namespace mnist {
namespace {

// ------------------------------------------------------------------------------------------
// F6W: conv2 weight gradient as Winograd F(2x2,3x3): 2.25x fewer MFMAs than direct.  The 2x2 output
// tiles of conv2 are exactly the pool windows, so dY2 of tile t has ONE nonzero (value dp, argmax
// code q) and its Winograd transform A dY A^T = dp * a(qy) a(qx)^T (a(0) = (1,1,1,0),
// a(1) = (0,1,-1,-1)) is built in registers.  16 GEMMs (one per Winograd point xi) over
// K = 144 tiles: dU[xi][co][ci] = sum_t W[xi][co][t] V[xi][t][ci], V = B^T a1_t B; then
// dw = G^T dU G lane-locally (all 16 xi of a (co, ci) sit in one lane), written as this image's
// slab of the weight gradient with plain stores (the finalize sums the B slabs in a fixed order).
// Block = (image, ci half): all 144 tiles.  Wave w = co 16w..16w+15.  6 chunks of 2 tile rows:
// (A) the chunk's 6 a1 rows that F2 published -> LDS (one chunk ahead, 3 float4 per thread in
// registers; recomputing conv1 here was 5.4 of 25 us), (B) V of 24 tiles x 16 ci -> LDS
// ([t][ci][20]: conflict-free ds_read_b128 of the 16 xi), (C) 6 k-steps of 16 MFMAs; K inside a
// chunk is ordered t = 6g + s (lane group g) so a lane's dp / q operands are 6 contiguous windows
// (float2 / u16 loads, prefetched one chunk ahead).  The a1 tile pitch 164: 16-byte rows for the
// float4 stores, 36 ci mod 64 banks keeps phase B's reads conflict-free.
// (Measured and removed, profiles/r3_cos2 and r2: 2-3 blocks per (image, ci half): 725k / 695k vs
// 748k img/s; blocks split over co halves: 917k vs 951k; round 5, profiles/r5_f6split: blocks split
// over the Winograd rows (2 x 8 of the 16 GEMMs, partial slabs): F6W 24 -> 18 us but F7W 19 -> 23 us
// beside the extra blocks, 903k vs 929k.)
constexpr int kF6WA1P = 164, kF6WVP = 20, kF6WV = 24 * 16 * kF6WVP;
// f6w_body: two V buffers (75 KB, two blocks per CU -- the grid without exchange blocks is exactly
// two per CU); f6w_body_serial: one (45 KB, three per CU)
constexpr size_t kF6WLdsPipe = sizeof(float) * (784 + 160 + 16 * kF6WA1P + 2 * kF6WV);
constexpr size_t kF6WLdsSerial = sizeof(float) * (784 + 160 + 16 * kF6WA1P + kF6WV);
// F6W epilogue (both variants): dw = G^T dU G of the block's accumulators -> the image's slab.
__device__ __forceinline__ void f6w_epilogue(const MnistFused& f, const Scratch& sc, float* sm, const f32x4 (&acc)[16],
                                             int b, int h, int braw, bool trc, uint32_t tA, uint32_t tB, uint32_t tC) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, m = lane & 15;
  MX_TRACE_B(f, 3, 2, braw);
  // dw = G^T dU G, G^T = [1 .5 .5 0; 0 .5 -.5 0; 0 .5 .5 1]; acc[4i + j'][j] = dU[i][j'] of
  // (co = 16w + 4g + j, ci = 16h + m).  This block's [64 co][16 ci][9] result is staged in LDS
  // (over the idle operand tiles) and written to the image's slab in canonical [co][ci][ky][kx]
  // order with coalesced 16-byte stores -- no atomics (the atomic epilogue was ~3 us and delayed
  // the F7W blocks' own atomics behind it); the finalize sums the B slabs in a fixed order.
  float* st = sm;  // [64 co][16 ci][9]
  __syncthreads();  // every wave's phase-C reads of the operand tiles are done
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
      float* sp = st + (cj * 16 + m) * 9 + 3 * ky;
      sp[0] = t[ky][0] + 0.5f * (t[ky][1] + t[ky][2]);
      sp[1] = 0.5f * (t[ky][1] - t[ky][2]);
      sp[2] = 0.5f * (t[ky][1] + t[ky][2]) + t[ky][3];
    }
  }
  __syncthreads();
  {
    // per co: 16 ci x 9 taps = 144 contiguous floats (36 float4) at (co * 32 + 16 h) * 9
    const float4* s4 = reinterpret_cast<const float4*>(st);
    float4* d4 = reinterpret_cast<float4*>(sc.wslab + (size_t)b * kPack + 144 * h);
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int i = tid + 256 * k, cq = i / 36, q = i - 36 * cq;
      st4(d4 + cq * 72 + q, s4[i], f.wt & 4);
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

// F6W with ONE V buffer and (B) as its own phase per chunk (45 KB, three blocks per CU): the
// variant for launches that also hold co-scheduled exchange blocks, which need CU slots beside
// the 512 conv blocks.
__device__ __forceinline__ void f6w_body_serial(const MnistFused& f, const Scratch& sc, float* sm, int braw, int nblk) {
  MX_TRACE_B(f, 3, 0, braw);
  constexpr int kA1P = kF6WA1P;
  float* a1s = sm + 784 + 160;  // [16 ci][kA1P]: 6 a1 rows x 26
  float* vs = a1s + 16 * kA1P;  // [24 t][16 ci][20]
  const int bid = xcd_remap(braw, nblk);
  const int b = bid / 2, h = bid & 1;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, m = lane & 15;
  // a1 rows 4c .. 4c+5 of the block's 16 ci = 16 x 39 float4 (624 of the 768 slots)
  // (three named registers, not an array: an array here was placed in scratch memory)
  const float* a1b = f.a1 + ((size_t)b * 32 + 16 * h) * 676;
  int a1src[3], a1dst[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int i = min(tid + 256 * k, 623), ci = i / 39, f4 = i - 39 * ci;
    a1src[k] = ci * 676 + 4 * f4;
    a1dst[k] = tid + 256 * k < 624 ? ci * kA1P + 4 * f4 : -1;
  }
  float4 pa0 = *reinterpret_cast<const float4*>(a1b + a1src[0]);
  float4 pa1 = *reinterpret_cast<const float4*>(a1b + a1src[1]);
  float4 pa2 = *reinterpret_cast<const float4*>(a1b + a1src[2]);
  const int co = 16 * w + m;  // A row of this lane
  const float* dpl = f.dp + (size_t)b * 9216 + co * 144 + 6 * g;
  const uint16_t* qpl = reinterpret_cast<const uint16_t*>(reinterpret_cast<const uint8_t*>(f.idx) + (size_t)b * 9216 + co * 144 + 6 * g);
  float2 dn[3];
  uint16_t qn[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    dn[k] = *reinterpret_cast<const float2*>(dpl + 2 * k);
    qn[k] = qpl[k];
  }
  f32x4 acc[16];
#pragma unroll
  for (int x = 0; x < 16; ++x) acc[x] = f32x4{0.f, 0.f, 0.f, 0.f};
  MX_TRACE_B(f, 3, 1, braw);
  uint32_t tA = 0, tB = 0, tC = 0, tq = 0;  // phase-time sums (trace only)
  const bool trc = f.trace && threadIdx.x == 0 && braw < 1024;
#pragma unroll 1
  for (int c = 0; c < 6; ++c) {
    if (trc) tq = (uint32_t)__builtin_amdgcn_s_memrealtime();
    // (A) published a1 rows -> LDS (the previous chunk's phase-B reads of a1s finished before the
    // barrier ahead of its phase C); next chunk's rows in flight
    *reinterpret_cast<float4*>(a1s + a1dst[0]) = pa0;
    *reinterpret_cast<float4*>(a1s + a1dst[1]) = pa1;
    if (a1dst[2] >= 0) *reinterpret_cast<float4*>(a1s + a1dst[2]) = pa2;
    if (c + 1 < 6) {
      const float* nb = a1b + 104 * (c + 1);
      pa0 = *reinterpret_cast<const float4*>(nb + a1src[0]);
      pa1 = *reinterpret_cast<const float4*>(nb + a1src[1]);
      pa2 = *reinterpret_cast<const float4*>(nb + a1src[2]);
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
    if (c + 1 < 6) {
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
    // (C) k-step s: tile t = 6g + s of the chunk.  The next k-step's B fragments are read from LDS
    // before this step's MFMAs (kept there by the scheduling barrier): loaded at their use, each
    // group of 8 MFMAs waited for an LDS round trip (lgkmcnt(0) in the ISA, ~30 % of phase C)
    const float4* vp0 = reinterpret_cast<const float4*>(vs + ((6 * g) * 16 + m) * kF6WVP);
    float4 bb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) bb[i] = vp0[i];
#pragma unroll
    for (int s = 0; s < 6; ++s) {
      float4 bn[4];
      if (s + 1 < 6) {
        const float4* vp = reinterpret_cast<const float4*>(vs + ((6 * g + s + 1) * 16 + m) * kF6WVP);
#pragma unroll
        for (int i = 0; i < 4; ++i) bn[i] = vp[i];
      }
      __builtin_amdgcn_sched_barrier(0);
      const float v = dv[s];
      const bool qy = (qv[s] >> 1) & 1, qx = qv[s] & 1;
      const float vy[4] = {qy ? 0.f : v, v, qy ? -v : v, qy ? -v : 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float w0 = qx ? 0.f : vy[i], w2 = qx ? -vy[i] : vy[i], w3 = qx ? -vy[i] : 0.f;
        acc[4 * i + 0] = mfma4(w0, bb[i].x, acc[4 * i + 0]);
        acc[4 * i + 1] = mfma4(vy[i], bb[i].y, acc[4 * i + 1]);
        acc[4 * i + 2] = mfma4(w2, bb[i].z, acc[4 * i + 2]);
        acc[4 * i + 3] = mfma4(w3, bb[i].w, acc[4 * i + 3]);
      }
      if (s + 1 < 6) {
#pragma unroll
        for (int i = 0; i < 4; ++i) bb[i] = bn[i];
      }
    }
    if (trc) tC += (uint32_t)__builtin_amdgcn_s_memrealtime() - tq;  // issue time of (C)
  }
  f6w_epilogue(f, sc, sm, acc, b, h, braw, trc, tA, tB, tC);
}

__device__ __forceinline__ void f6w_body(const MnistFused& f, const Scratch& sc, float* sm, int braw, int nblk) {
  MX_TRACE_B(f, 3, 0, braw);
  constexpr int kA1P = kF6WA1P;
  float* a1s = sm + 784 + 160;  // [16 ci][kA1P]: 6 a1 rows x 26
  float* vs = a1s + 16 * kA1P;  // 2 x [24 t][16 ci][20]: chunk c's V in buffer c & 1
  const int bid = xcd_remap(braw, nblk);
  const int b = bid / 2, h = bid & 1;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, m = lane & 15;
  // a1 rows 4c .. 4c+5 of the block's 16 ci = 16 x 39 float4 (624 of the 768 slots)
  // (three named registers, not an array: an array here was placed in scratch memory)
  const float* a1b = f.a1 + ((size_t)b * 32 + 16 * h) * 676;
  int a1src[3], a1dst[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int i = min(tid + 256 * k, 623), ci = i / 39, f4 = i - 39 * ci;
    a1src[k] = ci * 676 + 4 * f4;
    a1dst[k] = tid + 256 * k < 624 ? ci * kA1P + 4 * f4 : -1;
  }
  float4 pa0 = *reinterpret_cast<const float4*>(a1b + a1src[0]);
  float4 pa1 = *reinterpret_cast<const float4*>(a1b + a1src[1]);
  float4 pa2 = *reinterpret_cast<const float4*>(a1b + a1src[2]);
  const int co = 16 * w + m;  // A row of this lane
  const float* dpl = f.dp + (size_t)b * 9216 + co * 144 + 6 * g;
  const uint16_t* qpl = reinterpret_cast<const uint16_t*>(reinterpret_cast<const uint8_t*>(f.idx) + (size_t)b * 9216 + co * 144 + 6 * g);
  float2 dn[3];
  uint16_t qn[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    dn[k] = *reinterpret_cast<const float2*>(dpl + 2 * k);
    qn[k] = qpl[k];
  }
  f32x4 acc[16];
#pragma unroll
  for (int x = 0; x < 16; ++x) acc[x] = f32x4{0.f, 0.f, 0.f, 0.f};
  // (B) item i (< 384) of a chunk: V = B^T d B of tile tl = i / 16, channel ci = i % 16 (a1 rows
  // 2(tl/12).., cols 2(tl%12)..) -- its 16 LDS reads, then the transform into V buffer vb
  auto b_load = [&](int i, float (&d)[16]) {
    const int ci = i & 15, tl = i >> 4, tyl = tl / 12, tx = tl - 12 * tyl;
    const float* ap = a1s + ci * kA1P + 2 * tyl * 26 + 2 * tx;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) d[4 * r + cc] = ap[r * 26 + cc];
  };
  auto b_store = [&](int i, const float (&d)[16], float* vb) {
    float e[4][4];
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) {
      e[0][cc] = d[cc] - d[8 + cc];
      e[1][cc] = d[4 + cc] + d[8 + cc];
      e[2][cc] = d[8 + cc] - d[4 + cc];
      e[3][cc] = d[4 + cc] - d[12 + cc];
    }
    float4* vp = reinterpret_cast<float4*>(vb + ((i >> 4) * 16 + (i & 15)) * kF6WVP);
#pragma unroll
    for (int r = 0; r < 4; ++r)
      vp[r] = make_float4(e[r][0] - e[r][2], e[r][1] + e[r][2], e[r][2] - e[r][1], e[r][1] - e[r][3]);
  };
  MX_TRACE_B(f, 3, 1, braw);
  uint32_t tA = 0, tB = 0, tC = 0, tq = 0;  // phase-time sums (trace only)
  const bool trc = f.trace && threadIdx.x == 0 && braw < 1024;
  if (trc) tq = (uint32_t)__builtin_amdgcn_s_memrealtime();
  // prologue: chunk 0's a1 rows -> LDS, its V (the only (B) not hidden under MFMAs)
  *reinterpret_cast<float4*>(a1s + a1dst[0]) = pa0;
  *reinterpret_cast<float4*>(a1s + a1dst[1]) = pa1;
  if (a1dst[2] >= 0) *reinterpret_cast<float4*>(a1s + a1dst[2]) = pa2;
  {
    const float* nb = a1b + 104;
    pa0 = *reinterpret_cast<const float4*>(nb + a1src[0]);
    pa1 = *reinterpret_cast<const float4*>(nb + a1src[1]);
    pa2 = *reinterpret_cast<const float4*>(nb + a1src[2]);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = tid + 256 * k;
    if (i < 384) {
      float d[16];
      b_load(i, d);
      b_store(i, d, vs);
    }
  }
  __syncthreads();
  if (trc) {
    const uint32_t t = (uint32_t)__builtin_amdgcn_s_memrealtime();
    tB += t - tq;
  }
  // Chunk c: (A) chunk c + 1's a1 rows -> LDS (chunk c's were consumed by its (B) before the
  // barrier closing the previous chunk), then (C) -- chunk c's 36 k-steps of MFMAs on V buffer
  // c & 1 -- with chunk c + 1's (B) into the other buffer interleaved between the k-steps: the
  // transform's LDS reads, VALU and LDS writes issue while the MFMAs run (as two separate phases
  // with a barrier between them, the block's MFMAs idled through 3.7 us of (B), r5_f6pf).
#pragma unroll 1
  for (int c = 0; c < 6; ++c) {
    if (trc) tq = (uint32_t)__builtin_amdgcn_s_memrealtime();
    const bool nxt = c + 1 < 6;
    float* vcur = vs + (c & 1) * kF6WV;
    float* vnext = vs + ((c + 1) & 1) * kF6WV;
    if (nxt) {
      *reinterpret_cast<float4*>(a1s + a1dst[0]) = pa0;
      *reinterpret_cast<float4*>(a1s + a1dst[1]) = pa1;
      if (a1dst[2] >= 0) *reinterpret_cast<float4*>(a1s + a1dst[2]) = pa2;
      if (c + 2 < 6) {
        const float* nb = a1b + 104 * (c + 2);
        pa0 = *reinterpret_cast<const float4*>(nb + a1src[0]);
        pa1 = *reinterpret_cast<const float4*>(nb + a1src[1]);
        pa2 = *reinterpret_cast<const float4*>(nb + a1src[2]);
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
    if (nxt) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        dn[k] = *reinterpret_cast<const float2*>(dpl + 24 * (c + 1) + 2 * k);
        qn[k] = qpl[12 * (c + 1) + k];
      }
    }
    __syncthreads();  // chunk c + 1's a1 rows are in LDS
    if (trc) {
      const uint32_t t = (uint32_t)__builtin_amdgcn_s_memrealtime();
      tA += t - tq;
      tq = t;
    }
    // (C) k-step s: tile t = 6g + s of the chunk.  The next k-step's B fragments are read from LDS
    // before this step's MFMAs (kept there by the scheduling barrier): loaded at their use, each
    // group of 8 MFMAs waited for an LDS round trip (lgkmcnt(0) in the ISA, ~30 % of phase C).
    // Chunk c + 1's (B) items: item 0 read at k-step 0 and transformed + stored at k-step 1, item 1
    // (threads < 128) at k-steps 2 and 3.
    const float4* vp0 = reinterpret_cast<const float4*>(vcur + ((6 * g) * 16 + m) * kF6WVP);
    float4 bb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) bb[i] = vp0[i];
    float db[16];
#pragma unroll
    for (int s = 0; s < 6; ++s) {
      float4 bn[4];
      if (s + 1 < 6) {
        const float4* vp = reinterpret_cast<const float4*>(vcur + ((6 * g + s + 1) * 16 + m) * kF6WVP);
#pragma unroll
        for (int i = 0; i < 4; ++i) bn[i] = vp[i];
      }
      if (nxt && s == 0) b_load(tid, db);
      if (nxt && s == 2 && tid < 128) b_load(tid + 256, db);
      __builtin_amdgcn_sched_barrier(0);
      const float v = dv[s];
      const bool qy = (qv[s] >> 1) & 1, qx = qv[s] & 1;
      const float vy[4] = {qy ? 0.f : v, v, qy ? -v : v, qy ? -v : 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float w0 = qx ? 0.f : vy[i], w2 = qx ? -vy[i] : vy[i], w3 = qx ? -vy[i] : 0.f;
        acc[4 * i + 0] = mfma4(w0, bb[i].x, acc[4 * i + 0]);
        acc[4 * i + 1] = mfma4(vy[i], bb[i].y, acc[4 * i + 1]);
        acc[4 * i + 2] = mfma4(w2, bb[i].z, acc[4 * i + 2]);
        acc[4 * i + 3] = mfma4(w3, bb[i].w, acc[4 * i + 3]);
      }
      if (nxt && s == 1) b_store(tid, db, vnext);
      if (nxt && s == 3 && tid < 128) b_store(tid + 256, db, vnext);
      if (s + 1 < 6) {
#pragma unroll
        for (int i = 0; i < 4; ++i) bb[i] = bn[i];
      }
    }
    __syncthreads();  // chunk c + 1's V complete; every read of chunk c's V done
    if (trc) tC += (uint32_t)__builtin_amdgcn_s_memrealtime() - tq;  // (C) with the next (B)
  }
  f6w_epilogue(f, sc, sm, acc, b, h, braw, trc, tA, tB, tC);
}

// ------------------------------------------------------------------------------------------
// F7W: conv2 data gradient + conv1 ReLU mask + conv1 weight/bias grads, as Winograd F(2x2,3x3) on fp32 MFMA:
// 2.25x fewer MFMAs.  dA1 (26x26) = full correlation of dY2 with the flipped filter, in 13x13
// output tiles of 2x2.  Tile (ty, tx) reads the 4x4 patch of zero-padded dY2 at rows 2ty-2..2ty+1,
// cols 2tx-2..2tx+1 = exactly the 2x2 pool windows (ty-1..ty, tx-1..tx), each holding ONE nonzero
// (its argmax), so the input transform V = B^T d B is built from 4 (value, code) pairs straight
// out of the compact LDS tiles.  16 GEMMs (one per Winograd point xi, K = 64 co) share one MFMA
// fragment layout, so the output transform A^T M A of a (tile, ci) is lane-local.
// Block = (image, chunk of 32 tiles); wave w = (M-group w&1: 16 tiles, ci half w>>1: 16 ci);
// 16 k-steps of 4 co x 16 xi MFMAs.  B fragments (G w' G^T, written by F2) stream from L2 one
// k-step ahead, and the (value, code) LDS operands of k-step s + 1 are loaded during k-step s
// (the step's scheduling barrier otherwise keeps every step waiting for its own LDS reads).
// Epilogue: conv1 recomputed for the ReLU mask (a1 is never re-read), conv1 weight/bias grads
// reduced in registers -> lanes -> LDS (fixed order) -> int64 fixed-point atomics into slab
// image & 15 (order-independent sums).
constexpr int kF7WChunks = 6, kF7WRows = 5, kF7WCols = 14, kF7WCoP = 80;
constexpr size_t kF7WLds = sizeof(float) * (64 * kF7WCoP + 784 + 320 + 640) + 64 * kF7WCoP;
template <int kF7WPf>
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
    // fully unrolled; B fragments prefetched kF7WPf k-steps ahead (indices fold to registers;
    // 3 ahead measured equal to 2, profiles/r5_tune: 930 / 933k vs 932 / 928k img/s)
    float4 bq[16][4];
#pragma unroll
    for (int s = 0; s < kF7WPf; ++s)
#pragma unroll
      for (int k = 0; k < 4; ++k) bq[s][k] = wu[s * 512 + k];
    float vn[4];
    uint32_t qn[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int o = (k >> 1) * kF7WCols + (k & 1);
      vn[k] = dpp[o];
      qn[k] = qp[o];
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s + kF7WPf < 16) {
#pragma unroll
        for (int k = 0; k < 4; ++k) bq[s + kF7WPf][k] = wu[(s + kF7WPf) * 512 + k];
      }
      float v[4];
      uint32_t q[4];
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
      // keep the prefetch at the top of the step: left alone the scheduler sinks these loads
      // next to their use and every k-step then waits for L2 (vmcnt(0)) before its MFMAs
      __builtin_amdgcn_sched_barrier(0);
      const float4* bc = bq[s];
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
  long long* g1 = sc.g1 + (b & (kG1Slabs - 1)) * 320;
  for (int i = tid; i < 320; i += 256) {
    const float v = red[i] + red[320 + i];
    const int c = i / 10, k = i - c * 10;
    fix_add(g1 + (k < 9 ? c * 9 + k : 288 + c), v, kGScale, sc.bad);  // conv1.weight [32][9], conv1.bias [32]
  }
  MX_TRACE_B(f, 4, 3, braw);
}

// ------------------------------------------------------------------------------------------
// Deferred fc1 weight gradient + SGD update (MnistFused::fc1_defer, world size 1): F5 publishes
// dh and skips this work; these blocks come after F7W's in the conv-backward grid, so they take
// the CU slots the data-gradient blocks free first and run beside F6W's tail instead of on F5's
// critical path.  Block = one 48-column slice of fc1 (F5's slices), wave w = weight rows
// 32w .. 32w + 31: the same operand values, MFMA order and update as F5's folded path, so the
// trained weights are bitwise identical.  LDS: dh [B][132] + the pool slice [B][52] (B <= 96).
constexpr int kFc1DhP = 132, kFc1P = 52;
__device__ __forceinline__ void fc1_update_body(const MnistFused& f, float* sm, int slice) {
  const int B = f.B, c0 = slice * kFc1Cols;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, m = lane & 15;
  float* dhs = sm;                // [B][132]
  float* ps = dhs + B * kFc1DhP;  // [B][52]
  // this lane's 24 weights and momenta (requested first: their latency overlaps the staging)
  float mb[2][3][4], pw[2][3][4];
  if (f.fc1_sgd) {  // uniform: world size 1 updates here, otherwise only the gradient is stored
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const size_t e = L::fw1 + (size_t)(32 * w + 16 * a + 4 * g + j) * 9216 + c0 + 16 * c + m;
          mb[a][c][j] = f.mom[e];
          pw[a][c][j] = f.p[e];
        }
  }
  // dh [B][128] and the pool slice [B][48]: 8 + 3 float4 per thread at batch 64 (mode 2 takes
  // B <= 64), every load issued before the first LDS store -- a `load; store` loop pays one memory
  // round trip per float4.  Indices are clamped, not predicated (a predicated store lets the
  // compiler sink its load into the branch); past the end a thread rewrites the last element.
  constexpr int kDU = 8, kPU = 3;
  const int nd = B * 32, np = B * 12;
  float4 dv[kDU], pv4[kPU];
#pragma unroll
  for (int u = 0; u < kDU; ++u) {
    const int i = min(tid + 256 * u, nd - 1);
    dv[u] = *reinterpret_cast<const float4*>(f.dh + (i >> 5) * 128 + (i & 31) * 4);
  }
#pragma unroll
  for (int u = 0; u < kPU; ++u) {
    const int i = min(tid + 256 * u, np - 1), r = i / 12;
    pv4[u] = *reinterpret_cast<const float4*>(f.pool + (size_t)r * 9216 + c0 + (i - r * 12) * 4);
  }
#pragma unroll
  for (int u = 0; u < kDU; ++u) {
    const int i = min(tid + 256 * u, nd - 1);
    *reinterpret_cast<float4*>(dhs + (i >> 5) * kFc1DhP + (i & 31) * 4) = dv[u];
  }
#pragma unroll
  for (int u = 0; u < kPU; ++u) {
    const int i = min(tid + 256 * u, np - 1), r = i / 12;
    *reinterpret_cast<float4*>(ps + r * kFc1P + (i - r * 12) * 4) = pv4[u];
  }
  for (int i = tid + 256 * kDU; i < nd; i += 256) {  // B > 64 (mode 1): the rest
    const int r = i >> 5, c4 = (i & 31) * 4;
    *reinterpret_cast<float4*>(dhs + r * kFc1DhP + c4) = *reinterpret_cast<const float4*>(f.dh + r * 128 + c4);
  }
  for (int i = tid + 256 * kPU; i < np; i += 256) {
    const int r = i / 12, c4 = (i - r * 12) * 4;
    *reinterpret_cast<float4*>(ps + r * kFc1P + c4) = *reinterpret_cast<const float4*>(f.pool + (size_t)r * 9216 + c0 + c4);
  }
  __syncthreads();
  f32x4 acc[2][3];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 3; ++c) acc[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < B / 16; ++s) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int b = 16 * s + 4 * g + j;
      const float a0 = dhs[b * kFc1DhP + 32 * w + m], a1v = dhs[b * kFc1DhP + 32 * w + 16 + m];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float bv = ps[b * kFc1P + 16 * c + m];
        acc[0][c] = mfma4(a0, bv, acc[0][c]);
        acc[1][c] = mfma4(a1v, bv, acc[1][c]);
      }
    }
  }
  const bool wt = f.wt & 1;
  if (!f.fc1_sgd) {  // gradient collectives: the gradient goes to g (merged all-reduce, then SGD)
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          st1(f.g + L::fw1 + (size_t)(32 * w + 16 * a + 4 * g + j) * 9216 + c0 + 16 * c + m, acc[a][c][j], wt);
    return;
  }
  const float lr = *f.lr;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const size_t e = L::fw1 + (size_t)(32 * w + 16 * a + 4 * g + j) * 9216 + c0 + 16 * c + m;
        float pv = pw[a][c][j], bv = mb[a][c][j];
        sgd_upd(pv, bv, acc[a][c][j], 1.f, f.sgd_mom, f.sgd_wd, lr);
        st1(f.mom + e, bv, wt);
        st1(f.p + e, pv, wt);
      }
}

// ------------------------------------------------------------------------------------------
// XCD-aware block placement of the batch-64 F67 grid (704 blocks: 128 F6W, 384 F7W, 192 fc1 at
// three per CU).  Workgroup b goes to XCD b % 8, and an XCD hands its j-th workgroup (j = b / 8)
// to CU j % 32 of slot j / 32 while the slots fill in order, so the plain [F6W | F7W | fc1] order
// puts every F6W block (the longest MFMA chain, 2,304 16x16x4 MFMAs) on CUs 0-15 of its XCD
// beside an F7W block (~900) and an fc1 block (384).  Here the F6W blocks sit on CUs 16-31 beside
// fc1 blocks only, and CUs 0-15 run three F7W blocks: the heaviest CU drops from ~3,600 to
// ~3,100 MFMAs.  Every role keeps index % 8 == its XCD, so the bodies' xcd_remap still groups an
// image's blocks on one XCD.  (A placement assumption, not a guarantee: the order only moves
// work between CUs; any dispatch order computes the same result.)
struct F67Role {
  int kind, idx;  // kind 0 = F6W, 1 = F7W, 2 = fc1
};
__device__ __forceinline__ F67Role f67_role(int b) {
  const int x = b & 7, j = b >> 3;
  if (j < 16) return F67Role{1, j * 8 + x};                // slot 0, CUs 0-15: F7W 0..15
  if (j < 32) return F67Role{0, (j - 16) * 8 + x};         // slot 0, CUs 16-31: F6W
  if (j < 48) return F67Role{1, (16 + j - 32) * 8 + x};    // slot 1, CUs 0-15: F7W 16..31
  if (j < 64) return F67Role{2, (j - 48) * 8 + x};         // slot 1, CUs 16-31: fc1 0..15
  if (j < 80) return F67Role{1, (32 + j - 64) * 8 + x};    // slot 2, CUs 0-15: F7W 32..47
  return F67Role{2, (16 + j - 80) * 8 + x};                // slot 2, CUs 16-23: fc1 16..23
}
static int g_f67_order = 1;

// ------------------------------------------------------------------------------------------
// F6W + F7W in ONE launch: blocks [0, 2B) run the weight gradient, the rest the data gradient.
// The two are independent; sharing a grid lets the dispatcher backfill CUs as blocks retire, so
// one kernel's prologue/epilogue latency and the blocks-per-CU imbalance of each kernel alone
// are covered by the other's MFMA work.  2B is a multiple of 8, so the F7W part keeps its
// XCD-aware block mapping.
//
// Co-scheduled gradient exchange (f.co_blocks > 0): the first co_blocks blocks run the two-shot
// peer all-reduce of the fc bucket (complete since F5) instead -- dispatched first, they wait on
// the peers' matching blocks while the remaining blocks do the conv backward, so the 4.7 MB
// exchange overlaps it inside ONE launch (no side stream, no cross-queue fence).  co_blocks is
// a multiple of 8, so the conv part keeps its XCD-aware block mapping.
template <bool kPipe>
__global__ __launch_bounds__(256, kPipe ? 2 : 3) void f67_conv2_bwd_kernel(MnistFused f, Scratch sc) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  if ((int)blockIdx.x < f.co_blocks) {
    MX_TRACE_B(f, 5, 0, (int)blockIdx.x);  // trace: exchange blocks vs conv blocks of this launch
    peer_two_shot_f32_block(f.co_args, f.co_part, blockIdx.x, reinterpret_cast<uint32_t*>(sm));
    MX_TRACE_B(f, 5, 1, (int)blockIdx.x);
    return;
  }
  const int bid = (int)blockIdx.x - f.co_blocks;
  const int n6 = 2 * f.B, n7 = kF7WChunks * f.B;
  if (f.f67_order) {  // batch 64, three blocks per CU, no exchange blocks (see f67_role)
    const F67Role r = f67_role(bid);
    if (r.kind == 0) f6w_body_serial(f, sc, sm, r.idx, n6);
    else if (r.kind == 1) f7w_body<2>(f, sc, sm, r.idx, n7);
    else fc1_update_body(f, sm, r.idx);
    return;
  }
  if (bid < n6)
    if constexpr (kPipe) f6w_body(f, sc, sm, bid, n6);
    else f6w_body_serial(f, sc, sm, bid, n6);
  else if (bid < n6 + n7)
    f7w_body<2>(f, sc, sm, bid - n6, n7);
  else  // deferred fc1 update (f.fc1_defer): the grid's last kFc1Slices blocks
    fc1_update_body(f, sm, bid - n6 - n7);
}

// ------------------------------------------------------------------------------------------
// F8 (gradient collectives in the step): finalize bucket 1 into g before its all-reduce --
// conv2.weight grad = the fixed-order sum of the per-image slabs (blocks 0 .. 511, 4 (co, ci)
// pairs each); conv1 weight/bias grads = the exact int64 sum of the slabs, conv2 bias grad =
// its accumulator, both converted and reset (blocks 512, 513); h zeroed for the next step's F3
// (the last 8 blocks).  No memset launches.
__global__ __launch_bounds__(256) void f8_finalize_kernel(MnistFused f, Scratch sc) {
  __shared__ float red[576 + 36];
  const int tid = threadIdx.x, blk = blockIdx.x;
  if (blk < kWslabGroups) {
    wslab_group_sum(f, sc, blk, red, red + 576);
    if (tid < 36) f.g[L::w2 + 36 * blk + tid] = red[576 + tid];
  } else if (blk < kWslabGroups + 2) {
    const int j = (blk - kWslabGroups) * 256 + tid;
    if (j < 320) {  // conv1 w [32][9], b [32]
      long long v[kG1Slabs];
#pragma unroll
      for (int k = 0; k < kG1Slabs; ++k) v[k] = sc.g1[k * 320 + j];
      long long s = 0;
#pragma unroll
      for (int k = 0; k < kG1Slabs; ++k) s += v[k];
#pragma unroll
      for (int k = 0; k < kG1Slabs; ++k) sc.g1[k * 320 + j] = 0;
      f.g[L::w1 + j] = from_fix_chk(s, kGInv, *sc.bad);
    } else if (j < 384) {  // conv2 bias
      f.g[L::b2 + j - 320] = from_fix_chk(sc.db2[j - 320], kGInv, *sc.bad);
      sc.db2[j - 320] = 0;
    }
  } else {
    longlong2* h2 = reinterpret_cast<longlong2*>(f.h);
    for (int i = (blk - kWslabGroups - 2) * 256 + tid; i < f.B * 64; i += 8 * 256) h2[i] = make_longlong2(0, 0);
  }
}

}  // namespace
}  // namespace mnist

using namespace mnist;

void mnist_set_f67_order(int on) { g_f67_order = on ? 1 : 0; }
int mnist_f67_order() { return g_f67_order; }

void mnist_fused_conv_bwd(const MnistFused& f, hipStream_t st, bool finalize_in_sgd) {
  static bool attr = false;
  if (!attr) {
    for (const void* fn : {reinterpret_cast<const void*>(f67_conv2_bwd_kernel<true>),
                           reinterpret_cast<const void*>(f67_conv2_bwd_kernel<false>)})
      MX_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  const Scratch sc = carve(f.scratch, f.B);
  const bool defer = f.fc1_defer != 0;
  MX_CHECK(!defer || (f.co_blocks == 0 && sizeof(float) * f.B * (kFc1DhP + kFc1P) <= kF6WLdsPipe),
           "deferred fc1 update: world size 1, batch <= 96");
  const dim3 grid(f.co_blocks + 2 * f.B + kF7WChunks * f.B + (defer ? kFc1Slices : 0));
  const size_t fc1_lds = sizeof(float) * f.B * (kFc1DhP + kFc1P);
  if (defer && f.fc1_defer == 2 && 3 * fc1_lds <= 160 * 1024) {
    // the single-V-buffer F6W at three blocks per CU: the fc1 blocks are resident from the start,
    // beside the conv blocks, instead of waiting for F7W's slots
    size_t lds = kF6WLdsSerial > kF7WLds ? kF6WLdsSerial : kF7WLds;
    if (fc1_lds > lds) lds = fc1_lds;
    MnistFused fk = f;
    // f67_role's table: 16 F6W, 48 F7W and 24 fc1 blocks per XCD
    fk.f67_order = g_f67_order && f.B == 64 && 2 * f.B == 128 && kF7WChunks * f.B == 384 && kFc1Slices == 192 ? 1 : 0;
    MX_LAUNCH(f67_conv2_bwd_kernel<false>, grid, dim3(256), lds, st, fk, sc);
  } else if (f.co_blocks == 0) {
    constexpr size_t lds = kF6WLdsPipe > kF7WLds ? kF6WLdsPipe : kF7WLds;
    MX_LAUNCH(f67_conv2_bwd_kernel<true>, grid, dim3(256), lds, st, f, sc);
  } else {  // the exchange blocks need CU slots beside the conv blocks: three per CU
    constexpr size_t lds = kF6WLdsSerial > kF7WLds ? kF6WLdsSerial : kF7WLds;
    MX_LAUNCH(f67_conv2_bwd_kernel<false>, grid, dim3(256), lds, st, f, sc);
  }
  if (!finalize_in_sgd) MX_LAUNCH(f8_finalize_kernel, dim3(kWslabGroups + 2 + 8), dim3(256), 0, st, f, sc);
  MX_HIP_CHECK(hipGetLastError());
}

}  // namespace mx
