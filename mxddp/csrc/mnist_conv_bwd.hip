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
      atomicAdd(sc.wacc + (r * 64 + co) * 32 + ci, acc[c][j]);
    }
  MX_TRACE_B(f, 3, 3, braw);
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
  // per-image partial slab (11 chunk blocks per address instead of all 704 blocks hammering
  // the same 320 words: same-address float atomics serialise at the memory side)
  float* g1 = sc.g1 + b * 320;
  for (int i = tid; i < 320; i += 256) {
    const float v = red[i] + red[320 + i] + red[640 + i] + red[960 + i];
    const int ci = i / 10, k = i - ci * 10;
    if (k < 9) atomicAdd(g1 + ci * 9 + k, v);  // conv1.weight grad [32][9]
    else atomicAdd(g1 + 288 + ci, v);          // conv1.bias grad [32]
  }
  MX_TRACE_B(f, 4, 3, braw);
}

// ------------------------------------------------------------------------------------------
// F6 + F7 in ONE launch: blocks [0, 9B) run the weight gradient, the rest the data gradient.
// The two are independent; sharing a grid lets the dispatcher backfill CUs as blocks retire
// (576 + 704 blocks over 256 CUs at 3 per CU), so one kernel's prologue/epilogue latency and
// the 2-vs-3-blocks-per-CU imbalance of each kernel alone are covered by the other's MFMA work.
// 9B is a multiple of 8, so the F7 part keeps its XCD-aware block mapping.
__global__ __launch_bounds__(256) void f67_conv2_bwd_kernel(MnistFused f, Scratch sc) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int n6 = 9 * f.B;
  if ((int)blockIdx.x < n6)
    f6_body(f, sc, sm, blockIdx.x, n6);
  else
    f7_body(f, sc, sm, blockIdx.x - n6, 11 * f.B);
}

// ------------------------------------------------------------------------------------------
// F8: finalize bucket 1: conv2.weight grad = transpose of the [r][co][ci] accumulator into
// the canonical [co][ci][ky][kx] layout; conv1 weight/bias grads = sum over the per-image
// partial slabs.  Every accumulator it consumes (wacc, g1) and the fc1 split-K accumulator h
// are reset here for the next step, so the step needs no memset launches.
// Blocks 0..71: wacc transpose (256 outputs each).  Blocks 72..81: the slab sum, 32 outputs per
// block, 8 threads per output each summing B/8 images (strided so a wave's loads coalesce),
// combined with shuffles.  Blocks 82..: zero h.
constexpr int kF8Wacc = kPack / 256, kF8G1 = 10;
__global__ __launch_bounds__(256) void f8_finalize_kernel(MnistFused f, Scratch sc) {
  const int blk = blockIdx.x, tid = threadIdx.x;
  if (blk < kF8Wacc) {
    const int i = blk * 256 + tid;
    const int co = i / 288, rem = i - co * 288, ci = rem / 9, rr = rem - ci * 9;
    float* a = sc.wacc + (rr * 64 + co) * 32 + ci;
    f.g[L::w2 + i] = *a;
    *a = 0.f;
  } else if (blk < kF8Wacc + kF8G1) {
    const int j = (blk - kF8Wacc) * 32 + (tid & 31), part = tid >> 5;  // 8 parts
    float s = 0.f;
    for (int b = part; b < f.B; b += 8) {
      float* p = sc.g1 + b * 320 + j;
      s += *p;
      *p = 0.f;
    }
    s += __shfl_xor(s, 32, 64);  // parts (2k, 2k+1) share a wave: lanes j and j+32
    __shared__ float red[4][32];
    if ((tid & 63) < 32) red[tid >> 6][tid & 31] = s;
    __syncthreads();
    if (tid < 32) f.g[L::w1 + j] = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
  } else {
    for (int i = (blk - kF8Wacc - kF8G1) * 256 + tid; i < f.B * 128; i += 8 * 256) f.h[i] = 0.f;
  }
}

}  // namespace
}  // namespace mnist

using namespace mnist;

void mnist_fused_conv_bwd(const MnistFused& f, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    MX_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(f67_conv2_bwd_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  const Scratch sc = carve(f.scratch);
  constexpr size_t lds = kF6Lds > kF7Lds ? kF6Lds : kF7Lds;
  MX_LAUNCH(f67_conv2_bwd_kernel, dim3(9 * f.B + 11 * f.B), dim3(256), lds, st, f, sc);
  MX_LAUNCH(f8_finalize_kernel, dim3(kF8Wacc + kF8G1 + 8), dim3(256), 0, st, f, sc);
  MX_HIP_CHECK(hipGetLastError());
}

}  // namespace mx
