// Fused Winograd F(2x2, 3x3) convolution on fp32 MFMA (v_mfma_f32_16x16x4_f32), gfx950.
//
// 3x3 / stride-1 / pad-1 convolutions (PyramidNet: 101 of its 103 convs) computed as 16
// independent GEMMs in the Winograd domain: M[xi][co][tile] = sum_ci U[xi][co][ci] V[xi][ci][tile]
// with U = G g G^T (filters, transformed once per call by wino_wtrans_k) and V = B^T d B (4x4
// input windows, transformed in registers inside the GEMM kernel).  The output transform
// Y = A^T M A needs all 16 xi of one (co, tile): every one of the 16 GEMMs uses the SAME MFMA
// fragment layout, so the 16 values of an output tile sit in the same lane and register slot of
// the 16 accumulators and the transform is lane-local (no LDS round trip, no second kernel).
// 2.25x fewer MFMA FLOPs than the direct convolution; all arithmetic is fp32 (the 1/2 factors
// of G are exact), the same algorithm family cuDNN / MIOpen select for fp32 3x3 convolutions.
//
// Forward / data gradient (wino_fwd_kernel): block = 32 output channels x 32 output tiles
// (2x2 pixels each), 4 waves in 2 x 2, each 16 channels x 16 tiles = 1 MFMA tile x 16 xi
// = 64 accumulator registers (3 blocks / 12 waves per CU).  Per chunk of 8 input channels: each
// thread transforms one 4x4 window (prefetched into registers during the previous chunk's
// MFMAs) into V in LDS, copies its part of the chunk's U slice (float4) into LDS, then 32 MFMAs
// per wave.  The data gradient is the same
// kernel on dy with the flipped / transposed filters (wino_wtrans_k, dgrad=1).  (Splitting the
// input channels across blocks with atomic accumulation is available but measured slower.)
//
// Weight gradient (wino_wgrad_kernel): F(3x3, 2x2): dW = A'^T [ sum_tiles (G' dy G'^T) o
// (B^T x B) ] A', 16 GEMMs reducing over output tiles.  Block = 32 co x 32 ci x a range of
// 8-tile chunks; the 3x3 result of each (co, ci) is formed lane-locally and written to a
// per-range partial plane, summed in a fixed order by a second kernel (deterministic).
//
// Replaces (reference): cuDNN conv fwd / bwd-data / bwd-filter for pytorch/model.py:28-32.
#include "common.h"
#include "wgrad_defer.h"
#include "ops.h"

#include <algorithm>
#include <cstdlib>

namespace mx {

namespace {

constexpr int kCC = 8;   // reduction rows per chunk (2 MFMA k-steps of 4)
constexpr int kP = 48;   // LDS pitch of 32-wide rows: the 4 lane groups of an MFMA operand read
                         // land on banks 0/48/32/16 (mod 64) -> conflict-free
constexpr size_t kLds = sizeof(float) * (2 * 16 * kCC * kP);  // 49,152 B -> 3 blocks/CU

// V = B^T d B, B^T = [[1,0,-1,0],[0,1,1,0],[0,-1,1,0],[0,1,0,-1]]  (d, v: row-major 4x4)
__device__ __forceinline__ void in_transform(const float* d, float* v) {
  float e[16];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    e[0 + j] = d[0 + j] - d[8 + j];
    e[4 + j] = d[4 + j] + d[8 + j];
    e[8 + j] = d[8 + j] - d[4 + j];
    e[12 + j] = d[4 + j] - d[12 + j];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[4 * i + 0] = e[4 * i + 0] - e[4 * i + 2];
    v[4 * i + 1] = e[4 * i + 1] + e[4 * i + 2];
    v[4 * i + 2] = e[4 * i + 2] - e[4 * i + 1];
    v[4 * i + 3] = e[4 * i + 1] - e[4 * i + 3];
  }
}

// U = G g G^T, G = [[1,0,0],[1/2,1/2,1/2],[1/2,-1/2,1/2],[0,0,1]]  (g: 3x3 row-major)
__device__ __forceinline__ void filter_transform(const float* g, float* u) {
  float t[12];  // 4x3
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    t[0 + j] = g[j];
    t[3 + j] = 0.5f * (g[j] + g[3 + j] + g[6 + j]);
    t[6 + j] = 0.5f * (g[j] - g[3 + j] + g[6 + j]);
    t[9 + j] = g[6 + j];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    u[4 * i + 0] = t[3 * i];
    u[4 * i + 1] = 0.5f * (t[3 * i] + t[3 * i + 1] + t[3 * i + 2]);
    u[4 * i + 2] = 0.5f * (t[3 * i] - t[3 * i + 1] + t[3 * i + 2]);
    u[4 * i + 3] = t[3 * i + 2];
  }
}

// W = G' y G'^T, G' = [[1,0],[1/2,1/2],[1/2,-1/2],[0,1]]  (y: 2x2 row-major) -- F(3x3, 2x2)
__device__ __forceinline__ void dy_transform(const float* y, float* w) {
  float t[8];  // 4x2
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    t[0 + j] = y[j];
    t[2 + j] = 0.5f * (y[j] + y[2 + j]);
    t[4 + j] = 0.5f * (y[j] - y[2 + j]);
    t[6 + j] = y[2 + j];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    w[4 * i + 0] = t[2 * i];
    w[4 * i + 1] = 0.5f * (t[2 * i] + t[2 * i + 1]);
    w[4 * i + 2] = 0.5f * (t[2 * i] - t[2 * i + 1]);
    w[4 * i + 3] = t[2 * i + 1];
  }
}

// ------------------------------------------------------------------------------------------
// Filter transform: U[xi][ci][co] (ci padded to Cip = 8k, co padded to Cop = 32k, zeros in the
// padding).  fwd: co = k, ci = c, g = w[k][c].  dgrad: co = c, ci = k, g = flip(w[k][c]).
__global__ void wino_wtrans_k(const float* __restrict__ w, float* __restrict__ U, int K, int C, int Cip,
                              int Cop, int dgrad) {
  const int total = Cip * Cop;
  const size_t plane = (size_t)Cip * Cop;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int ci = i / Cop, co = i - ci * Cop;
    const int k = dgrad ? ci : co, c = dgrad ? co : ci;
    float g[9], u[16];
    if (k < K && c < C) {
      const float* src = w + ((size_t)k * C + c) * 9;
#pragma unroll
      for (int t = 0; t < 9; ++t) g[t] = dgrad ? src[8 - t] : src[t];
    } else {
#pragma unroll
      for (int t = 0; t < 9; ++t) g[t] = 0.f;
    }
    filter_transform(g, u);
#pragma unroll
    for (int xi = 0; xi < 16; ++xi) U[xi * plane + i] = u[xi];
  }
}

// Both layouts in one launch (forward U and the data-gradient U of the backward pass): the
// forward call precomputes what the backward will need, saving one launch per conv per step.
__global__ void wino_wtrans2_k(const float* __restrict__ w, float* __restrict__ Uf, float* __restrict__ Ud, int K,
                               int C, int Cipf, int Copf, int Cipd, int Copd) {
  const int tf = Cipf * Copf, td = Cipd * Copd;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < tf + td; i += gridDim.x * 256) {
    const bool dg = i >= tf;
    const int j = dg ? i - tf : i, Cop = dg ? Copd : Copf;
    const size_t plane = dg ? (size_t)td : (size_t)tf;
    float* U = dg ? Ud : Uf;
    const int ci = j / Cop, co = j - ci * Cop;
    const int k = dg ? ci : co, c = dg ? co : ci;
    float g[9], u[16];
    if (k < K && c < C) {
      const float* src = w + ((size_t)k * C + c) * 9;
#pragma unroll
      for (int t = 0; t < 9; ++t) g[t] = dg ? src[8 - t] : src[t];
    } else {
#pragma unroll
      for (int t = 0; t < 9; ++t) g[t] = 0.f;
    }
    filter_transform(g, u);
#pragma unroll
    for (int xi = 0; xi < 16; ++xi) U[xi * plane + j] = u[xi];
  }
}

// Filter bank refresh: the forward / data-gradient Winograd filters of MANY convolutions in one
// launch (after the optimizer step), instead of one transform launch per conv per forward.  The
// job table travels by value in the kernel arguments (graph-capturable, no upload); block b
// belongs to the job with the largest blk0 <= b (uniform scalar scan).
struct WFJob {
  const float* w;
  float* Uf;  // [16][Cipf][Copf]
  float* Ud;  // [16][Cipd][Copd] or null
  int K, C, Cipf, Copf, Cipd, Copd, blk0;
};
constexpr int kWFMaxJobs = 64;
struct WFBatch {
  WFJob j[kWFMaxJobs];
  int n;
};
__global__ __launch_bounds__(256) void wino_wtrans_batch_k(WFBatch b) {
  int q = 0;
  while (q + 1 < b.n && b.j[q + 1].blk0 <= (int)blockIdx.x) ++q;
  const WFJob& J = b.j[q];
  const int tf = J.Cipf * J.Copf, td = J.Ud ? J.Cipd * J.Copd : 0;
  const int i = ((int)blockIdx.x - J.blk0) * 256 + (int)threadIdx.x;
  if (i >= tf + td) return;
  const bool dg = i >= tf;
  const int j = dg ? i - tf : i, Cop = dg ? J.Copd : J.Copf;
  const size_t plane = dg ? (size_t)td : (size_t)tf;
  float* U = dg ? J.Ud : J.Uf;
  const int ci = j / Cop, co = j - ci * Cop;
  const int k = dg ? ci : co, c = dg ? co : ci;
  float g[9], u[16];
  if (k < J.K && c < J.C) {
    const float* src = J.w + ((size_t)k * J.C + c) * 9;
#pragma unroll
    for (int t = 0; t < 9; ++t) g[t] = dg ? src[8 - t] : src[t];
  } else {
#pragma unroll
    for (int t = 0; t < 9; ++t) g[t] = 0.f;
  }
  filter_transform(g, u);
#pragma unroll
  for (int xi = 0; xi < 16; ++xi) U[xi * plane + j] = u[xi];
}

// One chunk (8 reduction rows) of the 16 Winograd-domain GEMMs: 32 MFMAs, each fed by one A and
// one B operand read from LDS.  The schedule is pinned to a software pipeline (8 operand reads
// ahead, then {1 MFMA, 2 reads}): left alone the scheduler hoists all 64 reads above the first
// MFMA, which costs 64 registers and pushes the kernel off 3 waves per SIMD (pinned in the
// forward kernel; the weight-gradient kernel fits without it and measured worse with it).
template <bool kPin>
__device__ __forceinline__ void mfma_chunk(const float* ap, const float* bp, f32x4* acc) {
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int xi = 0; xi < 16; ++xi) {
      const int ro = (xi * kCC + 4 * s) * kP;
      acc[xi] = __builtin_amdgcn_mfma_f32_16x16x4f32(ap[ro], bp[ro], acc[xi], 0, 0, 0);
    }
  if constexpr (kPin) {
  __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);  // DS read
#pragma unroll
  for (int i = 0; i < 30; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS read
  }
  __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
  }
}

// A folded BN's output as the convolution input (ops.bn_conv): relu?(x * sc + sh) per input
// channel -- the BN apply kernel's exact fmaf -- formed while the input is staged; elements
// outside the image stay zero (the padding of the BN output, not BN(0)).
__device__ __forceinline__ float in_affine(float v, float2 t, int relu) {
  const float y = fmaf(v, t.x, t.y);
  return relu ? fmaxf(y, 0.f) : y;
}
// The (scale, shift) of input channel c, loaded unconditionally (no fold: an identity pair): a
// load behind the `ss != null` branch would make the waitcnt pass drain the prefetched tiles at
// the branch's join, in every call of these kernels, folded or not.
__device__ float2 g_no_affine = {1.f, 0.f};
__device__ __forceinline__ float2 load_ss(const float2* ss, int c) {
  const float2* p = ss ? ss + c : &g_no_affine;
  return *p;
}

struct WinoArgs {
  const float* x;     // [N][Ci][W][W]
  const float* U;     // [16][Cip][Cop]
  const float* bias;  // [Co] or null
  const float* mask;  // [N][Co][W][W] or null
  float* y;           // [N][Co][W][W]
  int N, Ci, Co, Cip, Cop;
  int tblocks, ktiles, splits, chunks_per_split;
  int relu, accumulate;  // accumulate: 0 store, 1 y += result, 2 atomicAdd (split reduction)
  const float2* ss;      // [Ci] (scale, shift) of a folded BN on the input, or null
  int in_relu;           // the folded BN's fused ReLU
};

// 4x4 window of one (plane, tile).  Every load is issued (clamped to the plane's first element
// when outside the image) and the zeros are selected later, in zero_outside() at LDS-store time:
// selecting right after the loads would make the wave wait for them before the MFMAs they are
// meant to overlap.  Offsets are 32-bit byte offsets from the kernel-uniform tensor base
// (saddr + voffset loads) and are made opaque to the loop, so the compiler recomputes the 16
// window offsets per chunk instead of hoisting them into 16 long-lived registers.
template <int W>
__device__ __forceinline__ void load_window(const float* __restrict__ base, uint32_t plane, int off, unsigned m,
                                            float* d) {
  asm volatile("" : "+v"(off), "+v"(m));
  const char* b = reinterpret_cast<const char*>(base);
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const bool ok = (m >> e) & 1u;
    const uint32_t byte = 4u * (plane + (ok ? (uint32_t)(off + (e >> 2) * W + (e & 3)) : 0u));
    d[e] = *reinterpret_cast<const float*>(b + byte);
  }
}

__device__ __forceinline__ void zero_outside(float* d, unsigned m) {
#pragma unroll
  for (int e = 0; e < 16; ++e) d[e] = (m >> e) & 1u ? d[e] : 0.f;
}

template <int W>
__device__ __forceinline__ unsigned window_mask(int h0, int w0) {
  unsigned m = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if ((unsigned)(h0 + i) < (unsigned)W && (unsigned)(w0 + j) < (unsigned)W) m |= 1u << (4 * i + j);
  return m;
}

// Output of one lane: 4 output channels co4 .. co4 + 3 of output tile T (2 x 2 pixels each) with
// bias / ReLU / mask / accumulate.  Every operand (bias, ReLU-mask source, accumulate source) is
// requested before any is used, with clamped indices and only flag-level (uniform) branches:
// the previous per-pixel form waited for each load in turn (~40 dependent round trips per lane in
// the forward kernels' epilogues, visible as s_waitcnt vmcnt(0) before every use in the ISA).
template <int W>
__device__ __forceinline__ void wino_epilogue(const WinoArgs& a, const float (&yt)[4][2][2], int T, int ntiles,
                                              int co4, int sp) {
  constexpr int TW = W / 2, TPI = TW * TW, HW = W * W;
  const bool tok = T < ntiles;
  const int Tc = tok ? T : 0;
  const int n = Tc / TPI, rem = Tc - n * TPI, oh = 2 * (rem / TW), ow = 2 * (rem % TW);
  size_t o[4][2];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int p = 0; p < 2; ++p)
      o[r][p] = ((size_t)n * a.Co + min(co4 + r, a.Co - 1)) * HW + (size_t)(oh + p) * W + ow;
  float bv[4] = {0.f, 0.f, 0.f, 0.f};
  float2 mk[4][2], old[4][2];
  if (a.bias && sp == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[r] = a.bias[min(co4 + r, a.Co - 1)];
  }
  if (a.mask) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int p = 0; p < 2; ++p) mk[r][p] = *reinterpret_cast<const float2*>(a.mask + o[r][p]);
  }
  if (a.accumulate == 1) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int p = 0; p < 2; ++p) old[r][p] = *reinterpret_cast<const float2*>(a.y + o[r][p]);
  }
  if (!tok) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (co4 + r >= a.Co) continue;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      float2 v = make_float2(yt[r][p][0] + bv[r], yt[r][p][1] + bv[r]);
      if (a.accumulate == 2) {
        atomicAdd(a.y + o[r][p], v.x);
        atomicAdd(a.y + o[r][p] + 1, v.y);
        continue;
      }
      if (a.relu) { v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); }
      if (a.mask) {
        if (!(mk[r][p].x > 0.f)) v.x = 0.f;
        if (!(mk[r][p].y > 0.f)) v.y = 0.f;
      }
      if (a.accumulate == 1) {
        v.x += old[r][p].x;
        v.y += old[r][p].y;
      }
      *reinterpret_cast<float2*>(a.y + o[r][p]) = v;
    }
  }
}

// Block: 32 output channels x 32 output tiles; wave (wm, wn) owns 16 x 16 of it for all 16 xi
// (16 accumulators = 64 registers) -> ~120 VGPRs, 3 blocks (12 waves) per CU.
// KS = 2 (small images, where 32 x 32 blocks leave ~1 wave per SIMD): 8 waves per block in two
// K groups; group k handles the chunks of parity k with its own U / V buffers, so every barrier
// interval carries twice the MFMAs per SIMD, and the groups' partial outputs are summed through
// LDS after the output transform (deterministic, no atomics).
template <int W, int kOcc, int KS = 1>
__global__ __launch_bounds__(256 * KS, kOcc) void wino_fwd_kernel(WinoArgs a) {
  constexpr int TW = W / 2, TPI = TW * TW, HW = W * W;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int grp = KS > 1 ? (int)(threadIdx.x >> 8) : 0;
  float* As = sm + grp * (2 * 16 * kCC * kP);  // U slice [16][8 ci][kP] (32 co) of this K group
  float* Bs = As + 16 * kCC * kP;              // V slice [16][8 ci][kP] (32 tiles)
  const int tid = threadIdx.x & 255, lane = tid & 63, wave = tid >> 6, wm = wave >> 1, wn = wave & 1;
  const int g = lane >> 4, l16 = lane & 15;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int kt = bid % a.ktiles, r1 = bid / a.ktiles;
  const int tb = r1 % a.tblocks, sp = r1 / a.tblocks;
  const int co0 = kt * 32;
  const int ntiles = a.N * TPI;
  const int ch_beg = sp * a.chunks_per_split, ch_end = min(a.Cip / kCC, ch_beg + a.chunks_per_split);

  // transform role: tile tid & 31 of the block, input channel tid >> 5 of each chunk
  const int tt = tid & 31, cl = tid >> 5;
  const int my_t = tb * 32 + tt;
  const bool t_ok = my_t < ntiles;
  const int tn = t_ok ? my_t / TPI : 0, trem = t_ok ? my_t - tn * TPI : 0;
  const int th = trem / TW, tw = trem - th * TW;
  const unsigned vmask = t_ok ? window_mask<W>(2 * th - 1, 2 * tw - 1) : 0u;
  const uint32_t xn = (uint32_t)tn * a.Ci * HW;
  const int woff = (2 * th - 1) * W + 2 * tw - 1;
  // U slice copy role: 16 xi x 8 ci rows of 32 floats = 1024 float4, 4 per thread: thread t
  // copies float4 (t & 7) of row (xi, ci) = (4q + (t >> 6), (t >> 3) & 7), q = 0..3
  const uint32_t u_lane = 4u * (((uint32_t)(tid >> 6) * a.Cip + ((tid >> 3) & 7)) * a.Cop + co0 + 4 * (tid & 7));
  const uint32_t u_q = 4u * 4u * a.Cip * a.Cop, u_ch = 4u * kCC * a.Cop;  // byte strides
  float* as_st = As + (tid >> 3) * kP + 4 * (tid & 7);                       // + q * 32 rows

  float raw[16];
  f32x4 ru[4];
  unsigned rmask = 0;
  float2 rss = make_float2(1.f, 0.f);
  auto gload = [&](int ch) {
    const int c = ch * kCC + cl;
    rmask = c < a.Ci ? vmask : 0u;
    load_window<W>(a.x, xn + (uint32_t)min(c, a.Ci - 1) * HW, woff, rmask, raw);
    rss = load_ss(a.ss, min(c, a.Ci - 1));
    const char* ub = reinterpret_cast<const char*>(a.U) + (size_t)ch * u_ch;
#pragma unroll
    for (int q = 0; q < 4; ++q) ru[q] = *reinterpret_cast<const f32x4*>(ub + u_lane + q * u_q);
  };
  auto sstore = [&]() {
#pragma unroll
    for (int q = 0; q < 4; ++q) *reinterpret_cast<f32x4*>(as_st + q * 32 * kP) = ru[q];
    float v[16];
    if (a.ss) {
#pragma unroll
      for (int e = 0; e < 16; ++e) raw[e] = in_affine(raw[e], rss, a.in_relu);
    }
    zero_outside(raw, rmask);
    in_transform(raw, v);
#pragma unroll
    for (int xi = 0; xi < 16; ++xi) Bs[(xi * kCC + cl) * kP + tt] = v[xi];
  };

  f32x4 acc[16];
#pragma unroll
  for (int xi = 0; xi < 16; ++xi) acc[xi] = f32x4{0.f, 0.f, 0.f, 0.f};

  const float* ap = As + g * kP + 16 * wm + l16;
  const float* bp = Bs + g * kP + 16 * wn + l16;
  // K group grp takes chunks ch_beg + grp, + KS, ...; every group runs the same number of
  // iterations (barriers are block-wide), a group past the end just waits them out
  const int npass = (ch_end - ch_beg + KS - 1) / KS;
  if (ch_beg + grp < ch_end) gload(ch_beg + grp);
  for (int it = 0; it < npass; ++it) {
    const int ch = ch_beg + it * KS + grp;
    if (it != 0) __syncthreads();  // previous chunk's LDS reads are done
    if (ch < ch_end) sstore();
    __syncthreads();
    if (ch + KS < ch_end) gload(ch + KS);
    if (ch < ch_end) mfma_chunk<true>(ap, bp, acc);
  }

  // epilogue: row = output channel, column = output tile; Y = A^T M A, A^T = [[1,1,1,0],[0,1,-1,-1]]
  float yt[4][2][2];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float t0[4], t1[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      t0[c] = acc[0 + c][r] + acc[4 + c][r] + acc[8 + c][r];
      t1[c] = acc[4 + c][r] - acc[8 + c][r] - acc[12 + c][r];
    }
    yt[r][0][0] = t0[0] + t0[1] + t0[2];
    yt[r][0][1] = t0[1] - t0[2] - t0[3];
    yt[r][1][0] = t1[0] + t1[1] + t1[2];
    yt[r][1][1] = t1[1] - t1[2] - t1[3];
  }
  if constexpr (KS > 1) {  // group 1's partial outputs -> LDS -> added by group 0 (fixed order)
    float* red = sm + (wave * 64 + lane) * 16;  // 16 KB, over group 0's (finished) U / V buffers
    __syncthreads();
    if (grp == 1) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        *reinterpret_cast<float4*>(red + 4 * r) = make_float4(yt[r][0][0], yt[r][0][1], yt[r][1][0], yt[r][1][1]);
    }
    __syncthreads();
    if (grp == 1) return;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float4 o = *reinterpret_cast<const float4*>(red + 4 * r);
      yt[r][0][0] += o.x;
      yt[r][0][1] += o.y;
      yt[r][1][0] += o.z;
      yt[r][1][1] += o.w;
    }
  }
  wino_epilogue<W>(a, yt, tb * 32 + 16 * wn + l16, ntiles, co0 + 16 * wm + 4 * g, sp);
}

// ------------------------------------------------------------------------------------------
// Forward / data gradient, patch-staged (the default): block = 32 output channels x 64 output
// tiles, 4 waves in 2 x 2, each 16 channels x 32 tiles (2 MFMA tiles) x 16 xi = 128 accumulator
// registers, 2 blocks (8 waves) per CU.  Per chunk of 8 input channels the block's zero-padded
// input patch (full rows: 8 x 10 x 34 for 32x32 images, the whole 18 x 18 image for 16x16, four
// 10 x 10 images for 8x8) is staged in LDS from coalesced row loads whose offsets and border
// masks are computed once per thread; each thread then reads its two 4x4 windows from the patch
// with constant offsets, transforms them and writes V.  Compared with per-window global loads
// this moves ~2.5x fewer bytes per MFMA through the load path and removes the per-element mask
// arithmetic.  Pipeline per chunk (two barriers):
//   A: U(ch) regs -> LDS, patch(ch) windows -> V in LDS
//   B: patch(ch+1) regs -> LDS patch (its reads ended at B); issue U(ch+1), patch(ch+2) loads;
//      64 MFMAs per wave on U(ch), V(ch)
template <int W>
struct PatchGeom {
  static constexpr int TW = W / 2, TPI = TW * TW, HW = W * W;
  static constexpr int IMGS = TPI >= 64 ? 1 : 64 / TPI;   // images per block
  static constexpr int TR = (TPI >= 64 ? 64 : TPI) / TW;  // tile rows per image in the block
  static constexpr int PRI = 2 * TR + 2, PW = W + 2;      // patch rows per image, patch row width
  static constexpr int P1 = IMGS * PRI * PW;              // patch floats per channel
  static constexpr int EP = (kCC * P1 + 255) / 256;       // patch floats per thread per chunk
  static constexpr int kBP = 80;                          // V pitch (64 tiles + 16)
  static constexpr int AS = 16 * kCC * kP, BS = 16 * kCC * kBP, PS = kCC * P1;
};

template <int W>
__global__ __launch_bounds__(256, 2) void wino_fwd_patch_kernel(WinoArgs a) {
  using G = PatchGeom<W>;
  constexpr int TW = G::TW, TPI = G::TPI, HW = G::HW, PRI = G::PRI, PW = G::PW, P1 = G::P1, EP = G::EP;
  constexpr int kBP = G::kBP;
  __shared__ __attribute__((aligned(16))) float As[G::AS];  // U slice [16][8 ci][kP] (32 co)
  __shared__ __attribute__((aligned(16))) float Bs[G::BS];  // V slice [16][8 ci][kBP] (64 tiles)
  __shared__ __attribute__((aligned(16))) float Ps[G::PS];  // input patch [8 ci][IMGS][PRI][PW]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave >> 1, wn = wave & 1;
  const int g = lane >> 4, l16 = lane & 15;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int kt = bid % a.ktiles, r1 = bid / a.ktiles;
  const int tb = r1 % a.tblocks, sp = r1 / a.tblocks;
  const int co0 = kt * 32;
  const int ntiles = a.N * TPI;
  const int ch_beg = sp * a.chunks_per_split, ch_end = min(a.Cip / kCC, ch_beg + a.chunks_per_split);
  // first tile of the block -> first image and first tile row
  const int T0 = tb * 64, n0 = T0 / TPI, th0 = (T0 - n0 * TPI) / TW;

  // ---- patch load role (loop-invariant offsets + spatial masks, computed once)
  uint32_t poff[EP];
  unsigned pvalid = 0;  // bit i: element i is inside the image (and the block's images)
  int pci[EP];          // channel within the chunk of element i (>= kCC: no element)
#pragma unroll
  for (int i = 0; i < EP; ++i) {
    const int e = tid + 256 * i;
    const int ci = e / P1, rem = e - ci * P1;
    const int il = rem / (PRI * PW), r2 = rem - il * (PRI * PW), pr = r2 / PW, pc = r2 - pr * PW;
    const int n = n0 + il, h = 2 * th0 - 1 + pr, w = pc - 1;
    const bool ok = e < kCC * P1 && n < a.N && (unsigned)h < (unsigned)W && (unsigned)w < (unsigned)W;
    pci[i] = e < kCC * P1 ? ci : kCC;
    poff[i] = ok ? (uint32_t)((n * a.Ci + ci) * HW + h * W + w) : 0u;
    if (ok) pvalid |= 1u << i;
  }
  float rp[EP];
  auto pload = [&](int ch) {  // patch of chunk ch -> registers (masked at store time)
    const uint32_t cbase = (uint32_t)(ch * kCC) * HW;
#pragma unroll
    for (int i = 0; i < EP; ++i) rp[i] = a.x[((pvalid >> i) & 1u) ? poff[i] + cbase : 0u];
  };
  auto pstore = [&](int ch) {
#pragma unroll
    for (int i = 0; i < EP; ++i) {
      const int e = tid + 256 * i;
      const bool ok = ((pvalid >> i) & 1u) && ch * kCC + pci[i] < a.Ci;
      if (e < kCC * P1) Ps[e] = ok ? rp[i] : 0.f;
    }
  };

  // ---- U copy role: 16 xi x 8 ci rows of 32 floats = 1024 float4, 4 per thread
  const uint32_t u_lane = 4u * (((uint32_t)(tid >> 6) * a.Cip + ((tid >> 3) & 7)) * a.Cop + co0 + 4 * (tid & 7));
  const uint32_t u_q = 4u * 4u * a.Cip * a.Cop, u_ch = 4u * kCC * a.Cop;  // byte strides
  float* as_st = As + (tid >> 3) * kP + 4 * (tid & 7);                       // + q * 32 rows
  f32x4 ru[4];
  auto uload = [&](int ch) {
    const char* ub = reinterpret_cast<const char*>(a.U) + (size_t)ch * u_ch;
#pragma unroll
    for (int q = 0; q < 4; ++q) ru[q] = *reinterpret_cast<const f32x4*>(ub + u_lane + q * u_q);
  };

  // ---- transform role: tile tid & 63, channels (tid >> 6) and (tid >> 6) + 4 of the chunk
  const int tt = tid & 63, csub = tid >> 6;
  int wbase;
  {
    const int il = tt / (G::TR * TW), rem = tt - il * (G::TR * TW), trw = rem / TW, tcl = rem - trw * TW;
    wbase = il * PRI * PW + 2 * trw * PW + 2 * tcl;
  }


  f32x4 acc[16][2];
#pragma unroll
  for (int xi = 0; xi < 16; ++xi)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[xi][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const float* ap = As + g * kP + 16 * wm + l16;
  const float* bp = Bs + g * kBP + 32 * wn + l16;
  if (ch_beg < ch_end) {
    pload(ch_beg);
    uload(ch_beg);
    pstore(ch_beg);  // waits for the first patch only
    if (ch_beg + 1 < ch_end) pload(ch_beg + 1);
  }
  for (int ch = ch_beg; ch < ch_end; ++ch) {
    __syncthreads();  // A: previous MFMAs done with As/Bs; patch(ch) visible
#pragma unroll
    for (int q = 0; q < 4; ++q) *reinterpret_cast<f32x4*>(as_st + q * 32 * kP) = ru[q];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int cl = csub + 4 * p;
      const float* src = Ps + cl * P1 + wbase;
      float d[16], v[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) d[e] = src[(e >> 2) * PW + (e & 3)];
      in_transform(d, v);
#pragma unroll
      for (int xi = 0; xi < 16; ++xi) Bs[(xi * kCC + cl) * kBP + tt] = v[xi];
    }
    __syncthreads();  // B: V(ch) complete; patch(ch) reads done
    if (ch + 1 < ch_end) {
      pstore(ch + 1);
      uload(ch + 1);
      if (ch + 2 < ch_end) pload(ch + 2);
    }
#pragma unroll
    for (int xi = 0; xi < 16; ++xi)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int ro = xi * kCC + 4 * s;
        const float av = ap[ro * kP];
        acc[xi][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bp[ro * kBP], acc[xi][0], 0, 0, 0);
        acc[xi][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bp[ro * kBP + 16], acc[xi][1], 0, 0, 0);
      }
  }

  // epilogue: row = output channel, column = output tile; Y = A^T M A, A^T = [[1,1,1,0],[0,1,-1,-1]]
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int T = tb * 64 + 32 * wn + 16 * j + l16;
    float yt[4][2][2];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float t0[4], t1[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        t0[c] = acc[0 + c][j][r] + acc[4 + c][j][r] + acc[8 + c][j][r];
        t1[c] = acc[4 + c][j][r] - acc[8 + c][j][r] - acc[12 + c][j][r];
      }
      yt[r][0][0] = t0[0] + t0[1] + t0[2];
      yt[r][0][1] = t0[1] - t0[2] - t0[3];
      yt[r][1][0] = t1[0] + t1[1] + t1[2];
      yt[r][1][1] = t1[1] - t1[2] - t1[3];
    }
    wino_epilogue<W>(a, yt, T, ntiles, co0 + 16 * wm + 4 * g, sp);
  }
}

// ------------------------------------------------------------------------------------------
struct WinoWArgs {
  const float* dy;  // [N][K][W][W]
  const float* x;   // [N][C][W][W]
  float* out;       // nblk == 1: dw [K][C][3][3]; else partials [nblk][K][C][9]
  int N, C, K;
  int ktiles, ctiles, nchunks, chunks_per_block;
  int accumulate;   // nblk == 1 only: dw += result
  const float2* ss; // [C] (scale, shift) of a folded BN on x (WinoArgs::ss), or null
  int in_relu;
};

// Block: 32 co x 32 ci x a range of 8-tile chunks; wave (wm, wn) owns 16 co x 16 ci for all 16 xi.
template <int W>
__global__ __launch_bounds__(256, 3) void wino_wgrad_kernel(WinoWArgs a) {
  constexpr int TW = W / 2, TPI = TW * TW, HW = W * W;
  static_assert(TPI % 8 == 0, "8-tile chunks must not straddle images");
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* As = sm;                   // transformed dy [16][8 tiles][kP] (32 co)
  float* Bs = sm + 16 * kCC * kP;   // transformed x  [16][8 tiles][kP] (32 ci)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave >> 1, wn = wave & 1;
  const int g = lane >> 4, l16 = lane & 15;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int kt = bid % a.ktiles, r1 = bid / a.ktiles;
  const int ct = r1 % a.ctiles, rb = r1 / a.ctiles;
  const int k0 = kt * 32, c0 = ct * 32;
  const int ch_beg = rb * a.chunks_per_block, ch_end = min(a.nchunks, ch_beg + a.chunks_per_block);

  const int tt = tid & 7, cl = tid >> 3;  // tile within the chunk; channel row (co for dy, ci for x)
  const bool k_ok = k0 + cl < a.K, c_ok = c0 + cl < a.C;
  const float* dyk = a.dy + (size_t)min(k0 + cl, a.K - 1) * HW;
  const uint32_t xc = (uint32_t)min(c0 + cl, a.C - 1) * HW;
  const float2 xss = load_ss(a.ss, min(c0 + cl, a.C - 1));  // this thread's channel
  float rdy[4], rx[16];
  unsigned xmask = 0;
  auto gload = [&](int ch) {
    const int T = ch * 8 + tt, n = T / TPI, rem = T - n * TPI, th = rem / TW, tw = rem - th * TW;
    const float* p = dyk + (size_t)n * a.K * HW + (2 * th) * W + 2 * tw;
    const float2 r0 = *reinterpret_cast<const float2*>(p), r1v = *reinterpret_cast<const float2*>(p + W);
    rdy[0] = r0.x;
    rdy[1] = r0.y;
    rdy[2] = r1v.x;
    rdy[3] = r1v.y;
    xmask = c_ok ? window_mask<W>(2 * th - 1, 2 * tw - 1) : 0u;
    load_window<W>(a.x, xc + (uint32_t)n * a.C * HW, (2 * th - 1) * W + 2 * tw - 1, xmask, rx);
  };
  // LDS column swizzle: col ^ 4 * ((row >> 1) & 3).  The transform stores put 8 tile rows x 4
  // columns in each 32-lane group; with the plain pitch-48 layout rows 0, 2, 4, 6 hit the same
  // 32-bank column (4-way conflicts on every store, more conflict cycles than LDS-active cycles
  // in the r1 counters).  The MFMA operand reads stay conflict-free: the XOR only permutes
  // columns inside each 16-aligned group.
  const int cs = cl ^ (4 * ((tt >> 1) & 3));
  auto sstore = [&]() {
    float v[16];
#pragma unroll
    for (int i = 0; i < 4; ++i) rdy[i] = k_ok ? rdy[i] : 0.f;
    if (a.ss) {
#pragma unroll
      for (int e = 0; e < 16; ++e) rx[e] = in_affine(rx[e], xss, a.in_relu);
    }
    zero_outside(rx, xmask);
    dy_transform(rdy, v);
#pragma unroll
    for (int xi = 0; xi < 16; ++xi) As[(xi * kCC + tt) * kP + cs] = v[xi];
    in_transform(rx, v);
#pragma unroll
    for (int xi = 0; xi < 16; ++xi) Bs[(xi * kCC + tt) * kP + cs] = v[xi];
  };

  f32x4 acc[16];
#pragma unroll
  for (int xi = 0; xi < 16; ++xi) acc[xi] = f32x4{0.f, 0.f, 0.f, 0.f};

  // operand rows 4s + g of every xi block: swizzle 4 * ((2s + (g >> 1)) & 3) per k-step s
  const int sw0 = 4 * ((g >> 1) & 3), sw1 = 4 * ((2 + (g >> 1)) & 3);
  const float* ap0 = As + g * kP + ((16 * wm + l16) ^ sw0);
  const float* ap1 = As + g * kP + ((16 * wm + l16) ^ sw1);
  const float* bp0 = Bs + g * kP + ((16 * wn + l16) ^ sw0);
  const float* bp1 = Bs + g * kP + ((16 * wn + l16) ^ sw1);
  if (ch_beg < ch_end) gload(ch_beg);
  for (int ch = ch_beg; ch < ch_end; ++ch) {
    if (ch != ch_beg) __syncthreads();
    sstore();
    __syncthreads();
    if (ch + 1 < ch_end) gload(ch + 1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int xi = 0; xi < 16; ++xi) {
        const int ro = (xi * kCC + 4 * s) * kP;
        acc[xi] = __builtin_amdgcn_mfma_f32_16x16x4f32(s ? ap1[ro] : ap0[ro], s ? bp1[ro] : bp0[ro], acc[xi], 0, 0, 0);
      }
  }

  // epilogue: row = co, column = ci; dW = A'^T M A', A'^T = [[1,1,1,0],[0,1,-1,0],[0,1,1,-1]]
  const int ci = c0 + 16 * wn + l16;
  if (ci >= a.C) return;
  const size_t pstride = ((size_t)a.K * a.C * 9 + 3) & ~(size_t)3;  // 16-byte aligned partial planes
  float* dst_base = a.out + (size_t)rb * pstride;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int co = k0 + 16 * wm + 4 * g + r;
    if (co >= a.K) continue;
    float t[3][4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float m0 = acc[c][r], m1 = acc[4 + c][r], m2 = acc[8 + c][r], m3 = acc[12 + c][r];
      t[0][c] = m0 + m1 + m2;
      t[1][c] = m1 - m2;
      t[2][c] = m1 + m2 - m3;
    }
    float* dst = dst_base + ((size_t)co * a.C + ci) * 9;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      float v0 = t[ky][0] + t[ky][1] + t[ky][2], v1 = t[ky][1] - t[ky][2], v2 = t[ky][1] + t[ky][2] - t[ky][3];
      if (a.accumulate) {
        v0 += dst[3 * ky];
        v1 += dst[3 * ky + 1];
        v2 += dst[3 * ky + 2];
      }
      dst[3 * ky] = v0;
      dst[3 * ky + 1] = v1;
      dst[3 * ky + 2] = v2;
    }
  }
}

// dw (+)= sum over nblk partial planes (fixed order -> deterministic).  Block = (256 / G) float4
// quads x G plane groups: thread (q, g) sums planes g, g + G, g + 2G, g + 3G, ... of its quad with
// four loads in flight per iteration, then the G group sums are combined by a fixed-shape LDS
// tree.  G is picked so a thread sums at most ~4 planes: the small stage-1 PyramidNet layers
// have 256 planes of only ~4 K floats, and a thread walking 16 of them as a dependent chain made
// those reductions latency-bound (22-43 us for ~4 MB).
__device__ __forceinline__ void wino_reduce_body(const float* __restrict__ part, float* __restrict__ dw, int64_t plane,
                                                 int64_t pstride, int nblk, int accumulate, int G, int blk,
                                                 int nblocks) {
  // partial plane b starts at part + b * pstride (pstride = plane rounded up to 4 floats)
  __shared__ float4 red[256];
  const int64_t n4 = plane >> 2, s4 = pstride >> 2;
  const int QB = 256 / G, q = threadIdx.x % QB, g = threadIdx.x / QB;
  const int64_t i = (int64_t)blk * QB + q;
  const float4* p4 = reinterpret_cast<const float4*>(part);
  float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n4) {
    for (int b = g; b < nblk; b += 4 * G) {
      float4 u[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int bb = b + k * G;
        u[k] = bb < nblk ? p4[bb * s4 + i] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        t.x += u[k].x; t.y += u[k].y; t.z += u[k].z; t.w += u[k].w;
      }
    }
  }
  red[threadIdx.x] = t;
  __syncthreads();
  for (int st = G >> 1; st > 0; st >>= 1) {
    if (g < st) {
      const float4 v = red[threadIdx.x + st * QB];
      float4& r = red[threadIdx.x];
      r.x += v.x; r.y += v.y; r.z += v.z; r.w += v.w;
    }
    __syncthreads();
  }
  if (g == 0 && i < n4) {
    float4 r = red[threadIdx.x];
    float4* d4 = reinterpret_cast<float4*>(dw);
    if (accumulate) {
      const float4 o = d4[i];
      r.x += o.x; r.y += o.y; r.z += o.z; r.w += o.w;
    }
    d4[i] = r;
  }
  // tail (plane % 4 <= 3 floats): one wave per float in the last block, lanes stride over the
  // planes, fixed-shape wave sum (a single thread walking 256 planes took tens of us)
  const int tail = (int)(plane - (n4 << 2));
  if (tail > 0 && blk == nblocks - 1 && (int)(threadIdx.x >> 6) < tail) {
    const int lane = threadIdx.x & 63;
    const int64_t k = (n4 << 2) + (threadIdx.x >> 6);
    float v = 0.f;
    for (int b = lane; b < nblk; b += 64) v += part[b * pstride + k];
    v = wave_sum(v);
    if (lane == 0) dw[k] = (accumulate ? dw[k] : 0.f) + v;
  }
}

__global__ __launch_bounds__(256) void wino_wgrad_reduce_k(const float* __restrict__ part, float* __restrict__ dw,
                                                            int64_t plane, int64_t pstride, int nblk, int accumulate,
                                                            int G) {
  wino_reduce_body(part, dw, plane, pstride, nblk, accumulate, G, blockIdx.x, gridDim.x);
}

// many deferred reductions in one launch (wgrad_defer.h): block b runs job q's block b - blk0[q]
__global__ __launch_bounds__(256) void wino_wgrad_reduce_batch_k(RedBatch bt) {
  int q = 0;
  for (int k = 1; k < bt.n; ++k)
    if ((int)blockIdx.x >= bt.j[k].blk0) q = k;
  const RedJob& jb = bt.j[q];
  wino_reduce_body(jb.part, jb.dw, jb.plane, jb.pstride, jb.nplanes, jb.acc, jb.G, (int)blockIdx.x - jb.blk0,
                   jb.blocks);
}

// same reduction for a destination that is not 16-byte aligned
__global__ void wino_wgrad_reduce_scalar_k(const float* __restrict__ part, float* __restrict__ dw, int64_t plane,
                                           int64_t pstride, int nblk, int accumulate) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < plane; i += (int64_t)gridDim.x * 256) {
    float t = accumulate ? dw[i] : 0.f;
    for (int b = 0; b < nblk; ++b) t += part[b * pstride + i];
    dw[i] = t;
  }
}

int pad_to(int v, int m) { return (v + m - 1) / m * m; }

void launch_fwd(const float* x, const float* w, const float* bias, const float* mask, float* y, int N, int Ci,
                int Co, int Wd, bool relu, bool accumulate, bool dgrad, float* U, int K_w, int C_w,
                hipStream_t st, float* U_dgrad_out = nullptr, bool pretransformed = false,
                const float* in_ss = nullptr, bool in_relu = false) {
  const int Cip = pad_to(Ci, kCC), Cop = pad_to(Co, 32);
  if (U_dgrad_out) {  // forward call that also prepares the backward's filters (one launch)
    const int Cipd = pad_to(K_w, kCC), Copd = pad_to(C_w, 32);
    const int total = Cip * Cop + Cipd * Copd;
    MX_LAUNCH(wino_wtrans2_k, dim3(std::min(cdiv(total, 256), 2048)), dim3(256), 0, st, w, U, U_dgrad_out, K_w, C_w,
              Cip, Cop, Cipd, Copd);
  } else if (!pretransformed) {
    const int total = Cip * Cop;
    MX_LAUNCH(wino_wtrans_k, dim3(std::min(cdiv(total, 256), 2048)), dim3(256), 0, st, w, U, K_w, C_w, Cip, Cop,
              dgrad ? 1 : 0);
  }
  WinoArgs a{};
  a.x = x;
  a.U = U;
  a.bias = bias;
  a.mask = mask;
  a.y = y;
  a.N = N;
  a.Ci = Ci;
  a.Co = Co;
  a.Cip = Cip;
  a.Cop = Cop;
  // 3 = patch-staged 32 x 64 blocks (fastest on 32x32 images), 2 = per-window 32 x 32 blocks
  // (fastest on 16x16 / 8x8, where the larger block leaves too few blocks to fill the chip);
  // measured per shape by scripts/bench_conv.py.
  const int tpi = (Wd / 2) * (Wd / 2);
  // 4 = two K groups per 32 x 32 block: where the 32 x 32 grid fits in one wave of blocks (one
  // block per CU, e.g. the 8x8 layers up to 256 channels), doubling the MFMAs per barrier
  // interval wins (45 -> 39 us at C = 191, 57 -> 49 us at C = 231); with more blocks than CUs it
  // loses (89 -> 99 us at C = 266: two waves of 98 KB-LDS blocks), as on 16x16 / 32x32
  // 32x32 images with one 32-channel output tile (the first stage-1 layers): the 32 x 64 patch
  // blocks leave one block per CU and the 32 x 32 blocks win (11.7 vs 14.5 us at C = 16)
  const int blocks32 = cdiv(N * tpi, 32) * (Cop / 32), cus = device_cu_count();
  // (a folded BN input runs the per-window kernels: the patch kernel stages raw rows in LDS)
  int variant = Wd == 32 && !in_ss ? (blocks32 / 2 >= 2 * cus ? 3 : 2) : (blocks32 <= cus ? 4 : 2);
  // A/B (scripts/bench_conv.py --only-wino): MXDDP_WINO_FWD = 2 / 3 / 4 forces a variant (3 only
  // without a folded input affine)
  static const int forced = [] {
    const char* e = std::getenv("MXDDP_WINO_FWD");
    return e ? std::atoi(e) : 0;
  }();
  if (forced >= 2 && forced <= 4 && !(forced == 3 && in_ss)) variant = forced;
  const int tile_blk = variant == 3 ? 64 : 32;
  a.tblocks = cdiv(N * tpi, tile_blk);
  a.ktiles = Cop / 32;
  // One block per (tile group, output-channel tile) over all input channels.  (Measured with
  // scripts/bench_conv.py: splitting the input channels over blocks with atomic accumulation
  // LOSES on every PyramidNet shape -- 8x8: 63 vs 45 us -- the atomics and the output memset
  // cost more than the extra blocks gain; removed.)
  a.chunks_per_split = Cip / kCC;
  a.splits = 1;
  a.relu = relu;
  a.accumulate = accumulate ? 1 : 0;
  a.ss = reinterpret_cast<const float2*>(in_ss);
  a.in_relu = in_relu ? 1 : 0;
  const dim3 grid(a.tblocks * a.ktiles * a.splits);
  if (variant == 3) {
    switch (Wd) {
      case 8: MX_LAUNCH(wino_fwd_patch_kernel<8>, grid, dim3(256), 0, st, a); break;
      case 16: MX_LAUNCH(wino_fwd_patch_kernel<16>, grid, dim3(256), 0, st, a); break;
      case 32: MX_LAUNCH(wino_fwd_patch_kernel<32>, grid, dim3(256), 0, st, a); break;
      default: MX_CHECK(false, "winograd: unsupported width");
    }
    return;
  }
  if (variant == 4) {  // two K groups of 4 waves per block (see wino_fwd_kernel)
    static bool attr = false;
    if (!attr) {
      for (const void* fn : {reinterpret_cast<const void*>(wino_fwd_kernel<8, 1, 2>),
                             reinterpret_cast<const void*>(wino_fwd_kernel<16, 1, 2>),
                             reinterpret_cast<const void*>(wino_fwd_kernel<32, 1, 2>)})
        MX_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(2 * kLds)));
      attr = true;
    }
    switch (Wd) {
      case 8: MX_LAUNCH((wino_fwd_kernel<8, 1, 2>), grid, dim3(512), 2 * kLds, st, a); break;
      case 16: MX_LAUNCH((wino_fwd_kernel<16, 1, 2>), grid, dim3(512), 2 * kLds, st, a); break;
      case 32: MX_LAUNCH((wino_fwd_kernel<32, 1, 2>), grid, dim3(512), 2 * kLds, st, a); break;
      default: MX_CHECK(false, "winograd: unsupported width");
    }
    return;
  }
  // 2 waves / SIMD: at 3 (launch bounds 256, 3) 17 VGPRs spill and every shape runs 20-70 % slower
  // (round 6, profiles/r6_winovar/occ3_*.log; e.g. 126 -> 131 at 16 x 16: 67.6 -> 82.3 us)
  switch (Wd) {
    case 8: MX_LAUNCH((wino_fwd_kernel<8, 2>), grid, dim3(256), kLds, st, a); break;
    case 16: MX_LAUNCH((wino_fwd_kernel<16, 2>), grid, dim3(256), kLds, st, a); break;
    case 32: MX_LAUNCH((wino_fwd_kernel<32, 2>), grid, dim3(256), kLds, st, a); break;
    default: MX_CHECK(false, "winograd: unsupported width");
  }
}

struct WgradPlan {
  int ktiles, ctiles, nchunks, cpb, nblk;
};
// resident weight-gradient blocks aimed at per CU (A/B: wino_wgrad_set_slots).  With the
// batched deferred reductions (round 6), on one box: 2 / 3 / 4 per CU = 2,915-2,921 / 2,958 /
// 2,900-2,902 img/s on PyramidNet-110 (profiles/r6_winoslots/)
int g_wgrad_slots_per_cu = 3;
WgradPlan wgrad_plan(const ConvShape& s) {
  WgradPlan p{};
  p.ktiles = cdiv(s.K, 32);
  p.ctiles = cdiv(s.C, 32);
  p.nchunks = s.N * (s.W / 2) * (s.W / 2) / 8;
  // ~3 blocks per CU, >= 8 chunks (256 MFMAs per wave) per block; the partial planes capped at
  // 8M floats of scratch (small layers may use many, large ones at least 16).  Filling the chip
  // wins over partial-sum traffic: with a 2M cap the PyramidNet step lost 3 ms of wgrad time to
  // gain 1 ms of reduction time.
  const int tiles = p.ktiles * p.ctiles;
  const int cap = std::max(16, (int)std::min<int64_t>(1024, (8ll << 20) / ((int64_t)s.K * s.C * 9)));
  // The grid must not exceed the 3 x 256 resident slots: a few blocks over (e.g. 25 tiles x 31
  // ranges = 775) run as a second round and nearly double the kernel time.
  const int slots = g_wgrad_slots_per_cu * device_cu_count();
  int nblk = std::max(1, std::min(slots / tiles, cap));
  nblk = std::min(nblk, std::max(1, p.nchunks / 8));
  p.cpb = cdiv(p.nchunks, nblk);
  p.nblk = cdiv(p.nchunks, p.cpb);
  return p;
}

}  // namespace

bool wino_eligible(const ConvShape& s) {
  return s.R == 3 && s.S == 3 && s.str_h == 1 && s.str_w == 1 && s.pad_h == 1 && s.pad_w == 1 && s.dil_h == 1 &&
         s.dil_w == 1 && s.H == s.W && s.P == s.H && s.Q == s.W && (s.W == 8 || s.W == 16 || s.W == 32);
}

size_t wino_scratch_floats(const ConvShape& s) {
  // fwd: Cip(C) x Cop(K); dgrad: Cip(K) x Cop(C)
  const size_t f = (size_t)pad_to(s.C, kCC) * pad_to(s.K, 32), d = (size_t)pad_to(s.K, kCC) * pad_to(s.C, 32);
  return 16 * std::max(f, d);
}

size_t wino_wgrad_scratch_floats(const ConvShape& s) {
  const WgradPlan p = wgrad_plan(s);
  return p.nblk > 1 ? (size_t)p.nblk * (((size_t)s.K * s.C * 9 + 3) & ~(size_t)3) : 0;
}

void wino_fwd(const float* x, const float* w, const float* bias, float* y, const ConvShape& s, bool relu,
              float* scratch, hipStream_t st, float* U_dgrad_out, bool pretransformed, const float* in_ss,
              bool in_relu) {
  launch_fwd(x, w, bias, nullptr, y, s.N, s.C, s.K, s.W, relu, false, false, scratch, s.K, s.C, st,
             pretransformed ? nullptr : U_dgrad_out, pretransformed, in_ss, in_relu);
}

void wino_wgrad_set_slots(int per_cu) { g_wgrad_slots_per_cu = per_cu < 1 ? 1 : per_cu; }

size_t wino_fwd_filter_floats(const ConvShape& s) { return 16 * (size_t)pad_to(s.C, kCC) * pad_to(s.K, 32); }

void WinoFilterBank::add(const float* w, float* U_fwd, float* U_dgrad, int K, int C) {
  MX_CHECK(w && U_fwd, "filter bank: weight and forward filter buffer required");
  jobs_.push_back(Job{w, U_fwd, U_dgrad, K, C});
}

void WinoFilterBank::refresh(hipStream_t st) const {
  for (size_t b0 = 0; b0 < jobs_.size(); b0 += kWFMaxJobs) {
    WFBatch bt{};
    int blocks = 0;
    bt.n = (int)std::min<size_t>(kWFMaxJobs, jobs_.size() - b0);
    for (int q = 0; q < bt.n; ++q) {
      const Job& j = jobs_[b0 + q];
      WFJob& J = bt.j[q];
      J.w = j.w;
      J.Uf = j.Uf;
      J.Ud = j.Ud;
      J.K = j.K;
      J.C = j.C;
      J.Cipf = pad_to(j.C, kCC);
      J.Copf = pad_to(j.K, 32);
      J.Cipd = pad_to(j.K, kCC);
      J.Copd = pad_to(j.C, 32);
      J.blk0 = blocks;
      blocks += cdiv(J.Cipf * J.Copf + (j.Ud ? J.Cipd * J.Copd : 0), 256);
    }
    MX_LAUNCH(wino_wtrans_batch_k, dim3(blocks), dim3(256), 0, st, bt);
  }
}

size_t wino_dgrad_filter_floats(const ConvShape& s) { return 16 * (size_t)pad_to(s.K, kCC) * pad_to(s.C, 32); }

void wino_dgrad(const float* dy, const float* w, float* dx, const ConvShape& s, const float* relu_mask,
                bool accumulate, float* scratch, hipStream_t st, bool pretransformed) {
  launch_fwd(dy, w, nullptr, relu_mask, dx, s.N, s.K, s.C, s.W, false, accumulate, true, scratch, s.K, s.C, st,
             nullptr, pretransformed);
}

void wino_reduce_batch_launch(const RedBatch& b, int blocks, hipStream_t st) {
  MX_LAUNCH(wino_wgrad_reduce_batch_k, dim3(blocks), dim3(256), 0, st, b);
}

void wino_wgrad(const float* dy, const float* x, float* dw, const ConvShape& s, bool accumulate, float* scratch,
                hipStream_t st, const float* in_ss, bool in_relu) {
  const WgradPlan p = wgrad_plan(s);
  MX_CHECK(p.nblk == 1 || scratch, "winograd wgrad: partial-sum scratch required");
  WinoWArgs a{};
  a.dy = dy;
  a.x = x;
  a.out = p.nblk > 1 ? scratch : dw;
  a.N = s.N;
  a.C = s.C;
  a.K = s.K;
  a.ktiles = p.ktiles;
  a.ctiles = p.ctiles;
  a.nchunks = p.nchunks;
  a.chunks_per_block = p.cpb;
  a.accumulate = (p.nblk == 1 && accumulate) ? 1 : 0;
  a.ss = reinterpret_cast<const float2*>(in_ss);
  a.in_relu = in_relu ? 1 : 0;
  const dim3 grid(p.ktiles * p.ctiles * p.nblk);
  switch (s.W) {
    case 8: MX_LAUNCH(wino_wgrad_kernel<8>, grid, dim3(256), kLds, st, a); break;
    case 16: MX_LAUNCH(wino_wgrad_kernel<16>, grid, dim3(256), kLds, st, a); break;
    case 32: MX_LAUNCH(wino_wgrad_kernel<32>, grid, dim3(256), kLds, st, a); break;
    default: MX_CHECK(false, "winograd wgrad: unsupported width");
  }
  if (p.nblk > 1) {
    const int64_t plane = (int64_t)s.K * s.C * 9, pstride = (plane + 3) & ~(int64_t)3;
    if (reinterpret_cast<uintptr_t>(dw) & 15) {
      MX_LAUNCH(wino_wgrad_reduce_scalar_k, dim3((unsigned)std::min<int64_t>((plane + 255) / 256, 2048)), dim3(256), 0,
                st, scratch, dw, plane, pstride, p.nblk, accumulate ? 1 : 0);
      return;
    }
    int G = 1;  // plane groups per reduce block: each thread sums <= ~4 planes
    while (G < 64 && G * 4 < p.nblk) G *= 2;
    const int64_t blocks = std::max<int64_t>(1, (plane / 4 + 256 / G - 1) / (256 / G));
    MX_CHECK(blocks < (1ll << 31), "winograd wgrad: reduce grid too large");
    if (wgrad_defer_active()) {  // summed later by the optimizer's batched flush (wgrad_defer.h)
      RedJob j{};
      j.part = scratch;
      j.dw = dw;
      j.plane = plane;
      j.pstride = pstride;
      j.nplanes = p.nblk;
      j.G = G;
      j.acc = accumulate ? 1 : 0;
      j.kind = 0;
      j.blocks = (int)blocks;
      wgrad_defer_push(j);
      return;
    }
    MX_LAUNCH(wino_wgrad_reduce_k, dim3((unsigned)blocks), dim3(256), 0, st, scratch, dw, plane, pstride, p.nblk,
              accumulate ? 1 : 0, G);
  }
}

}  // namespace mx
