// Channels-last (NHWC) bf16 training kernels for gfx950: the ResNet-50 mixed-precision path
// (BASELINE.json config 5).  Activations are bf16 [N][H][W][C] (C a multiple of 8), master
// weights / gradients fp32 in torch layout [K][C][R][S], statistics and accumulation fp32.
//
// Why NHWC: every implicit-GEMM operand element is then a 16-byte vector of 8 consecutive
// channels of one pixel, so the im2col gather is one 16-byte load per (pixel, r, s, 8 channels)
// with a single bounds test, instead of a per-element index computation and 4-byte load as in
// NCHW.  The reduction dimension of the forward / data-gradient GEMM is (r, s, c) with c
// fastest, exactly the order of the MFMA operand fragments (8 consecutive k per lane).
//
// conv_nhwc_kernel   forward and data gradient.  GEMM rows = output channels (A = weights
//                    [Ng][R*S*Ca] bf16, k-contiguous), columns = output pixels (B = the 16-byte
//                    gather), v_mfma_f32_16x16x32_bf16, 128 x 128 (or 64 x 128) tiles, BK = 32,
//                    register-staged double-buffered LDS.  The C/D layout puts 4 consecutive
//                    output channels of one pixel in a lane: one 8-byte bf16 store each.
//                    Data gradient: the same GEMM over dy with weights [Cin][R][S][Kout] and
//                    the transposed-convolution gather (stride 1 or 2).
// wgrad_nhwc_kernel  dW[k][(r,s,c)] = sum_pixels dy[pix][k] x[pix'][c]: the reduction runs over
//                    pixels, which are the SLOW dimension of both NHWC operands, so the LDS
//                    tiles are stored pixel-major as loaded and read with the gfx950 transpose
//                    read ds_read_b64_tr_b16 (4 pixels x 16 channels per 16-lane group,
//                    delivered channel-major); split over pixel ranges into fp32 partial
//                    planes, summed in a fixed order and scattered to [K][C][R][S] by a second
//                    kernel (deterministic; no same-address atomics).
// BN / pooling       per-channel statistics with 8-channel vectors per thread; fused ReLU and
//                    fused residual add + ReLU (Bottleneck tail) in the apply kernels.
//
// Replaces (reference): cuDNN conv / BN via torch.nn in a channels_last + autocast(bf16)
// ResNet-50; BASELINE.json config 5 (not in the reference repository).
#include "common.h"
#include "igemm_bf16.h"
#include "ops.h"
#include "wgrad_defer.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace mx {

namespace {

using bf16 = unsigned short;
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // register-promotable (HIP's uint4 arrays are not)
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float bf2f(uint32_t v16) { return __uint_as_float(v16 << 16); }
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}
// 8 bf16 (one uint4) <-> 8 floats
__device__ __forceinline__ void unpack8(const uint4& u, float* f) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = bf2f(w[i] & 0xffffu);
    f[2 * i + 1] = bf2f(w[i] >> 16);
  }
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}
// bit e set <=> bf16 element e of the packed vector is > 0 (unpack8 order): the ReLU mask of a
// stored activation, 1/16 of its bytes
__device__ __forceinline__ uint32_t pos_bits8(const uint4& u) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
  uint32_t b = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    b |= (uint32_t)((int16_t)(w[i] & 0xffffu) > 0) << (2 * i);
    b |= (uint32_t)((int16_t)(w[i] >> 16) > 0) << (2 * i + 1);
  }
  return b;
}
// 8 bf16 c + 8 bf16 d, summed in fp32 and rounded once
__device__ __forceinline__ u32x4 add8(u32x4 c, u32x4 d) {
  float x[8], y[8];
  unpack8(make_uint4(c[0], c[1], c[2], c[3]), x);
  unpack8(make_uint4(d[0], d[1], d[2], d[3]), y);
#pragma unroll
  for (int e = 0; e < 8; ++e) x[e] += y[e];
  const uint4 r = pack8(x);
  return u32x4{r.x, r.y, r.z, r.w};
}
// the 8 bf16 of d with element e zeroed unless bit e of mb is set (ReLU mask bits)
__device__ __forceinline__ u32x4 mask8(u32x4 d, uint32_t mb) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
    d[j] &= ((mb >> (2 * j)) & 1u ? 0x0000ffffu : 0u) | ((mb >> (2 * j + 1)) & 1u ? 0xffff0000u : 0u);
  return d;
}
// 16-byte store with agent scope (sc1, a vector store): the line is not kept dirty in this XCD's
// L2, so a streaming output drains while the kernel runs instead of at its end
__device__ __forceinline__ void st16(void* p, const uint4& v, bool wt) {
  if (wt) {
    const u32x4 q = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(q) : "memory");
  } else {
    *reinterpret_cast<uint4*>(p) = v;
  }
}

// epilogue of a data gradient: the residual join's addend, optionally masked by its ReLU bits
__device__ __forceinline__ u32x4 join8(u32x4 v, const bf16* addend, const uint8_t* amask, size_t o) {
  u32x4 d = *reinterpret_cast<const u32x4*>(addend + o);
  if (amask) d = mask8(d, amask[o >> 3]);
  return add8(v, d);
}

// ------------------------------------------------------------------------------------------
// forward / data-gradient implicit GEMM
struct ConvNArgs {
  const bf16* act;  // gathered tensor [N][IH][IW][Ca]
  const bf16* wt;   // [Ng][Kg], Kg = R * S * Ca
  bf16* out;        // [M][Ng]  (M = N * OH * OW output pixels)
  int M, Ng, Kg, Ca;
  int OH, OW, IH, IW;
  int R, S, sh, sw, ph, pw;
  int dgrad;        // 0: y = conv(x); 1: dx = conv_transpose(dy) (sh, sw in {1, 2})
  int kt_per_split; // split-K: blockIdx.y covers k-tiles [y * kt_per_split, ...)
  float* part;      // split-K > 1: fp32 partials [splits][M][Ng] (else null: bf16 store)
  // par = 1 (stride-2 data gradient, even OH / OW, wide path): blockIdx.z = output parity class
  // (h & 1, w & 1); class pixels are (n, 2 i + h&1, 2 j + w&1), i < Hc, j < Wc, and only the
  // taps of matching parity contribute, so each class is a dense stride-1 GEMM over its own
  // taps (the zero-inserted transposed gather would multiply 3 zeros out of 4)
  int par, Hc, Wc;
  const bf16* addend;  // data gradient: added to the result in the epilogue ([M][Ng], or null) -- a
                       // residual block's two input-gradient branches joined without another pass
  const uint8_t* amask;  // addend masked by these ReLU bits (bit e of byte o / 8), or null: the
                         // identity shortcut's gradient taken straight from the block's output
                         // gradient, never materialised by the last BN's backward
  int owt;   // outputs stored write-through (g_conv_wt): bit 0 epilogue, 1 split-K partials, 2 reduce
  int asub;  // the addend is [N][OH / 2][OW / 2][Ng] and joins at even (h, w) only: a stride-2 1x1
             // projection shortcut's input gradient, computed compact (zero at the odd positions)
  // forward feeding a training BatchNorm (LDS-DMA kernel, no split): the epilogue writes the BN's
  // per-channel partial sums of (y - shift[c]) and its square over each 256-pixel tile to
  // bnpart[tile][2 Ng] (the layout bn_nhwc_partial_k writes), so the BN skips its statistics pass
  float* bnpart;
  const float* bnshift;  // per-channel shift (the BN's running mean: well conditioned), or null = 0
  // data gradient whose result is the output gradient of a training BatchNorm (the BN feeding
  // this conv): the epilogue also writes that BN's backward partial sums -- sum(g) and
  // sum(g (x - mean)), g = the stored gradient masked by the BN's fused ReLU -- per pixel tile to
  // bnpart (same layout as bn_nhwc_partial_k<true>), so the BN backward skips its statistics
  // pass over dy and x.  bx: the BN's input; bmean: its batch mean; the ReLU mask from the
  // forward's (scale, shift) (bfcoef, ReLU without residual) or from its mask bits (bmask), or none.
  const bf16* bx;
  const float* bmean;
  const float* bfcoef;
  const uint8_t* bmask;
  int brelu;
  FastDiv fOW, fOHW, fCa, fS, fWc, fHWc;
};

// Backward BN statistics of one 8-channel vector of the stored data gradient (see ConvNArgs::bx):
// g = v masked, s1 += g, s2 += g (x - mean).  The loads of x / mask are issued by the caller.
__device__ __forceinline__ void bn_bwd_acc8(const ConvNArgs& a, const u32x4& v, const uint4& xr, uint32_t mb,
                                            const float* mean8, const float* sc8, const float* sh8, float* s1,
                                            float* s2) {
  float g[8], xv[8];
  unpack8(make_uint4(v[0], v[1], v[2], v[3]), g);
  unpack8(xr, xv);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    if (a.brelu) {
      const bool live = a.bfcoef ? fmaf(xv[e], sc8[e], sh8[e]) > 0.f : ((mb >> e) & 1u) != 0u;
      g[e] = live ? g[e] : 0.f;
    }
    s1[e] += g[e];
    s2[e] = fmaf(g[e], xv[e] - mean8[e], s2[e]);
  }
}

// The per-thread sums of a fixed 8-channel vector cv (threads tid = cv mod VPR) reduced in a fixed
// order and written as partial row `row` (channels ch0 .. ch0 + 8 VPR - 1): first across the lanes
// of a wave that share cv (lane shuffles), then the NT / 64 wave partials through LDS by one
// thread per (cv, value).  (The former all-LDS version had 8 VPR threads each walk NT / VPR
// slots in series.)
template <int NT, int VPR>
__device__ __forceinline__ void bn_bwd_flush(const ConvNArgs& a, float* red, const float* s1, const float* s2,
                                             int row, int ch0) {
  static_assert(64 % VPR == 0 || VPR == 64, "a channel vector's threads tile the wave");
  constexpr int NW = NT / 64;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  float v[16];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    v[e] = s1[e];
    v[8 + e] = s2[e];
  }
#pragma unroll
  for (int off = VPR; off < 64; off <<= 1)
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] += __shfl_xor(v[j], off);
  if (lane < VPR) {
#pragma unroll
    for (int j = 0; j < 16; ++j) red[(j * NW + wv) * VPR + lane] = v[j];
  }
  __syncthreads();
  if (tid < 16 * VPR) {
    const int j = tid / VPR, cv = tid - j * VPR;
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) t += red[(j * NW + w) * VPR + cv];
    const int e = j & 7, ch = ch0 + 8 * cv + e;
    if (ch < a.Ng) a.bnpart[(size_t)row * 2 * a.Ng + 2 * ch + (j >> 3)] = t;
  }
}

// Epilogue of the implicit-GEMM kernels: NV 16-byte vectors per thread of the C tile staged in
// LDS (rows = pixels from px0, VPR vectors per row) -> residual addend (masked by its ReLU bits)
// -> 16-byte store -> backward BN statistics.  Every global operand of the NV vectors (the BN's
// x and mask bits, the addend and its bits) is requested at a clamped address before the first
// is used: behind the per-lane range check, hipcc branched around each load and waited for it
// vector by vector (8 dependent round trips per tile in the LDS-DMA kernel's data gradient).
template <int NT, int NV, int VPR, typename PF>
__device__ __forceinline__ void epi_vectors(const ConvNArgs& a, const bf16* Cs, int CP, int px0, int ch0, int Mlim,
                                            PF pfull, bool bst, const float* mean8, const float* sc8,
                                            const float* sh8, float* s1, float* s2) {
  const int tid = threadIdx.x;
  size_t o[NV];
  bool ok[NV];
  uint4 xr[NV];
  u32x4 ad[NV];
  uint32_t mb[NV], am[NV];
  size_t oa[NV];  // addend offsets (asub: half resolution)
  bool aok[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int v = tid + NT * k, row = v / VPR, cv = v - row * VPR;
    const int px = px0 + row, ch = ch0 + 8 * cv;
    ok[k] = px < Mlim && ch < a.Ng;
    const int pf = ok[k] ? pfull(px) : 0;
    o[k] = ok[k] ? (size_t)pf * a.Ng + ch : 0;
    oa[k] = o[k];
    aok[k] = true;
    if (a.asub) {  // full-resolution pixel (n, h, w) -> (n, h / 2, w / 2) when h and w are even
      const int n = (int)a.fOHW.div((uint32_t)pf), rem = pf - n * a.OH * a.OW;
      const int h = (int)a.fOW.div((uint32_t)rem), w = rem - h * a.OW;
      aok[k] = ok[k] && !((h | w) & 1);
      oa[k] = aok[k] ? ((size_t)(n * (a.OH >> 1) + (h >> 1)) * (a.OW >> 1) + (w >> 1)) * a.Ng + ch : 0;
    }
    xr[k] = make_uint4(0u, 0u, 0u, 0u);
    ad[k] = u32x4{0u, 0u, 0u, 0u};
    mb[k] = 0u;
    am[k] = 0xffu;
  }
  if (bst) {
#pragma unroll
    for (int k = 0; k < NV; ++k) xr[k] = *reinterpret_cast<const uint4*>(a.bx + o[k]);
    if (a.bmask) {
#pragma unroll
      for (int k = 0; k < NV; ++k) mb[k] = a.bmask[o[k] >> 3];
    }
  }
  if (a.addend) {
#pragma unroll
    for (int k = 0; k < NV; ++k) ad[k] = *reinterpret_cast<const u32x4*>(a.addend + oa[k]);
    if (a.amask) {
#pragma unroll
      for (int k = 0; k < NV; ++k) am[k] = a.amask[o[k] >> 3];
    }
  }
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    if (!ok[k]) continue;
    const int v = tid + NT * k, row = v / VPR, cv = v - row * VPR;
    u32x4 val = *reinterpret_cast<const u32x4*>(Cs + row * CP + 8 * cv);
    if (a.addend && aok[k]) val = add8(val, a.amask ? mask8(ad[k], am[k]) : ad[k]);
    if (a.owt & 1) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(a.out + o[k]), "v"(val) : "memory");
    else *reinterpret_cast<u32x4*>(a.out + o[k]) = val;
    if (bst) bn_bwd_acc8(a, val, xr[k], mb[k], mean8, sc8, sh8, s1, s2);
  }
}

// __launch_bounds__(256, 2): at least two waves per SIMD (<= 256 VGPRs); the LDS tiles allow two
// 256-thread blocks per CU anyway, so a larger register budget would only lose occupancy
template <int TM, int TN, bool kWide>
__global__ __launch_bounds__(256, 2) void conv_nhwc_kernel(ConvNArgs a) {
  // kWide (Ca % 64 == 0, every ResNet layer but the 8-channel stem): the 64 k of a stage lie in
  // ONE filter tap (r, s), so the tap decomposition is a per-stage scalar and each 16-byte
  // operand load is a per-lane base plus a uniform offset (a few VALU per load instead of two
  // divisions and a 64-bit address per load).
  // BK = 64 (two MFMA k-steps per stage) keeps each stage's MFMA phase long enough to cover the
  // next stage's global loads.  LDS rows of 80 bf16 = 160 B = 10 x 16 B: a ds_read_b128 lane group
  // ({0-3,12-15,20-27}, ... : 8 rows at one 16-B column and 8 rows at the next) then hits 16
  // distinct 16-byte bank slots (conflict-free, found by enumerating pitches against the
  // gfx950 lane groups); the 144-B pitch it replaces was conflict-free only for plain 16-row
  // groups and measured more bank-conflict cycles than LDS-active cycles.
  constexpr int BK = 64, LD = BK + 16;
  constexpr int EA = TM * 8 / 256, EB = TN * 8 / 256;  // 16-byte vectors per thread per stage
  constexpr int WMT = TM / 32, WNT = TN / 32;           // 16x16 MFMA tiles per wave (wave tile = TM/2 x TN/2)
  __shared__ __attribute__((aligned(16))) bf16 As[2][TM * LD];
  __shared__ __attribute__((aligned(16))) bf16 Bs[2][TN * LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave >> 1, wn = wave & 1;
  const int tiles_m = (a.Ng + TM - 1) / TM;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int ch0 = (bid % tiles_m) * TM, px0 = (bid / tiles_m) * TN;
  const int kv = tid & 7, row0 = tid >> 3;  // vector kv of rows row0 + 32 i

  // parity class (par mode): its pixel count, tap origin (r0, s0), taps per row and GEMM depth
  const int pca = a.par ? (int)blockIdx.z >> 1 : 0, pcb = a.par ? (int)blockIdx.z & 1 : 0;
  const int r0 = a.par ? (pca + a.ph) & 1 : 0, s0 = a.par ? (pcb + a.pw) & 1 : 0;
  const int nS = a.par ? (a.S - s0 + 1) >> 1 : a.S;
  const int Kgc = a.par ? ((a.R - r0 + 1) >> 1) * nS * a.Ca : a.Kg;
  const int Mc = a.par ? a.M >> 2 : a.M;
  // output pixel of GEMM column m (the full dx index in par mode)
  auto pfull = [&](int m) -> int {
    if (!a.par) return m;
    const int n = (int)a.fHWc.div((uint32_t)m), rem = m - n * a.Hc * a.Wc;
    const int i = (int)a.fWc.div((uint32_t)rem), j = rem - i * a.Wc;
    return (n * a.OH + 2 * i + pca) * a.OW + 2 * j + pcb;
  };

  int pn[EB], poh[EB], pow_[EB];
  bool pok[EB];
#pragma unroll
  for (int i = 0; i < EB; ++i) {
    const int m = px0 + row0 + 32 * i;
    pok[i] = m < Mc;
    const int mm = pok[i] ? m : 0;
    if (a.par) {
      pn[i] = (int)a.fHWc.div((uint32_t)mm);
      const int rem = mm - pn[i] * a.Hc * a.Wc;
      const int ii = (int)a.fWc.div((uint32_t)rem);
      poh[i] = 2 * ii + pca;
      pow_[i] = 2 * (rem - ii * a.Wc) + pcb;
    } else {
      pn[i] = (int)a.fOHW.div((uint32_t)mm);
      const int rem = mm - pn[i] * a.OH * a.OW;
      poh[i] = (int)a.fOW.div((uint32_t)rem);
      pow_[i] = rem - poh[i] * a.OW;
    }
  }
  // two register stages: the loads of k-tile t + 2 are issued while tile t is computed, so each
  // has a whole compute phase plus a barrier to land (one stage hid L2 latency only)
  u32x4 ra0[EA], rb0[EB], ra1[EA], rb1[EB];  // (set 1 unused by the one-stage 128 x 128 tile)
  bool ma0[EA], mb0[EB], ma1[EA], mb1[EB];     // their validity: applied when staged into LDS
  const u32x4 z4 = {0u, 0u, 0u, 0u};
  // wide path: per-lane byte bases (loop invariant)
  uint32_t abase[EA], pbase[EB];
  int ihb[EB], iwb[EB];
  bool aok[EA];
#pragma unroll
  for (int i = 0; i < EA; ++i) aok[i] = ch0 + row0 + 32 * i < a.Ng;
  // every operand load below is issued unconditionally from a valid (clamped) address and its
  // validity kept beside it; the mask is applied when the stage is written to LDS.  (A per-lane
  // `ok ? load : 0` makes hipcc branch around each load, which it then cannot count, and a mask
  // applied right after the load is scheduled there: either way the loads of the second register
  // stage were waited for before the current stage's MFMAs.)
  if constexpr (kWide) {
#pragma unroll
    for (int i = 0; i < EA; ++i) abase[i] = 2u * ((uint32_t)(aok[i] ? ch0 + row0 + 32 * i : 0) * a.Kg + 8 * kv);
#pragma unroll
    for (int i = 0; i < EB; ++i) {
      pbase[i] = 2u * ((uint32_t)pn[i] * a.IH * a.IW * a.Ca + 8 * kv);
      ihb[i] = a.dgrad ? poh[i] + a.ph : poh[i] * a.sh - a.ph;
      iwb[i] = a.dgrad ? pow_[i] + a.pw : pow_[i] * a.sw - a.pw;
    }
  }
  auto gload = [&](int k0, u32x4 (&ra)[EA], u32x4 (&rb)[EB], bool (&ma)[EA], bool (&mb)[EB]) {
    if constexpr (kWide) {
      const int rs = (int)a.fCa.div((uint32_t)k0), c0 = k0 - rs * a.Ca;  // uniform
      int r, s, kw = k0;
      if (a.par) {  // class tap rs -> (r0 + 2 ri, s0 + 2 si); weight column of that tap
        const int ri = rs / nS, si = rs - ri * nS;
        r = r0 + 2 * ri;
        s = s0 + 2 * si;
        kw = (r * a.S + s) * a.Ca + c0;
      } else {
        r = (int)a.fS.div((uint32_t)rs);
        s = rs - r * a.S;
      }
      const char* wb = reinterpret_cast<const char*>(a.wt) + 2u * (uint32_t)kw;
#pragma unroll
      for (int i = 0; i < EA; ++i) {
        ra[i] = *reinterpret_cast<const u32x4*>(wb + abase[i]);
        ma[i] = aok[i];
      }
      const char* xb = reinterpret_cast<const char*>(a.act) + 2u * (uint32_t)c0;
#pragma unroll
      for (int i = 0; i < EB; ++i) {
        int ih, iw;
        bool ok = pok[i];
        if (!a.dgrad) {
          ih = ihb[i] + r;
          iw = iwb[i] + s;
        } else {
          const int th = ihb[i] - r, tw = iwb[i] - s;
          ih = a.sh == 1 ? th : th >> 1;
          iw = a.sw == 1 ? tw : tw >> 1;
          ok = ok && th >= 0 && tw >= 0 && ih * a.sh == th && iw * a.sw == tw;
        }
        ok = ok && (unsigned)ih < (unsigned)a.IH && (unsigned)iw < (unsigned)a.IW;
        const uint32_t off = ok ? pbase[i] + 2u * (uint32_t)((ih * a.IW + iw) * a.Ca) : 0u;
        rb[i] = *reinterpret_cast<const u32x4*>(xb + off);
        mb[i] = ok;
      }
      return;
    }
    const int k = k0 + 8 * kv;
    const bool kok = k < a.Kg;
    const int kk = kok ? k : 0;
    const int rs = (int)a.fCa.div((uint32_t)kk), c = kk - rs * a.Ca;
    const int r = (int)a.fS.div((uint32_t)rs), s = rs - r * a.S;
#pragma unroll
    for (int i = 0; i < EA; ++i) {
      const int row = aok[i] ? ch0 + row0 + 32 * i : 0;
      ra[i] = *reinterpret_cast<const u32x4*>(a.wt + (size_t)row * a.Kg + kk);
      ma[i] = kok && aok[i];
    }
#pragma unroll
    for (int i = 0; i < EB; ++i) {
      int ih, iw;
      bool ok = pok[i] && kok;
      if (!a.dgrad) {
        ih = poh[i] * a.sh - a.ph + r;
        iw = pow_[i] * a.sw - a.pw + s;
      } else {  // transposed conv: output pixel (h, w) gathers dy[(h + ph - r) / sh] when divisible
        const int th = poh[i] + a.ph - r, tw = pow_[i] + a.pw - s;
        ih = a.sh == 1 ? th : th >> 1;
        iw = a.sw == 1 ? tw : tw >> 1;
        ok = ok && th >= 0 && tw >= 0 && ih * a.sh == th && iw * a.sw == tw;
      }
      ok = ok && (unsigned)ih < (unsigned)a.IH && (unsigned)iw < (unsigned)a.IW;
      const size_t off = ok ? (((size_t)pn[i] * a.IH + ih) * a.IW + iw) * a.Ca + c : 0;
      rb[i] = *reinterpret_cast<const u32x4*>(a.act + off);
      mb[i] = ok;
    }
  };
  auto sstore = [&](int buf, const u32x4 (&ra)[EA], const u32x4 (&rb)[EB], const bool (&ma)[EA],
                    const bool (&mb)[EB]) {
#pragma unroll
    for (int i = 0; i < EA; ++i)
      *reinterpret_cast<u32x4*>(&As[buf][(row0 + 32 * i) * LD + 8 * kv]) = ma[i] ? ra[i] : z4;
#pragma unroll
    for (int i = 0; i < EB; ++i)
      *reinterpret_cast<u32x4*>(&Bs[buf][(row0 + 32 * i) * LD + 8 * kv]) = mb[i] ? rb[i] : z4;
  };

  f32x4 acc[WMT][WNT];
#pragma unroll
  for (int i = 0; i < WMT; ++i)
#pragma unroll
    for (int j = 0; j < WNT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int kt0 = blockIdx.y * a.kt_per_split;
  // nt <= 0: a split (or a parity class without taps) with nothing to reduce writes zeros
  const int nt = min((Kgc + BK - 1) / BK - kt0, a.kt_per_split);
  const int a_row = wm * (TM / 2) + (lane & 15), b_row = wn * (TN / 2) + (lane & 15), koff = 8 * (lane >> 4);
  auto compute = [&](int cur) {
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 av[WMT], bv[WNT];
#pragma unroll
      for (int i = 0; i < WMT; ++i)
        av[i] = *reinterpret_cast<const bf16x8*>(&As[cur][(a_row + 16 * i) * LD + 32 * ks + koff]);
#pragma unroll
      for (int j = 0; j < WNT; ++j)
        bv[j] = *reinterpret_cast<const bf16x8*>(&Bs[cur][(b_row + 16 * j) * LD + 32 * ks + koff]);
#pragma unroll
      for (int i = 0; i < WMT; ++i)
#pragma unroll
        for (int j = 0; j < WNT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
  };
  if constexpr (TM * TN <= 64 * 128) {
    if (nt > 0) {
      gload(kt0 * BK, ra0, rb0, ma0, mb0);
      if (nt > 1) gload((kt0 + 1) * BK, ra1, rb1, ma1, mb1);
      sstore(0, ra0, rb0, ma0, mb0);
    }
    __syncthreads();
    // unrolled by two so each register stage is a compile-time array (runtime-indexed register
    // arrays would go to scratch): even steps compute buffer 0 and hold stage set 1, odd steps
    // the reverse
    for (int t = 0; t < nt; t += 2) {
      if (t + 2 < nt) gload((kt0 + t + 2) * BK, ra0, rb0, ma0, mb0);
      compute(0);
      if (t + 1 < nt) sstore(1, ra1, rb1, ma1, mb1);
      __syncthreads();
      if (t + 1 >= nt) break;
      if (t + 3 < nt) gload((kt0 + t + 3) * BK, ra1, rb1, ma1, mb1);
      compute(1);
      if (t + 2 < nt) sstore(0, ra0, rb0, ma0, mb0);
      __syncthreads();
    }
  } else {
    // 128 x 128: one register stage (two would exceed 256 VGPRs and spill)
    if (nt > 0) {
      gload(kt0 * BK, ra0, rb0, ma0, mb0);
      sstore(0, ra0, rb0, ma0, mb0);
    }
    __syncthreads();
    for (int t = 0; t < nt; ++t) {
      const int cur = t & 1;
      if (t + 1 < nt) gload((kt0 + t + 1) * BK, ra0, rb0, ma0, mb0);
      compute(cur);
      if (t + 1 < nt) sstore(cur ^ 1, ra0, rb0, ma0, mb0);
      __syncthreads();
    }
  }

  // C/D: row (output channel) = 4 * (lane >> 4) + r, column (pixel) = lane & 15
  if (a.part) {  // split-K: fp32 partials, summed by conv_nhwc_splitk_reduce_k
#pragma unroll
    for (int i = 0; i < WMT; ++i) {
      const int ch = ch0 + wm * (TM / 2) + 16 * i + 4 * (lane >> 4);
      if (ch >= a.Ng) continue;
#pragma unroll
      for (int j = 0; j < WNT; ++j) {
        const int px = px0 + wn * (TN / 2) + 16 * j + (lane & 15);
        if (px >= Mc) continue;
        float* pp = a.part + ((size_t)blockIdx.y * a.M + pfull(px)) * a.Ng + ch;
        if (a.owt & 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(pp), "v"(acc[i][j]) : "memory");
        else *reinterpret_cast<float4*>(pp) = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      }
    }
    return;
  }
  // bf16 output staged through LDS ([TN pixels][TM channels]) so the global stores are full
  // 16-byte vectors along each pixel's channel row (an 8-byte store per lane straight from the
  // MFMA layout touches 16 rows per 16 lanes)
  constexpr int CP = TM + 8;  // pitch (bf16): 16-byte aligned rows, rotating banks
  static_assert(TN * CP <= 2 * TM * LD, "C tile must fit in the A operand buffers");
  bf16* Cs = &As[0][0];  // the k loop ended on a barrier: the operand buffers are free
#pragma unroll
  for (int i = 0; i < WMT; ++i) {
    const int cl = wm * (TM / 2) + 16 * i + 4 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < WNT; ++j) {
      const int pl = wn * (TN / 2) + 16 * j + (lane & 15);
      *reinterpret_cast<uint2*>(Cs + pl * CP + cl) =
          make_uint2(pack2(acc[i][j][0], acc[i][j][1]), pack2(acc[i][j][2], acc[i][j][3]));
    }
  }
  __syncthreads();
  constexpr int VPR = TM / 8;  // 16-byte vectors per pixel row
  // backward BN statistics (a.bx): this thread's channel vector is fixed (256 % VPR == 0)
  const bool bst = a.bx != nullptr;
  float s1[8], s2[8], mean8[8], sc8[8], sh8[8];
  if (bst) {
    const int ch = min(ch0 + 8 * (tid % VPR), a.Ng - 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s1[e] = s2[e] = 0.f;
      mean8[e] = a.bmean[ch + e];
      sc8[e] = a.bfcoef ? a.bfcoef[2 * (ch + e)] : 0.f;
      sh8[e] = a.bfcoef ? a.bfcoef[2 * (ch + e) + 1] : 0.f;
    }
  }
  epi_vectors<256, TN * VPR / 256, VPR>(a, Cs, CP, px0, ch0, Mc, pfull, bst, mean8, sc8, sh8, s1, s2);
  if (bst) {
    __syncthreads();  // every read of the C tile is done: its LDS becomes the reduction buffer
    // partial row = (parity class, pixel tile): rows_per_class = ceil(Mc / TN)
    bn_bwd_flush<256, VPR>(a, reinterpret_cast<float*>(&As[0][0]), s1, s2,
                           (int)blockIdx.z * ((Mc + TN - 1) / TN) + px0 / TN, ch0);
  }
}

// ------------------------------------------------------------------------------------------
// Large-layer forward / stride-1 data gradient: TM (64 | 128) output channels x 256 pixels per
// 512-thread block, one block per CU, operands staged global -> LDS by LDS-DMA
// (global_load_lds_dwordx4: no VGPR round trip, no ds_write) into THREE stage buffers, so two
// k-tiles are in flight while the third is computed; the wait before each stage is a counted
// vmcnt (the other stage's loads stay in flight) plus a raw s_barrier (a __syncthreads() would
// drain every LDS-DMA).
//   LDS image per operand: rows of 64 k (128 B), each wave-instruction fills 8 rows x 8 16-byte
//   chunks lane-linearly; the chunk a lane fetches is XOR-swizzled by (row & 7) on the SOURCE
//   address, which makes the ds_read_b128 fragment reads conflict-free for the gfx950 lane
//   groups (enumerated, see conv_nhwc_kernel's pitch note).
//   Padding / out-of-range rows: the lane loads 16 zero bytes from g_zero16 instead.
__device__ uint4 g_zero16;

typedef __attribute__((address_space(3))) void lds_void_t;

// device-only wrapper: the builtin needs a gfx950 target feature, which the host pass of an
// (implicitly host-device) lambda would reject, silently dropping the kernel's host stub
__device__ __forceinline__ void glds16(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds(src, (lds_void_t*)lds, 16, 0, 0);
}

// Epilogue shared by the two-/three-stage LDS-DMA kernels once the bf16 C tile ([TN pixels][TM
// channels], pitch TM + 8) is staged at the start of smem: residual addend, 16-byte stores and the
// backward (kBst: reduction slots fit after the C tile) or forward (STATS) BN statistics.
template <int TM, int TN, bool STATS, bool kBst, int kSmem, typename PF>
__device__ __forceinline__ void glds_tail(const ConvNArgs& a, char* smem, int px0, int ch0, int Mc, PF pfull) {
  const int tid = threadIdx.x;
  constexpr int CP = TM + 8;
  const bf16* Cs = reinterpret_cast<const bf16*>(smem);
  constexpr int VPR = TM / 8;
  const bool bst = kBst && !STATS && a.bx != nullptr;
  float s1[8], s2[8], mean8[8], sc8[8], sh8[8];
  if (bst) {
    const int ch = min(ch0 + 8 * (tid % VPR), a.Ng - 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s1[e] = s2[e] = 0.f;
      mean8[e] = a.bmean[ch + e];
      sc8[e] = a.bfcoef ? a.bfcoef[2 * (ch + e)] : 0.f;
      sh8[e] = a.bfcoef ? a.bfcoef[2 * (ch + e) + 1] : 0.f;
    }
  }
  epi_vectors<512, TN * VPR / 512, VPR>(a, Cs, CP, px0, ch0, Mc, pfull, bst, mean8, sc8, sh8, s1, s2);
  if constexpr (kBst) {
    if (bst) {
      // reduction slots after the C tile in the (idle) stage buffers
      float* bred = reinterpret_cast<float*>(smem + ((TN * CP * 2 + 255) & ~255));
      // partial row = (parity class, pixel tile)
      bn_bwd_flush<512, VPR>(a, bred, s1, s2, (int)blockIdx.z * ((Mc + TN - 1) / TN) + px0 / TN, ch0);
    }
  }
  if constexpr (STATS) {  // BN statistics of the stored (bf16) tile: 512 / TM threads per channel
    constexpr int TPC = 512 / TM, RPT = TN / TPC, U = 8;
    static_assert(RPT % U == 0, "rows per thread");
    // reduction slots after the C tile in the (idle) stage buffers
    float* bred = reinterpret_cast<float*>(smem + ((TN * CP * 2 + 255) & ~255));
    static_assert(((TN * CP * 2 + 255) & ~255) + 2 * 512 * 4 <= kSmem, "BN reduction slots must fit");
    const int c = tid % TM, q = tid / TM, ch = ch0 + c;
    const float K = (a.bnshift && ch < a.Ng) ? a.bnshift[ch] : 0.f;
    const int rows = min(TN, a.M - px0);
    const uint16_t* col = reinterpret_cast<const uint16_t*>(Cs) + c;
    float s1[U], s2[U];
#pragma unroll
    for (int u = 0; u < U; ++u) s1[u] = s2[u] = 0.f;
    if (rows == TN) {  // full tile: U independent rows per iteration (loads in flight together)
      for (int r0 = q * RPT; r0 < (q + 1) * RPT; r0 += U) {
        uint16_t h[U];
#pragma unroll
        for (int u = 0; u < U; ++u) h[u] = col[(r0 + u) * CP];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const float d = bf2f(h[u]) - K;
          s1[u] += d;
          s2[u] = fmaf(d, d, s2[u]);
        }
      }
    } else {
      for (int r = q * RPT; r < min(rows, (q + 1) * RPT); ++r) {
        const float d = bf2f(col[r * CP]) - K;
        s1[0] += d;
        s2[0] = fmaf(d, d, s2[0]);
      }
    }
#pragma unroll
    for (int u = 1; u < U; ++u) {
      s1[0] += s1[u];
      s2[0] += s2[u];
    }
    bred[tid] = s1[0];
    bred[512 + tid] = s2[0];
    __syncthreads();
    if (q == 0 && ch < a.Ng) {
      float t1 = s1[0], t2 = s2[0];
      for (int k = 1; k < TPC; ++k) {
        t1 += bred[tid + k * TM];
        t2 += bred[512 + tid + k * TM];
      }
      float* dst = a.bnpart + (size_t)(px0 / TN) * 2 * a.Ng + 2 * ch;
      dst[0] = t1;
      dst[1] = t2;
    }
  }
}

// STATS: the forward BN-statistics epilogue (bnpart / bnshift); the backward BN-statistics
// epilogue of a data gradient runs whenever a.bx is set (ConvNArgs::bx).
// TN = 128, NS = 2 (the short-reduction variant, 1x1 layers with <= 2 k-tiles): 64 KB of LDS
// (TM = 128), two blocks per CU, so one block's loads and MFMAs run under the other's epilogue;
// with one 144 KB block per CU every tile's load -> MFMA -> store chain was serial (the 56 x 56
// 1x1 layers ran at 2-2.3x their HBM floor).
template <int TM, bool STATS = false, int TN = 256, int NS = 3>
__global__ __launch_bounds__(512, TN == 128 ? 2 : 1) void conv_nhwc_glds_kernel(ConvNArgs a) {
  constexpr int BK = 64;
  static_assert((TN == 256 && NS == 3) || (TN == 128 && NS == 2), "glds kernel variants");
  constexpr int AB = TM * 128, SB = AB + TN * 128;        // bytes: A image, whole stage
  constexpr int NA = TM / 64, NB = TN / 64, NPW = NA + NB;  // LDS-DMA instructions per wave per stage
  constexpr int WM = TM / 64, WN = 8 / WM, WPX = TN / WN, WMT = 4, WNT = WPX / 16;
  // after the k loop the stage buffers hold the bf16 C tile ([TN][TM + 8]) and, for the backward
  // BN statistics, 16 reduction floats per thread; the two-stage variant's 64 KB of stages are
  // topped up to fit them (67.6 KB at TM = 128: still two blocks per CU)
  constexpr int kCB = ((TN * (TM + 8) * 2 + 255) & ~255), kBstB = kCB + 16 * 512 * 4;
  constexpr int kSmem = (TN == 128 && kBstB > NS * SB) ? kBstB : NS * SB;
  __shared__ __attribute__((aligned(1024))) char smem[kSmem];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave / WN, wn = wave % WN;
  const int tiles_m = (a.Ng + TM - 1) / TM;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int ch0 = (bid % tiles_m) * TM, px0 = (bid / tiles_m) * TN;
  const char* zero = reinterpret_cast<const char*>(&g_zero16);

  // per-lane A rows (NA) and B rows (NB): slot = (wave * N + j) * 64 + lane -> row = slot >> 3
  const int pch = lane & 7;  // physical chunk this lane fills
  int arow[NA];
  uint32_t abase[NA];
  bool aok[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    arow[j] = ((wave * NA + j) * 64 + lane) >> 3;
    aok[j] = ch0 + arow[j] < a.Ng;
    abase[j] = 2u * ((uint32_t)(ch0 + (aok[j] ? arow[j] : 0)) * a.Kg + 8 * (pch ^ (arow[j] & 7)));
  }
  // par (stride-2 data gradient, as in conv_nhwc_kernel): blockIdx.z = output parity class
  // (h & 1, w & 1), its pixels (n, 2 i + pca, 2 j + pcb), only the taps of matching parity
  const int pca = a.par ? (int)blockIdx.z >> 1 : 0, pcb = a.par ? (int)blockIdx.z & 1 : 0;
  const int r0 = a.par ? (pca + a.ph) & 1 : 0, s0 = a.par ? (pcb + a.pw) & 1 : 0;
  const int nS = a.par ? (a.S - s0 + 1) >> 1 : a.S;
  const int Kgc = a.par ? ((a.R - r0 + 1) >> 1) * nS * a.Ca : a.Kg;
  const int Mc = a.par ? a.M >> 2 : a.M;
  auto pfull = [&](int m) -> int {  // output pixel of GEMM row m (the full dx index in par mode)
    if (!a.par) return m;
    const int n = (int)a.fHWc.div((uint32_t)m), rem = m - n * a.Hc * a.Wc;
    const int i = (int)a.fWc.div((uint32_t)rem), j = rem - i * a.Wc;
    return (n * a.OH + 2 * i + pca) * a.OW + 2 * j + pcb;
  };
  uint32_t pbase[NB];
  int ihb[NB], iwb[NB], lchb[NB];
  bool pok[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int row = ((wave * NB + j) * 64 + lane) >> 3;
    const int m = px0 + row;
    pok[j] = m < Mc;
    const int mm = pok[j] ? m : 0;
    int n, oh, ow;
    if (a.par) {
      n = (int)a.fHWc.div((uint32_t)mm);
      const int rem = mm - n * a.Hc * a.Wc, i = (int)a.fWc.div((uint32_t)rem);
      oh = 2 * i + pca;
      ow = 2 * (rem - i * a.Wc) + pcb;
    } else {
      n = (int)a.fOHW.div((uint32_t)mm);
      const int rem = mm - n * a.OH * a.OW;
      oh = (int)a.fOW.div((uint32_t)rem);
      ow = rem - oh * a.OW;
    }
    pbase[j] = 2u * ((uint32_t)n * a.IH * a.IW * a.Ca);
    ihb[j] = a.dgrad ? oh + a.ph : oh * a.sh - a.ph;
    iwb[j] = a.dgrad ? ow + a.pw : ow * a.sw - a.pw;
    lchb[j] = 8 * (pch ^ (row & 7));
  }

  const int kt0 = blockIdx.y * a.kt_per_split;
  auto issue = [&](int t, int buf) {
    const int k0 = (kt0 + t) * BK;
    const int rs = (int)a.fCa.div((uint32_t)k0), c0 = k0 - rs * a.Ca;  // uniform: one tap per stage
    int r, s, kw = k0;
    if (a.par) {  // class tap rs -> (r0 + 2 ri, s0 + 2 si); weight column of that tap
      const int ri = rs / nS, si = rs - ri * nS;
      r = r0 + 2 * ri;
      s = s0 + 2 * si;
      kw = (r * a.S + s) * a.Ca + c0;
    } else {
      r = (int)a.fS.div((uint32_t)rs);
      s = rs - r * a.S;
    }
    char* st = smem + buf * SB;
    const char* wb = reinterpret_cast<const char*>(a.wt) + 2u * (uint32_t)kw;
#pragma unroll
    for (int j = 0; j < NA; ++j)
      glds16(aok[j] ? (const void*)(wb + abase[j]) : (const void*)zero, st + (wave * NA + j) * 1024);
    const char* xb = reinterpret_cast<const char*>(a.act) + 2u * (uint32_t)c0;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      int ih, iw;
      bool ok = pok[j];
      if (!a.dgrad) {
        ih = ihb[j] + r;
        iw = iwb[j] + s;
      } else {  // transposed: dy[(h + ph - r) / sh] where divisible (always, for a parity class's taps)
        const int th = ihb[j] - r, tw = iwb[j] - s;
        ih = a.sh == 1 ? th : th >> 1;
        iw = a.sw == 1 ? tw : tw >> 1;
        ok = ok && th >= 0 && tw >= 0 && ih * a.sh == th && iw * a.sw == tw;
      }
      ok = ok && (unsigned)ih < (unsigned)a.IH && (unsigned)iw < (unsigned)a.IW;
      const char* src = xb + pbase[j] + 2u * (uint32_t)((ih * a.IW + iw) * a.Ca + lchb[j]);
      glds16(ok ? (const void*)src : (const void*)zero, st + AB + (wave * NB + j) * 1024);
    }
  };

  f32x4 acc[WMT][WNT];
#pragma unroll
  for (int i = 0; i < WMT; ++i)
#pragma unroll
    for (int j = 0; j < WNT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // split-K over blockIdx.y (fp32 partials, summed by conv_nhwc_splitk_reduce_k); par: the class's taps
  const int nt = min(Kgc / BK - kt0, a.kt_per_split);
  // NS - 1 stages in flight ahead of the one computed
  if (nt > 0) issue(0, 0);
  if (NS == 3 && nt > 1) issue(1, 1);
  for (int t = 0; t < nt; ++t) {
    if (NS == 3 && t + 1 < nt) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // stage t landed for every wave; stage t-1's buffer is free
    if (t + NS - 1 < nt) issue(t + NS - 1, (t + NS - 1) % NS);
    const char* sA = smem + (t % NS) * SB;
    const char* sB = sA + AB;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      const int lch = 4 * ks + (lane >> 4);
      bf16x8 av[WMT], bv[WNT];
#pragma unroll
      for (int i = 0; i < WMT; ++i) {
        const int row = wm * 64 + 16 * i + (lane & 15);
        av[i] = *reinterpret_cast<const bf16x8*>(sA + row * 128 + 16 * (lch ^ (row & 7)));
      }
#pragma unroll
      for (int j = 0; j < WNT; ++j) {
        const int row = wn * WPX + 16 * j + (lane & 15);
        bv[j] = *reinterpret_cast<const bf16x8*>(sB + row * 128 + 16 * (lch ^ (row & 7)));
      }
#pragma unroll
      for (int i = 0; i < WMT; ++i)
#pragma unroll
        for (int j = 0; j < WNT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
  }
  if (a.part) {  // split-K: fp32 partials of 4 consecutive channels per lane
#pragma unroll
    for (int i = 0; i < WMT; ++i) {
      const int ch = ch0 + wm * 64 + 16 * i + 4 * (lane >> 4);
      if (ch >= a.Ng) continue;
#pragma unroll
      for (int j = 0; j < WNT; ++j) {
        const int px = px0 + wn * WPX + 16 * j + (lane & 15);
        if (px >= a.M) continue;
        float* pp = a.part + ((size_t)blockIdx.y * a.M + px) * a.Ng + ch;
        if (a.owt & 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(pp), "v"(acc[i][j]) : "memory");
        else *reinterpret_cast<float4*>(pp) = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      }
    }
    return;
  }
  __syncthreads();  // every wave done with the stage buffers (no LDS-DMA outstanding)
  // bf16 output staged through LDS ([TN pixels][TM channels], pitch TM + 8) -> 16-byte stores
  constexpr int CP = TM + 8;
  static_assert(TN * CP * 2 <= kSmem, "C tile must fit in the stage buffers");
  bf16* Cs = reinterpret_cast<bf16*>(smem);
#pragma unroll
  for (int i = 0; i < WMT; ++i) {
    const int cl = wm * 64 + 16 * i + 4 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < WNT; ++j) {
      const int pl = wn * WPX + 16 * j + (lane & 15);
      *reinterpret_cast<uint2*>(Cs + pl * CP + cl) =
          make_uint2(pack2(acc[i][j][0], acc[i][j][1]), pack2(acc[i][j][2], acc[i][j][3]));
    }
  }
  __syncthreads();
  glds_tail<TM, TN, STATS, kBstB <= kSmem, kSmem>(a, smem, px0, ch0, Mc, pfull);
}

// ------------------------------------------------------------------------------------------
// Two-stage 128 x 128 LDS-DMA tile with 64 x 64 wave tiles (gk2).  The 8 waves form two k-groups of
// four (kg = wave >> 2): each stage's 64-k tile is split into its two 32-k halves and group kg
// computes half kg over the whole 128 x 128 tile (4 waves x 64 x 64).  Per MFMA that is half an
// LDS operand read (ds_read_b128) against three quarters for the 8-wave 64 x 32 wave tiles of
// conv_nhwc_glds_kernel<128, *, 128, 2> -- the same MFMAs, stages and 16 waves per CU; the
// groups' fp32 tiles are summed through LDS after the k loop.  MF32: v_mfma_f32_32x32x16_bf16
// (2 x 2 tiles of 32 x 32 per wave) instead of v_mfma_f32_16x16x32_bf16 (4 x 4 of 16 x 16).
// LDS image: rows of 64 k (128 B); the 16-byte chunk a lane fills is XOR-swizzled by (row >> 1) & 7
// on the SOURCE address, which makes both MFMA shapes' ds_read_b128 fragment reads conflict-free
// (16-lane groups {0-3,12-15,20-27}, ...: rows r and r + 8 differ in bit 0 of r >> 3 only through
// the 128-B half of the 256-B bank row; scripts/ldsbank/bank.py enumerates it).
__device__ __forceinline__ int gk2_swz(int row) { return (row >> 1) & 7; }

template <bool STATS, bool MF32>
__global__ __launch_bounds__(512, 2) void conv_nhwc_gk2_kernel(ConvNArgs a) {
  constexpr int TM = 128, TN = 128, BK = 64, NS = 2;
  constexpr int AB = TM * 128, SB = AB + TN * 128;
  constexpr int NA = TM / 64, NB = TN / 64;
  constexpr int kCB = ((TN * (TM + 8) * 2 + 255) & ~255), kBstB = kCB + 16 * 512 * 4;
  constexpr int kRed = 4 * 16 * 64 * 16;  // k-group 1's fp32 tile: 4 waves x 16 float4 x 64 lanes
  constexpr int kSmem0 = NS * SB > kBstB ? NS * SB : kBstB;
  constexpr int kSmem = kSmem0 > kRed ? kSmem0 : kRed;
  __shared__ __attribute__((aligned(1024))) char smem[kSmem];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kg = wave >> 2, wq = wave & 3, wm = wq >> 1, wn = wq & 1;
  const int tiles_m = (a.Ng + TM - 1) / TM;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int ch0 = (bid % tiles_m) * TM, px0 = (bid / tiles_m) * TN;
  const char* zero = reinterpret_cast<const char*>(&g_zero16);

  const int pch = lane & 7;  // physical chunk this lane fills
  uint32_t abase[NA];
  bool aok[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int arow = ((wave * NA + j) * 64 + lane) >> 3;
    aok[j] = ch0 + arow < a.Ng;
    abase[j] = 2u * ((uint32_t)(ch0 + (aok[j] ? arow : 0)) * a.Kg + 8 * (pch ^ gk2_swz(arow)));
  }
  const int pca = a.par ? (int)blockIdx.z >> 1 : 0, pcb = a.par ? (int)blockIdx.z & 1 : 0;
  const int r0 = a.par ? (pca + a.ph) & 1 : 0, s0 = a.par ? (pcb + a.pw) & 1 : 0;
  const int nS = a.par ? (a.S - s0 + 1) >> 1 : a.S;
  const int Kgc = a.par ? ((a.R - r0 + 1) >> 1) * nS * a.Ca : a.Kg;
  const int Mc = a.par ? a.M >> 2 : a.M;
  auto pfull = [&](int m) -> int {
    if (!a.par) return m;
    const int n = (int)a.fHWc.div((uint32_t)m), rem = m - n * a.Hc * a.Wc;
    const int i = (int)a.fWc.div((uint32_t)rem), j = rem - i * a.Wc;
    return (n * a.OH + 2 * i + pca) * a.OW + 2 * j + pcb;
  };
  uint32_t pbase[NB];
  int ihb[NB], iwb[NB], lchb[NB];
  bool pok[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int row = ((wave * NB + j) * 64 + lane) >> 3;
    const int m = px0 + row;
    pok[j] = m < Mc;
    const int mm = pok[j] ? m : 0;
    int n, oh, ow;
    if (a.par) {
      n = (int)a.fHWc.div((uint32_t)mm);
      const int rem = mm - n * a.Hc * a.Wc, i = (int)a.fWc.div((uint32_t)rem);
      oh = 2 * i + pca;
      ow = 2 * (rem - i * a.Wc) + pcb;
    } else {
      n = (int)a.fOHW.div((uint32_t)mm);
      const int rem = mm - n * a.OH * a.OW;
      oh = (int)a.fOW.div((uint32_t)rem);
      ow = rem - oh * a.OW;
    }
    pbase[j] = 2u * ((uint32_t)n * a.IH * a.IW * a.Ca);
    ihb[j] = a.dgrad ? oh + a.ph : oh * a.sh - a.ph;
    iwb[j] = a.dgrad ? ow + a.pw : ow * a.sw - a.pw;
    lchb[j] = 8 * (pch ^ gk2_swz(row));
  }

  auto issue = [&](int t, int buf) {
    const int k0 = t * BK;
    const int rs = (int)a.fCa.div((uint32_t)k0), c0 = k0 - rs * a.Ca;  // uniform: one tap per stage
    int r, s, kw = k0;
    if (a.par) {
      const int ri = rs / nS, si = rs - ri * nS;
      r = r0 + 2 * ri;
      s = s0 + 2 * si;
      kw = (r * a.S + s) * a.Ca + c0;
    } else {
      r = (int)a.fS.div((uint32_t)rs);
      s = rs - r * a.S;
    }
    char* st = smem + buf * SB;
    const char* wb = reinterpret_cast<const char*>(a.wt) + 2u * (uint32_t)kw;
#pragma unroll
    for (int j = 0; j < NA; ++j)
      glds16(aok[j] ? (const void*)(wb + abase[j]) : (const void*)zero, st + (wave * NA + j) * 1024);
    const char* xb = reinterpret_cast<const char*>(a.act) + 2u * (uint32_t)c0;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      int ih, iw;
      bool ok = pok[j];
      if (!a.dgrad) {
        ih = ihb[j] + r;
        iw = iwb[j] + s;
      } else {
        const int th = ihb[j] - r, tw = iwb[j] - s;
        ih = a.sh == 1 ? th : th >> 1;
        iw = a.sw == 1 ? tw : tw >> 1;
        ok = ok && th >= 0 && tw >= 0 && ih * a.sh == th && iw * a.sw == tw;
      }
      ok = ok && (unsigned)ih < (unsigned)a.IH && (unsigned)iw < (unsigned)a.IW;
      const char* src = xb + pbase[j] + 2u * (uint32_t)((ih * a.IW + iw) * a.Ca + lchb[j]);
      glds16(ok ? (const void*)src : (const void*)zero, st + AB + (wave * NB + j) * 1024);
    }
  };

  // accumulators: 64 floats per lane either way
  constexpr int NI = MF32 ? 2 : 4;
  typedef typename std::conditional<MF32, f32x16, f32x4>::type accv;
  accv acc[NI][NI];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int e = 0; e < (MF32 ? 16 : 4); ++e) acc[i][j][e] = 0.f;

  const int nt = Kgc / BK;
  if (nt > 0) issue(0, 0);
  for (int t = 0; t < nt; ++t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // stage t landed for every wave; stage t-1's buffer is free
    if (t + 1 < nt) issue(t + 1, (t + 1) % NS);
    const char* sA = smem + (t % NS) * SB;
    const char* sB = sA + AB;
    if constexpr (!MF32) {
      const int lch = 4 * kg + (lane >> 4);
      bf16x8 av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wm * 64 + 16 * i + (lane & 15);
        av[i] = *reinterpret_cast<const bf16x8*>(sA + row * 128 + 16 * (lch ^ gk2_swz(row)));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = wn * 64 + 16 * j + (lane & 15);
        bv[j] = *reinterpret_cast<const bf16x8*>(sB + row * 128 + 16 * (lch ^ gk2_swz(row)));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int lch = 4 * kg + 2 * kk + (lane >> 5);
        bf16x8 av[2], bv[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int row = wm * 64 + 32 * i + (lane & 31);
          av[i] = *reinterpret_cast<const bf16x8*>(sA + row * 128 + 16 * (lch ^ gk2_swz(row)));
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int row = wn * 64 + 32 * j + (lane & 31);
          bv[j] = *reinterpret_cast<const bf16x8*>(sB + row * 128 + 16 * (lch ^ gk2_swz(row)));
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
      }
    }
  }
  __syncthreads();  // every wave done with the stage buffers (no LDS-DMA outstanding)
  // k-group 1 hands its tile to k-group 0 (lane-linear float4s: conflict-free both ways)
  float4* red = reinterpret_cast<float4*>(smem);
  if (kg == 1) {
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
#pragma unroll
        for (int q = 0; q < (MF32 ? 4 : 1); ++q) {
          const int qi = (i * NI + j) * (MF32 ? 4 : 1) + q;
          red[(wq * 16 + qi) * 64 + lane] =
              make_float4(acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]);
        }
  }
  __syncthreads();
  if (kg == 0) {
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
#pragma unroll
        for (int q = 0; q < (MF32 ? 4 : 1); ++q) {
          const int qi = (i * NI + j) * (MF32 ? 4 : 1) + q;
          const float4 v = red[(wq * 16 + qi) * 64 + lane];
          acc[i][j][4 * q] += v.x;
          acc[i][j][4 * q + 1] += v.y;
          acc[i][j][4 * q + 2] += v.z;
          acc[i][j][4 * q + 3] += v.w;
        }
  }
  __syncthreads();  // the reduction slots become the C tile
  constexpr int CP = TM + 8;
  static_assert(TN * CP * 2 <= kSmem, "C tile must fit in the stage buffers");
  bf16* Cs = reinterpret_cast<bf16*>(smem);
  if (kg == 0) {
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        if constexpr (!MF32) {
          const int cl = wm * 64 + 16 * i + 4 * (lane >> 4), pl = wn * 64 + 16 * j + (lane & 15);
          *reinterpret_cast<uint2*>(Cs + pl * CP + cl) =
              make_uint2(pack2(acc[i][j][0], acc[i][j][1]), pack2(acc[i][j][2], acc[i][j][3]));
        } else {
          const int pl = wn * 64 + 32 * j + (lane & 31);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int cl = wm * 64 + 32 * i + 8 * q + 4 * (lane >> 5);
            *reinterpret_cast<uint2*>(Cs + pl * CP + cl) = make_uint2(pack2(acc[i][j][4 * q], acc[i][j][4 * q + 1]),
                                                                      pack2(acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]));
          }
        }
      }
  }
  __syncthreads();
  glds_tail<TM, TN, STATS, kBstB <= kSmem, kSmem>(a, smem, px0, ch0, Mc, pfull);
}

// ------------------------------------------------------------------------------------------
// 256 x 256 tile of the LDS-DMA kernel, for layers with Ng % 256 == 0 and enough pixel tiles to
// fill the chip: 256 output channels x 256 pixels per 512-thread block, wave tile 64 channels x
// 128 pixels (4 x 8 MFMA fragments: 12 ds_read_b128 per 32 MFMAs, against 16 per 32 for the
// 128-channel tile), TWO 64 KB stage buffers: wait for stage t, barrier (every wave is done with
// stage t - 1, so its buffer is free), issue stage t + 1 into it, compute stage t -- one k-tile in
// flight behind the MFMAs, the structure the CDNA4 guide measures as tying a register pipeline
// on a 256 x 256 tile at one block per CU.  Same operand images, swizzle, zero-row handling and
// epilogues as conv_nhwc_glds_kernel; the C tile is staged through LDS in two 128-pixel halves
// (the waves of pixel column wn own half wn), so the BN reduction slots still fit.
template <bool STATS>
__global__ __launch_bounds__(512) void conv_nhwc_glds256_kernel(ConvNArgs a) {
  constexpr int TM = 256, TN = 256, BK = 64, NS = 2;
  constexpr int AB = TM * 128, SB = AB + TN * 128;   // bytes: A image, whole stage (64 KB)
  constexpr int NA = TM / 64, NB = 4;                 // LDS-DMA instructions per wave per stage
  constexpr int WN = 2, WPX = TN / WN, WMT = 4, WNT = WPX / 16;
  constexpr int CP = TM + 8, HT = TN / 2, VPR = TM / 8;
  constexpr int RED = (HT * CP * 2 + 255) & ~255;    // reduction slots after the C half tile
  static_assert(RED + 16 * 512 * 4 <= NS * SB, "BN reduction slots must fit");
  __shared__ __attribute__((aligned(1024))) char smem[NS * SB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave / WN, wn = wave % WN;
  const int tiles_m = a.Ng / TM;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int ch0 = (bid % tiles_m) * TM, px0 = (bid / tiles_m) * TN;
  const char* zero = reinterpret_cast<const char*>(&g_zero16);

  const int pch = lane & 7;  // physical 16-byte chunk this lane fills
  uint32_t abase[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int row = ((wave * NA + j) * 64 + lane) >> 3;  // < 256 = TM, and ch0 + TM <= Ng
    abase[j] = 2u * ((uint32_t)(ch0 + row) * a.Kg + 8 * (pch ^ (row & 7)));
  }
  uint32_t pbase[NB];
  int ihb[NB], iwb[NB], lchb[NB];
  bool pok[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int row = ((wave * NB + j) * 64 + lane) >> 3;
    const int m = px0 + row;
    pok[j] = m < a.M;
    const int mm = pok[j] ? m : 0;
    const int n = (int)a.fOHW.div((uint32_t)mm), rem = mm - n * a.OH * a.OW;
    const int oh = (int)a.fOW.div((uint32_t)rem), ow = rem - oh * a.OW;
    pbase[j] = 2u * ((uint32_t)n * a.IH * a.IW * a.Ca);
    ihb[j] = a.dgrad ? oh + a.ph : oh * a.sh - a.ph;
    iwb[j] = a.dgrad ? ow + a.pw : ow * a.sw - a.pw;
    lchb[j] = 8 * (pch ^ (row & 7));
  }
  auto issue = [&](int t, int buf) {
    const int k0 = t * BK;
    const int rs = (int)a.fCa.div((uint32_t)k0), c0 = k0 - rs * a.Ca;  // uniform: one tap per stage
    const int r = (int)a.fS.div((uint32_t)rs), s = rs - r * a.S;
    char* st = smem + buf * SB;
    const char* wb = reinterpret_cast<const char*>(a.wt) + 2u * (uint32_t)k0;
#pragma unroll
    for (int j = 0; j < NA; ++j) glds16(wb + abase[j], st + (wave * NA + j) * 1024);
    const char* xb = reinterpret_cast<const char*>(a.act) + 2u * (uint32_t)c0;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int ih = a.dgrad ? ihb[j] - r : ihb[j] + r, iw = a.dgrad ? iwb[j] - s : iwb[j] + s;
      const bool ok = pok[j] && (unsigned)ih < (unsigned)a.IH && (unsigned)iw < (unsigned)a.IW;
      const char* src = xb + pbase[j] + 2u * (uint32_t)((ih * a.IW + iw) * a.Ca + lchb[j]);
      glds16(ok ? (const void*)src : (const void*)zero, st + AB + (wave * NB + j) * 1024);
    }
  };

  f32x4 acc[WMT][WNT];
#pragma unroll
  for (int i = 0; i < WMT; ++i)
#pragma unroll
    for (int j = 0; j < WNT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nt = a.Kg / BK;
  issue(0, 0);
  for (int t = 0; t < nt; ++t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // stage t landed for every wave; stage t - 1's buffer is free
    if (t + 1 < nt) issue(t + 1, (t + 1) & 1);
    const char* sA = smem + (t & 1) * SB;
    const char* sB = sA + AB;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      const int lch = 4 * ks + (lane >> 4);
      bf16x8 av[WMT], bv[WNT];
#pragma unroll
      for (int i = 0; i < WMT; ++i) {
        const int row = wm * 64 + 16 * i + (lane & 15);
        av[i] = *reinterpret_cast<const bf16x8*>(sA + row * 128 + 16 * (lch ^ (row & 7)));
      }
#pragma unroll
      for (int j = 0; j < WNT; ++j) {
        const int row = wn * WPX + 16 * j + (lane & 15);
        bv[j] = *reinterpret_cast<const bf16x8*>(sB + row * 128 + 16 * (lch ^ (row & 7)));
      }
#pragma unroll
      for (int i = 0; i < WMT; ++i)
#pragma unroll
        for (int j = 0; j < WNT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();  // every wave done with the stage buffers (no LDS-DMA outstanding)

  bf16* Cs = reinterpret_cast<bf16*>(smem);
  float* bred = reinterpret_cast<float*>(smem + RED);
  const bool bst = !STATS && a.bx != nullptr;  // backward BN statistics (fixed vector per thread)
  float s1[8], s2[8], mean8[8], sc8[8], sh8[8];
  if (bst) {
    const int ch = ch0 + 8 * (tid % VPR);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s1[e] = s2[e] = 0.f;
      mean8[e] = a.bmean[ch + e];
      sc8[e] = a.bfcoef ? a.bfcoef[2 * (ch + e)] : 0.f;
      sh8[e] = a.bfcoef ? a.bfcoef[2 * (ch + e) + 1] : 0.f;
    }
  }
  // forward BN statistics: channel c = tid % TM, rows q * 64 .. + 63 of each half
  const int sc_c = tid % TM, sc_q = tid / TM;
  const float shiftK = (STATS && a.bnshift) ? a.bnshift[ch0 + sc_c] : 0.f;
  float f1 = 0.f, f2 = 0.f;
  const int rows = min(TN, a.M - px0);
#pragma unroll 1
  for (int h = 0; h < 2; ++h) {
    if (wn == h) {  // this wave's accumulators are pixels h * 128 .. + 127
#pragma unroll
      for (int i = 0; i < WMT; ++i) {
        const int cl = wm * 64 + 16 * i + 4 * (lane >> 4);
#pragma unroll
        for (int j = 0; j < WNT; ++j) {
          const int pl = 16 * j + (lane & 15);
          *reinterpret_cast<uint2*>(Cs + pl * CP + cl) =
              make_uint2(pack2(acc[i][j][0], acc[i][j][1]), pack2(acc[i][j][2], acc[i][j][3]));
        }
      }
    }
    __syncthreads();
    epi_vectors<512, HT * VPR / 512, VPR>(a, Cs, CP, px0 + h * HT, ch0, a.M, [](int px) { return px; }, bst, mean8,
                                          sc8, sh8, s1, s2);
    if constexpr (STATS) {  // column sums of the stored (bf16) half tile
      const int hr = min(max(rows - h * HT, 0), HT);
      const uint16_t* col = reinterpret_cast<const uint16_t*>(Cs) + sc_c;
      const int r0 = sc_q * (HT / 2), r1 = min(r0 + HT / 2, hr);
      float u1[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, u2[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (r1 - r0 == HT / 2) {  // full: 8 independent rows per iteration
        for (int r = r0; r < r1; r += 8) {
          uint16_t hv[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) hv[u] = col[(r + u) * CP];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const float d = bf2f(hv[u]) - shiftK;
            u1[u] += d;
            u2[u] = fmaf(d, d, u2[u]);
          }
        }
      } else {
        for (int r = r0; r < r1; ++r) {
          const float d = bf2f(col[r * CP]) - shiftK;
          u1[0] += d;
          u2[0] = fmaf(d, d, u2[0]);
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        f1 += u1[u];
        f2 += u2[u];
      }
    }
    __syncthreads();  // the half tile is read: the next half (or the reduction slots) may overwrite it
  }
  if (bst) bn_bwd_flush<512, VPR>(a, bred, s1, s2, px0 / TN, ch0);
  if constexpr (STATS) {
    bred[tid] = f1;
    bred[512 + tid] = f2;
    __syncthreads();
    if (sc_q == 0) {
      float* dst = a.bnpart + (size_t)(px0 / TN) * 2 * a.Ng + 2 * (ch0 + sc_c);
      dst[0] = f1 + bred[tid + TM];
      dst[1] = f2 + bred[512 + tid + TM];
    }
  }
}

// ------------------------------------------------------------------------------------------
// Stem forward: 7x7 / stride 2 / pad 3 over an 8-channel (padded) image, 64 output channels,
// output height and width multiples of 16 (ResNet-50's conv1 at any batch).  The generic gather
// kernel re-fetches every input pixel from L2 for each of the 49 taps that read it (Kg = 392 in
// 8-channel gathers with per-element tap arithmetic: 510 us at batch 256, 8x its byte floor).
// Here a block owns a 16 x 16 output tile and stages its 37 x 38 input patch in LDS ONCE, plus
// the whole filter bank in an MFMA-ready layout; the B fragments are then read straight out of
// the patch with no im2col: with k ordered (r, s, c) and s padded to 8 (s = 7 has zero weights),
// one 32-deep k-step is half a filter row, and lane group g's 8 consecutive k are the 8 channels
// of tap s = 4h + g -- one 16-byte LDS read of patch pixel (2 oh + r, 2 ow + s).  For the 16
// lanes of a group the reads are 32 bytes apart, which the ds_read_b128 lane groups
// ({0-3,12-15,20-27}, ...) map onto 16 distinct 16-byte bank slots.
//   8 waves: wave w computes output rows 2w, 2w + 1 (two 16-pixel column tiles) x 64 channels
//   (4 row tiles), 14 k-steps of 8 MFMAs.  LDS: filters [64][448 bf16], 16-byte chunks XOR-swizzled
//   by (row >> 1) & 7 so the 16 rows of a ds_read_b128 lane group hit 16 distinct bank slots
//   (scripts/ldsbank/bank.py: 4 LDS cycles per read; the former 456-bf16 pitch was 2-way, 8),
//   patch [37][38][16 B]: 78 KB, two blocks per CU.  Epilogue as the LDS-DMA kernel: C tile staged in LDS -> 16-byte stores, optional BN
//   partial sums (one row per tile).
constexpr int kStemWP = 448, kStemPW = 38, kStemPH = 37;
// filter chunk q (16 B) of output channel row ch: slot q ^ ((ch >> 1) & 7) (stays in the row: 56 chunks)
__device__ __forceinline__ int stem_swz(int ch, int q) { return q ^ ((ch >> 1) & 7); }
constexpr int kStemA = 64 * kStemWP * 2, kStemP = kStemPH * kStemPW * 16;

template <bool STATS>
__global__ __launch_bounds__(512, 4) void conv_nhwc_stem_kernel(ConvNArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[kStemA + kStemP];
  char* As = smem;
  char* Ps = smem + kStemA;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, m = lane & 15;
  const int tw_n = a.OW >> 4, th_n = a.OH >> 4;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int n = bid / (th_n * tw_n), trem = bid - n * th_n * tw_n;
  const int oh0 = (trem / tw_n) * 16, ow0 = (trem % tw_n) * 16;
  const int ih0 = 2 * oh0 - 3, iw0 = 2 * ow0 - 3;

  // stage: filters (64 ch x 7 r x 8 s 16-byte vectors, s = 7 zero) and the input patch; every
  // load of the thread is issued before the first store
  constexpr int NAV = 64 * 7 * 8 / 512, NPV = (kStemPH * kStemPW + 511) / 512;
  u32x4 av[NAV], pv[NPV];
  const u32x4 z4 = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int i = 0; i < NAV; ++i) {
    const int v = tid + 512 * i, ch = v / 56, rs8 = v - ch * 56, r = rs8 >> 3, s = rs8 & 7;
    av[i] = s < 7 ? *reinterpret_cast<const u32x4*>(a.wt + ((size_t)ch * 49 + r * 7 + s) * 8) : z4;
  }
  const bf16* xin = a.act + (size_t)n * a.IH * a.IW * 8;
#pragma unroll
  for (int i = 0; i < NPV; ++i) {
    const int v = min(tid + 512 * i, kStemPH * kStemPW - 1), pr = v / kStemPW, pc = v - pr * kStemPW;
    const int ih = ih0 + pr, iw = iw0 + pc;
    const bool ok = (unsigned)ih < (unsigned)a.IH && (unsigned)iw < (unsigned)a.IW && pc < 37;
    pv[i] = *reinterpret_cast<const u32x4*>(xin + (size_t)(ok ? ih * a.IW + iw : 0) * 8);
    if (!ok) pv[i] = z4;
  }
#pragma unroll
  for (int i = 0; i < NAV; ++i) {
    const int v = tid + 512 * i, ch = v / 56, rs8 = v - ch * 56;
    *reinterpret_cast<u32x4*>(As + ch * (kStemWP * 2) + stem_swz(ch, rs8) * 16) = av[i];
  }
#pragma unroll
  for (int i = 0; i < NPV; ++i) {
    const int v = tid + 512 * i;
    if (v < kStemPH * kStemPW) *reinterpret_cast<u32x4*>(Ps + v * 16) = pv[i];
  }
  __syncthreads();

  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const char* arow = As + m * (kStemWP * 2);  // rows m + 16 i share (row >> 1) & 7
  const char* prow = Ps + ((4 * w) * kStemPW + 2 * m + g) * 16;  // output row 2w, tap (0, g)
#pragma unroll 2
  for (int r = 0; r < 7; ++r) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bf16x8 fa[4], fb[2];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        fa[i] = *reinterpret_cast<const bf16x8*>(arow + i * 16 * (kStemWP * 2) + stem_swz(m, 8 * r + 4 * h + g) * 16);
#pragma unroll
      for (int j = 0; j < 2; ++j)  // output row 2w + j reads patch row 2 (2w + j) + r
        fb[j] = *reinterpret_cast<const bf16x8*>(prow + ((2 * j + r) * kStemPW + 4 * h) * 16);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();  // every wave done with the filters and the patch

  // C tile [256 pixels][64 channels] (pitch 72) over the filter region; pixel = 16 row + col
  constexpr int CP = 72;
  bf16* Cs = reinterpret_cast<bf16*>(smem);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      *reinterpret_cast<uint2*>(Cs + ((2 * w + j) * 16 + m) * CP + 16 * i + 4 * g) =
          make_uint2(pack2(acc[i][j][0], acc[i][j][1]), pack2(acc[i][j][2], acc[i][j][3]));
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int v = tid + 512 * k, px = v >> 3, cv = v & 7;
    const size_t o = (((size_t)n * a.OH + oh0 + (px >> 4)) * a.OW + ow0 + (px & 15)) * 64 + 8 * cv;
    *reinterpret_cast<u32x4*>(a.out + o) = *reinterpret_cast<const u32x4*>(Cs + px * CP + 8 * cv);
  }
  if constexpr (STATS) {  // BN partial sums of the stored (bf16) tile: 8 threads per channel
    float* bred = reinterpret_cast<float*>(smem + 256 * CP * 2);
    const int c = tid & 63, q = tid >> 6;
    const float K = a.bnshift ? a.bnshift[c] : 0.f;
    const uint16_t* col = reinterpret_cast<const uint16_t*>(Cs) + c;
    float s1[8], s2[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) s1[u] = s2[u] = 0.f;
#pragma unroll
    for (int r0 = 0; r0 < 32; r0 += 8) {
      uint16_t hv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) hv[u] = col[(32 * q + r0 + u) * CP];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float d = bf2f(hv[u]) - K;
        s1[u] += d;
        s2[u] = fmaf(d, d, s2[u]);
      }
    }
#pragma unroll
    for (int u = 1; u < 8; ++u) {
      s1[0] += s1[u];
      s2[0] += s2[u];
    }
    bred[tid] = s1[0];
    bred[512 + tid] = s2[0];
    __syncthreads();
    if (q == 0) {
      float t1 = s1[0], t2 = s2[0];
      for (int k = 1; k < 8; ++k) {
        t1 += bred[tid + 64 * k];
        t2 += bred[512 + tid + 64 * k];
      }
      float* dst = a.bnpart + (size_t)blockIdx.x * 128 + 2 * c;
      dst[0] = t1;
      dst[1] = t2;
    }
  }
}

// ------------------------------------------------------------------------------------------
// 3x3 / stride 1 / pad 1, 64 -> 64 channels (ResNet-50 layer1's conv2: forward, and its data
// gradient, which is the same correlation over dy with the taps flipped).  The LDS-DMA kernel
// re-fetches each input vector from L2 for every one of the 9 taps through a 128-channel-row
// tile; here PERSISTENT blocks keep the whole filter bank in LDS ([64][576 + 8] bf16, loaded once
// per block) and walk bands of RT full-width output rows (RT x W <= 256 pixels, 56 x 56: 4 rows):
// the (RT + 2) x (W + 2) x 64 input patch of a band is staged in LDS once (the next band's patch
// in flight in registers during this band's MFMAs) and the B fragments are read straight out of
// it -- k = (tap, channel), so a lane's 8 consecutive k are one 16-byte channel chunk of one patch
// pixel.  8 waves: wave w = pixel groups 2w, 2w + 1 (16 band pixels each, row-major) x 64
// channels, 18 k-steps.
// LDS banking (gfx950 ds_read_b128 lane groups {0-3,12-15,20-27}, ...; scripts/ldsbank/bank.py):
// a group holds lanes m = 0-3, 12-15 of k-chunk g and m = 4-11 of chunk g + 1.  The filter row
// pitch 576 + 16 bf16 (296 dwords) puts those 16 rows on 16 distinct 4-bank slots (the former
// 576 + 8, 292 dwords, was 2-way: 8 LDS cycles per A read instead of 4).  Patch chunk c of pixel p
// sits at slot (c + 2 (p >> 1)) & 7: for any run of 16 consecutive pixels the two chunks' lanes
// fall on distinct slots (4.6 cycles per B read averaged over the 56 x 56 band reads incl. row
// wraps, against 6.9 for the former XOR (p >> 1) & 7).
__device__ __forceinline__ int c3_swz(int pix, int c) { return (c + (pix & ~1)) & 7; }
constexpr int kC3WP = 576 + 16, kC3A = 64 * kC3WP * 2, kC3PMax = 360, kC3C = 256 * 72 * 2;

__host__ __device__ inline int c3_band_rows(int H, int W) {  // largest RT | H with RT * W <= 256
  int rt = 0;
  for (int r = 1; r <= 256 / W && r <= H; ++r)
    if (H % r == 0 && (r + 2) * (W + 2) <= kC3PMax) rt = r;
  return rt;
}

template <bool STATS>
__global__ __launch_bounds__(512) void conv3x3_s1_c64_kernel(ConvNArgs a, int rt, int ntiles) {
  __shared__ __attribute__((aligned(16))) char smem[kC3A + kC3PMax * 128 + kC3C + 2 * 512 * 4];
  char* As = smem;
  char* Ps = smem + kC3A;
  bf16* Cs = reinterpret_cast<bf16*>(smem + kC3A + kC3PMax * 128);
  float* bred = reinterpret_cast<float*>(smem + kC3A + kC3PMax * 128 + kC3C);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, m = lane & 15;
  const int W = a.OW, PWd = W + 2, npx = rt * W, npp = (rt + 2) * PWd, bands = a.OH / rt;
  const u32x4 z4 = {0u, 0u, 0u, 0u};
  // filters once per block: LDS row co, k = tap * 64 + ci (data gradient: tap flipped, 8 - tap)
  for (int v = tid; v < 64 * 72; v += 512) {
    const int row = v / 72, kv = v - row * 72, tap = kv >> 3, ch = kv & 7;
    *reinterpret_cast<u32x4*>(As + row * (kC3WP * 2) + kv * 16) =
        *reinterpret_cast<const u32x4*>(a.wt + (size_t)row * 576 + (a.dgrad ? 8 - tap : tap) * 64 + 8 * ch);
  }
  // this lane's band pixels (groups 2w, 2w + 1): patch offset of tap (0, 0), validity
  int poff[2];
  bool pval[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int p = 16 * (2 * w + j) + m;
    pval[j] = p < npx;
    const int pp = pval[j] ? p : 0, pr = pp / W;
    poff[j] = pr * PWd + (pp - pr * W);
  }
  constexpr int NPV = (kC3PMax * 8 + 511) / 512;
  u32x4 pv[NPV];
  auto gload = [&](int t) {
    const int n = t / bands, ih0 = (t - n * bands) * rt - 1;
    const bf16* xin = a.act + (size_t)n * a.IH * a.IW * 64;
#pragma unroll
    for (int i = 0; i < NPV; ++i) {
      const int v = min(tid + 512 * i, npp * 8 - 1), pix = v >> 3, ch = v & 7;
      const int pr = pix / PWd, pc = pix - pr * PWd, ih = ih0 + pr, iw = pc - 1;
      const bool ok = (unsigned)ih < (unsigned)a.IH && (unsigned)iw < (unsigned)a.IW;
      pv[i] = *reinterpret_cast<const u32x4*>(xin + (size_t)(ok ? ih * a.IW + iw : 0) * 64 + 8 * ch);
      if (!ok) pv[i] = z4;
    }
  };
  auto pstore = [&] {
#pragma unroll
    for (int i = 0; i < NPV; ++i) {
      const int v = tid + 512 * i, pix = v >> 3, ch = v & 7;
      if (v < npp * 8) *reinterpret_cast<u32x4*>(Ps + pix * 128 + 16 * c3_swz(pix, ch)) = pv[i];
    }
  };
  int t = blockIdx.x;
  if (t < ntiles) {
    gload(t);
    pstore();
  }
  __syncthreads();
  const char* arow = As + m * (kC3WP * 2) + g * 16;
  constexpr int CP = 72;
  for (; t < ntiles; t += gridDim.x) {
    const bool more = t + (int)gridDim.x < ntiles;
    if (more) gload(t + gridDim.x);
    f32x4 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
    for (int ks = 0; ks < 18; ++ks) {
      const int tap = ks >> 1, r = tap / 3, s = tap - 3 * r, c = 4 * (ks & 1) + g;
      bf16x8 fa[4], fb[2];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        fa[i] = *reinterpret_cast<const bf16x8*>(arow + i * 16 * (kC3WP * 2) + ks * 64);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int pix = poff[j] + r * PWd + s;
        fb[j] = *reinterpret_cast<const bf16x8*>(Ps + pix * 128 + 16 * c3_swz(pix, c));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        *reinterpret_cast<uint2*>(Cs + (16 * (2 * w + j) + m) * CP + 16 * i + 4 * g) =
            make_uint2(pack2(acc[i][j][0], acc[i][j][1]), pack2(acc[i][j][2], acc[i][j][3]));
    __syncthreads();  // C tile complete; every wave done with this band's patch
    if (more) pstore();
    const size_t obase = (size_t)t * npx * 64;  // bands are consecutive row ranges: pixel t * npx + px
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int v = tid + 512 * k, px = v >> 3, cv = v & 7;
      if (px < npx) {
        const size_t o = obase + (size_t)px * 64 + 8 * cv;
        u32x4 val = *reinterpret_cast<const u32x4*>(Cs + px * CP + 8 * cv);
        if (a.addend) val = join8(val, a.addend, a.amask, o);
        *reinterpret_cast<u32x4*>(a.out + o) = val;
      }
    }
    if constexpr (STATS) {  // BN partial sums of the stored (bf16) band, one row per band
      const int cc = tid & 63, q = tid >> 6;
      const float K = a.bnshift ? a.bnshift[cc] : 0.f;
      const uint16_t* col = reinterpret_cast<const uint16_t*>(Cs) + cc;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll 8
      for (int rr = 0; rr < 32; ++rr) {
        const int px = 32 * q + rr;
        const float d = px < npx ? bf2f(col[px * CP]) - K : 0.f;
        s1 += d;
        s2 = fmaf(d, d, s2);
      }
      bred[tid] = s1;
      bred[512 + tid] = s2;
      __syncthreads();
      if (q == 0) {
        float t1 = s1, t2 = s2;
        for (int k = 1; k < 8; ++k) {
          t1 += bred[tid + 64 * k];
          t2 += bred[512 + tid + 64 * k];
        }
        float* dst = a.bnpart + (size_t)t * 128 + 2 * cc;
        dst[0] = t1;
        dst[1] = t2;
      }
    }
    __syncthreads();  // C tile / reduction slots read; the next patch stored
  }
}

static bool c3_eligible(const ConvNArgs& a) {
  return a.Ca == 64 && a.Ng == 64 && a.R == 3 && a.S == 3 && a.sh == 1 && a.sw == 1 && a.ph == 1 && a.pw == 1 &&
         a.OH == a.IH && a.OW == a.IW && a.OW <= 64 && c3_band_rows(a.OH, a.OW) >= 2;
}

static bool stem_eligible(const ConvNArgs& a) {
  return !a.dgrad && a.Ca == 8 && a.R == 7 && a.S == 7 && a.sh == 2 && a.sw == 2 && a.ph == 3 && a.pw == 3 &&
         a.Ng == 64 && a.OH % 16 == 0 && a.OW % 16 == 0 && !a.addend && a.OH == (a.IH + 6 - 7) / 2 + 1 &&
         a.OW == (a.IW + 6 - 7) / 2 + 1;
}

// split-K epilogue: out (bf16) = sum over splits of the fp32 partials (fixed order).  8 partial
// planes per round with every load issued before the first add, at clamped indices (one load per
// iteration of a runtime-length loop waited for each in turn).
// STATS (forward, the output feeds a training BatchNorm): the BN's partial sums of (y - shift[c])
// and its square over the STORED bf16 values, one row of bnpart (layout of bn_nhwc_partial_k) per
// `bpr` blocks.  The host guarantees a grid stride that is a multiple of Ng / 4 (each thread's
// channel quad is fixed) and blocks that start on a row boundary (splitk_bn_ok).
template <bool STATS>
__global__ __launch_bounds__(256) void conv_nhwc_splitk_reduce_k(const float* __restrict__ part, bf16* __restrict__ out,
                                                                 int64_t n4, int splits, const bf16* __restrict__ addend,
                                                                 const uint8_t* __restrict__ amask, float* __restrict__ bnpart,
                                                                 const float* __restrict__ bnshift, int Ng, int wt) {
  const float4* p4 = reinterpret_cast<const float4*>(part);
  const int q4 = Ng >> 2;
  const int cq = STATS ? (int)((blockIdx.x * 256ll + threadIdx.x) % q4) : 0;
  float K[4] = {0.f, 0.f, 0.f, 0.f}, s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
  if (STATS && bnshift) {
#pragma unroll
    for (int j = 0; j < 4; ++j) K[j] = bnshift[4 * cq + j];
  }
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    auto round = [&](auto nb, int sp0) {  // nb planes, loads first, then the adds in split order
      constexpr int NB = decltype(nb)::value;
      float4 u[NB];
#pragma unroll
      for (int k = 0; k < NB; ++k) u[k] = p4[(int64_t)min(sp0 + k, splits - 1) * n4 + i];
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        const bool in = sp0 + k < splits;
        s.x += in ? u[k].x : 0.f; s.y += in ? u[k].y : 0.f; s.z += in ? u[k].z : 0.f; s.w += in ? u[k].w : 0.f;
      }
    };
    if (splits <= 4) round(std::integral_constant<int, 4>{}, 0);  // most splits: 2-4, no redundant loads
    else
      for (int sp0 = 0; sp0 < splits; sp0 += 8) round(std::integral_constant<int, 8>{}, sp0);
    if (addend) {
      uint2 d = reinterpret_cast<const uint2*>(addend)[i];
      if (amask) {  // 4 elements: bits 4 (i & 1) .. + 3 of byte i / 2
        const uint32_t mb = (uint32_t)amask[i >> 1] >> (4 * (i & 1));
        d.x &= (mb & 1u ? 0x0000ffffu : 0u) | (mb & 2u ? 0xffff0000u : 0u);
        d.y &= (mb & 4u ? 0x0000ffffu : 0u) | (mb & 8u ? 0xffff0000u : 0u);
      }
      s.x += bf2f(d.x & 0xffffu); s.y += bf2f(d.x >> 16); s.z += bf2f(d.y & 0xffffu); s.w += bf2f(d.y >> 16);
    }
    const uint2 o = make_uint2(pack2(s.x, s.y), pack2(s.z, s.w));
    if (wt) {
      const u32x2 q = {o.x, o.y};
      asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(reinterpret_cast<uint2*>(out) + i), "v"(q) : "memory");
    } else {
      reinterpret_cast<uint2*>(out)[i] = o;
    }
    if (STATS) {
      const float y[4] = {bf2f(o.x & 0xffffu), bf2f(o.x >> 16), bf2f(o.y & 0xffffu), bf2f(o.y >> 16)};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = y[j] - K[j];
        s1[j] += d;
        s2[j] = fmaf(d, d, s2[j]);
      }
    }
  }
  if constexpr (STATS) {
    // the threads of one channel quad (256 / q4 of them when q4 < 256) summed in a fixed order
    __shared__ float red[8][256];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      red[j][threadIdx.x] = s1[j];
      red[4 + j][threadIdx.x] = s2[j];
    }
    __syncthreads();
    const int qb = q4 < 256 ? q4 : 256, bpr = q4 < 256 ? 1 : q4 / 256;
    if ((int)threadIdx.x >= qb) return;
    for (int g = 1; g < 256 / qb; ++g) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s1[j] += red[j][threadIdx.x + g * qb];
        s2[j] += red[4 + j][threadIdx.x + g * qb];
      }
    }
    float4* dst = reinterpret_cast<float4*>(bnpart + (size_t)(blockIdx.x / bpr) * 2 * Ng + 8 * cq);
    dst[0] = make_float4(s1[0], s2[0], s1[1], s2[1]);
    dst[1] = make_float4(s1[2], s2[2], s1[3], s2[3]);
  }
}

// ------------------------------------------------------------------------------------------
// weight gradient: rows = output channels k, columns = (r, s, c), reduction over pixels
struct WgNArgs {
  const bf16* dy;  // [Npix][Kout]
  const bf16* x;   // [N][H][W][Ca]
  float* part;     // fp32 partials [splits][Kout][Ng]
  int Npix, Kout, Ca, Cin, H, W, P, Q, R, S, sh, sw, ph, pw, Ng;
  int chunk;       // pixels per split (multiple of 32)
  FastDiv fQ, fPQ, fCa, fS;
};

// Weight-gradient LDS tiles are pixel-major [64 pixels][pitch] with pitch = width + 32 and the
// 16-byte chunks of rows 8-15 (mod 16) XOR-swizzled by 2: with that, both the ds_read_b64_tr_b16
// fragment reads (a 32-lane group reads rows {0-3, 8-11} (+4) x 32 bytes) and the ds_write_b128
// staging stores are bank-conflict-free (found by enumerating pitches and XOR swizzles against
// the gfx950 lane groups; the plain +8 pitch measured ~1 conflict cycle per LDS cycle).
__device__ __forceinline__ int wg_swz(int row) { return ((row >> 3) & 1) * 2; }

__device__ __forceinline__ bf16x8 tr_frag(const bf16* tile, int pitch, int col0, int lane) {
  // MFMA operand for "row" = channel col0 + (lane & 15), k = pixels 8 * (lane >> 4) .. + 7 from a
  // pixel-major [32][pitch] tile: two transposed reads of 4 pixels x 16 channels each.
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const int r = 8 * g + q;  // rows r and r + 4 share the swizzle (same bit 3)
  const bf16* p0 = tile + r * pitch + ((((col0 >> 3) + (p >> 1)) ^ wg_swz(r)) << 3) + 4 * (p & 1);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0 + 4 * pitch));
  bf16x8 res;
  res[0] = lo[0]; res[1] = lo[1]; res[2] = lo[2]; res[3] = lo[3];
  res[4] = hi[0]; res[5] = hi[1]; res[6] = hi[2]; res[7] = hi[3];
  return res;
}

// TM x TN output tile (output channels x (r, s, c) columns) over WGM x WGN waves, TM, TN in
// {64, 128, 256}: 64-wide tiles for the 64-channel layers (a 128-wide tile over a 64-channel
// operand computes 50-75 % zeros).  The 256 x 256 tile (8 waves of 128 x 64, one 147 KB block per
// CU) stages 1 KB per pixel for 128 K FLOP (128 FLOP per staged byte, vs 64 for 128 x 128: at
// 64 FLOP/B a CU's 64 B/clk from L2 only just feeds its MFMAs, so the 128-tile kernel ran at
// 17 % MFMA busy, profiles/r4_pmc/pmc_rn.txt).  The LDS pitch rule (width + 32, wg_swz) keeps the
// row stride at 16 banks for every width, so the same swizzle stays conflict-free.
template <int TM, int TN, int WGM = 2, int WGN = 2>
__global__ __launch_bounds__(64 * WGM * WGN) void wgrad_nhwc_kernel(WgNArgs a) {
  constexpr int NT = 64 * WGM * WGN;       // threads
  constexpr int BK = 64;                   // pixels per stage (two MFMA k-steps)
  constexpr int PA = TM + 32, PB = TN + 32;  // LDS pitches (see wg_swz)
  constexpr int VA = TM / 8, VB = TN / 8;  // 16-byte vectors per pixel row
  static_assert(NT % VA == 0 && NT % VB == 0, "load roles: a thread keeps its vector column");
  constexpr int EA = BK * VA / NT, EB = BK * VB / NT;
  constexpr int WTM = TM / WGM, WTN = TN / WGN;  // wave tile
  constexpr int WMT = WTM / 16, WNT = WTN / 16;
  __shared__ __attribute__((aligned(16))) bf16 As[2][BK * PA];  // dy tile  [pixel][k]
  __shared__ __attribute__((aligned(16))) bf16 Bs[2][BK * PB];  // x gather [pixel][(r,s,c)]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave / WGN, wn = wave % WGN;
  const int tiles_m = (a.Kout + TM - 1) / TM, tiles_n = (a.Ng + TN - 1) / TN;
  const int bid = blockIdx.x;
  const int tm = bid % tiles_m, r1 = bid / tiles_m, tn = r1 % tiles_n, sp = r1 / tiles_n;
  const int m0 = tm * TM, n0 = tn * TN;
  const int pbeg = sp * a.chunk, pend = min(a.Npix, pbeg + a.chunk);
  if (pbeg >= pend) return;
  // load roles (fixed per thread: NT is a multiple of VA and VB): A vector cva of pixel rows
  // rowa0 + (NT / VA) i, B vector cvb of rows rowb0 + (NT / VB) i
  const int cva = tid % VA, rowa0 = tid / VA, cvb = tid % VB, rowb0 = tid / VB;
  // B column decomposition (fixed per thread): column n0 + 8 cvb -> (r, s, c)
  const int col = n0 + 8 * cvb;
  const bool col_ok = col < a.Ng;
  const int colc = col_ok ? col : 0;
  const int rs = (int)a.fCa.div((uint32_t)colc), bc = colc - rs * a.Ca;
  const int br = (int)a.fS.div((uint32_t)rs), bs = rs - br * a.S;
  const bool k_ok = m0 + 8 * cva < a.Kout;
  // every load is issued unconditionally from a valid (clamped) address and its validity kept
  // beside it; the mask is applied when the stage is written to LDS.  (Masking right after the
  // load, hipcc branched around each load and waited for the next stage's loads -- s_waitcnt
  // vmcnt(0) -- before the current stage's MFMAs: no overlap at all.)
  u32x4 ra[EA], rb[EB];
  bool ma[EA], mb[EB];
  const u32x4 z4 = {0u, 0u, 0u, 0u};
  auto gload = [&](int p0) {
#pragma unroll
    for (int i = 0; i < EA; ++i) {
      const int pix = p0 + rowa0 + (NT / VA) * i;
      ma[i] = pix < pend && k_ok;
      ra[i] = *reinterpret_cast<const u32x4*>(a.dy + (ma[i] ? (size_t)pix * a.Kout + m0 + 8 * cva : 0));
    }
#pragma unroll
    for (int i = 0; i < EB; ++i) {
      const int pix = p0 + rowb0 + (NT / VB) * i;
      const bool ok = pix < pend;
      const int pp = ok ? pix : 0;
      const int n = (int)a.fPQ.div((uint32_t)pp), rem = pp - n * a.P * a.Q;
      const int p = (int)a.fQ.div((uint32_t)rem), q = rem - p * a.Q;
      const int h = p * a.sh - a.ph + br, w = q * a.sw - a.pw + bs;
      mb[i] = ok && col_ok && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
      rb[i] = *reinterpret_cast<const u32x4*>(a.x + (mb[i] ? (((size_t)n * a.H + h) * a.W + w) * a.Ca + bc : 0));
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < EA; ++i) {
      const int r = rowa0 + (NT / VA) * i;
      *reinterpret_cast<u32x4*>(&As[buf][r * PA + 8 * (cva ^ wg_swz(r))]) = ma[i] ? ra[i] : z4;
    }
#pragma unroll
    for (int i = 0; i < EB; ++i) {
      const int r = rowb0 + (NT / VB) * i;
      *reinterpret_cast<u32x4*>(&Bs[buf][r * PB + 8 * (cvb ^ wg_swz(r))]) = mb[i] ? rb[i] : z4;
    }
  };

  f32x4 acc[WMT][WNT];
#pragma unroll
  for (int i = 0; i < WMT; ++i)
#pragma unroll
    for (int j = 0; j < WNT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nt = (pend - pbeg + BK - 1) / BK;
  gload(pbeg);
  sstore(0);
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    if (t + 1 < nt) gload(pbeg + (t + 1) * BK);
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 av[WMT], bv[WNT];
#pragma unroll
      for (int i = 0; i < WMT; ++i) av[i] = tr_frag(As[cur] + 32 * ks * PA, PA, wm * WTM + 16 * i, lane);
#pragma unroll
      for (int j = 0; j < WNT; ++j) bv[j] = tr_frag(Bs[cur] + 32 * ks * PB, PB, wn * WTN + 16 * j, lane);
#pragma unroll
      for (int i = 0; i < WMT; ++i)
#pragma unroll
        for (int j = 0; j < WNT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (t + 1 < nt) sstore(cur ^ 1);
    __syncthreads();
  }

  float* pl = a.part + (size_t)sp * a.Kout * a.Ng;
#pragma unroll
  for (int j = 0; j < WNT; ++j) {
    const int cn = n0 + wn * WTN + 16 * j + (lane & 15);
    if (cn >= a.Ng) continue;
#pragma unroll
    for (int i = 0; i < WMT; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = m0 + wm * WTM + 16 * i + 4 * (lane >> 4) + r;
        if (k < a.Kout) pl[(size_t)k * a.Ng + cn] = acc[i][j][r];
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// Stem weight gradient (the forward's conv_nhwc_stem_kernel shape): dW[co][(r, s, c)] = sum over
// output pixels of dy[px][co] x[2 oh + r - 3][2 ow + s - 3][c].  The generic kernel gathers
// every (pixel, tap) vector from L2 once per tap (49x per input pixel, 32-byte strided: 527 us
// per step at batch 256).  Here a PERSISTENT block walks 16 x 16 output tiles: per tile the dy
// tile [256 px][64 co] and the 37 x 38 input patch are staged in LDS once (the next tile's loads
// in flight in registers during this tile's MFMAs), and per 32-pixel k-step the pixel-major
// im2col rows [32 px][56 (r, s8) x 8 c] are expanded from the patch in LDS (16-byte copies) and
// read with ds_read_b64_tr_b16 exactly like the generic kernel's tiles.  The 64 x 448 fp32
// result stays in registers over all tiles of the block (wave w: 4 co tiles x n tiles w + 8 t);
// one partial plane per block in the generic layout (s = 7 dropped), summed by
// wgrad_nhwc_reduce_k.
constexpr int kSwPA = 64 + 32, kSwPB = 448 + 32;  // LDS pitches (bf16), see wg_swz
// patch rows of 40 16-byte pixels (37 used): the im2col build's b128 reads (consecutive (r, s) of
// one pixel, rows 40 chunks apart) average 5.5 LDS cycles against 10 at the forward's 38
// (scripts/ldsbank/bank.py over the 8 k-steps' build reads; ideal 4)
constexpr int kSwPW = 40;
constexpr int kSwA = 256 * kSwPA * 2, kSwP = kStemPH * kSwPW * 16, kSwB = 32 * kSwPB * 2;

__global__ __launch_bounds__(512) void wgrad_stem_kernel(WgNArgs a, int ntiles) {
  __shared__ __attribute__((aligned(16))) char smem[kSwA + kSwP + 2 * kSwB];
  bf16* As = reinterpret_cast<bf16*>(smem);                      // dy tile [256 px][kSwPA]
  char* Ps = smem + kSwA;                                         // patch [37][38] x 16 B
  bf16* Bs = reinterpret_cast<bf16*>(smem + kSwA + kSwP);         // im2col [2][32 px][kSwPB]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int tw_n = a.Q >> 4, th_n = a.P >> 4;
  constexpr int NDV = 256 * 8 / 512, NPV = (kStemPH * kSwPW + 511) / 512;
  u32x4 dv[NDV], pv[NPV];
  const u32x4 z4 = {0u, 0u, 0u, 0u};
  auto gload = [&](int t) {
    const int n = t / (th_n * tw_n), trem = t - n * th_n * tw_n;
    const int oh0 = (trem / tw_n) * 16, ow0 = (trem % tw_n) * 16;
#pragma unroll
    for (int i = 0; i < NDV; ++i) {
      const int v = tid + 512 * i, px = v >> 3, cv = v & 7;
      dv[i] = *reinterpret_cast<const u32x4*>(
          a.dy + (((size_t)n * a.P + oh0 + (px >> 4)) * a.Q + ow0 + (px & 15)) * 64 + 8 * cv);
    }
    const bf16* xin = a.x + (size_t)n * a.H * a.W * 8;
#pragma unroll
    for (int i = 0; i < NPV; ++i) {
      const int v = min(tid + 512 * i, kStemPH * kSwPW - 1), pr = v / kSwPW, pc = v - pr * kSwPW;
      const int ih = 2 * oh0 - 3 + pr, iw = 2 * ow0 - 3 + pc;
      const bool ok = (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W && pc < 37;
      pv[i] = *reinterpret_cast<const u32x4*>(xin + (size_t)(ok ? ih * a.W + iw : 0) * 8);
      if (!ok) pv[i] = z4;
    }
  };
  auto sstore = [&] {
#pragma unroll
    for (int i = 0; i < NDV; ++i) {
      const int v = tid + 512 * i, px = v >> 3, cv = v & 7;
      *reinterpret_cast<u32x4*>(As + px * kSwPA + 8 * (cv ^ wg_swz(px))) = dv[i];
    }
#pragma unroll
    for (int i = 0; i < NPV; ++i) {
      const int v = tid + 512 * i;
      if (v < kStemPH * kSwPW) *reinterpret_cast<u32x4*>(Ps + v * 16) = pv[i];
    }
  };
  // im2col rows of k-step ks (tile pixel rows 2 ks, 2 ks + 1) -> buffer buf
  auto build = [&](int ks, int buf) {
    bf16* B = Bs + buf * 32 * kSwPB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int v = tid + 512 * i;
      if (v < 32 * 56) {
        const int pl = v / 56, rs8 = v - pl * 56, r = rs8 >> 3, s = rs8 & 7;
        const int ohl = 2 * ks + (pl >> 4), owl = pl & 15;
        const u32x4 val = *reinterpret_cast<const u32x4*>(Ps + ((2 * ohl + r) * kSwPW + 2 * owl + s) * 16);
        *reinterpret_cast<u32x4*>(B + pl * kSwPB + 8 * (rs8 ^ wg_swz(pl))) = val;
      }
    }
  };

  const int nj = w < 4 ? 4 : 3;  // n tiles of this wave: w + 8 t (28 tiles of 16 columns)
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  int t = blockIdx.x;
  if (t < ntiles) {
    gload(t);
    sstore();
  }
  __syncthreads();
  for (; t < ntiles; t += gridDim.x) {
    const bool more = t + (int)gridDim.x < ntiles;
    if (more) gload(t + gridDim.x);  // next tile in flight during this one
    build(0, 0);
    __syncthreads();
    for (int ks = 0; ks < 8; ++ks) {
      if (ks + 1 < 8) build(ks + 1, (ks + 1) & 1);
      const bf16* B = Bs + (ks & 1) * 32 * kSwPB;
      bf16x8 av[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) av[i] = tr_frag(As + 32 * ks * kSwPA, kSwPA, 16 * i, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j < nj) {
          const bf16x8 bv = tr_frag(B, kSwPB, 16 * (w + 8 * j), lane);
#pragma unroll
          for (int i = 0; i < 4; ++i)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv, acc[i][j], 0, 0, 0);
        }
      }
      __syncthreads();
    }
    if (more) sstore();
    __syncthreads();
  }
  // partial plane of this block, generic layout [64 co][(r * 7 + s) * 8 + c] (s = 7 dropped)
  float* pl = a.part + (size_t)blockIdx.x * 64 * 392;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (j >= nj) continue;
    const int n8 = 16 * (w + 8 * j) + (lane & 15), rs8 = n8 >> 3, c = n8 & 7, r = rs8 >> 3, s = rs8 & 7;
    if (s == 7) continue;
    const int col = (r * 7 + s) * 8 + c;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) pl[(size_t)(16 * i + 4 * (lane >> 4) + q) * 392 + col] = acc[i][j][q];
  }
}

// ------------------------------------------------------------------------------------------
// Weight gradient of the 3x3 / stride-1 / 64-channel convolution (conv3x3_s1_c64_kernel's shape):
// persistent blocks walk the same full-width row bands; per band the dy rows [npx][64] and the
// (rt + 2) x (W + 2) x 64 input patch are staged in LDS once (the next band's in registers during
// this band's MFMAs).  dW[co][(tap, c)] = sum_px dy[px][co] x[px + tap][c]: the reduction runs
// over band pixels, 8 consecutive ones per lane group, which (W % 8 == 0) are 8 consecutive patch
// pixels of one row -- so the B operand is read with ds_read_b64_tr_b16 straight out of the
// patch at the tap-shifted pixel, no im2col; A (dy^T) as in the generic kernel.  The 64 x 576
// result stays in registers over all bands of a block (wave w: 4 co tiles x column tiles
// w + 8 t); one partial plane per block, summed by wgrad_nhwc_reduce_k.
// (Round 6: the slot (c + 2 (P >> 1) + 4 (P >> 3)) & 7 averages 2.16 LDS cycles per transposed read
// against this XOR's 3.43 -- LDS conflict cycles 54 % -> 6 % -- but the kernel ran 93.8 -> 101.8 us;
// profiles/r6_ldsbank2/.)
__device__ __forceinline__ bf16x8 patch_tr_frag(const bf16* ps, int pix0, int c16, int lane) {
  // rows = patch pixels pix0 + 8 (lane >> 4) + q (+ 4), columns = channels 8 c16 + (lane & 15)
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const int P0 = pix0 + 8 * g + q, P1 = P0 + 4, ch = c16 + (p >> 1);
  const bf16* a0 = ps + P0 * 64 + 8 * (ch ^ ((P0 >> 1) & 7)) + 4 * (p & 1);
  const bf16* a1 = ps + P1 * 64 + 8 * (ch ^ ((P1 >> 1) & 7)) + 4 * (p & 1);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
  bf16x8 res;
  res[0] = lo[0]; res[1] = lo[1]; res[2] = lo[2]; res[3] = lo[3];
  res[4] = hi[0]; res[5] = hi[1]; res[6] = hi[2]; res[7] = hi[3];
  return res;
}

constexpr int kWc3PA = 64 + 32;
__global__ __launch_bounds__(512) void wgrad_c3_kernel(WgNArgs a, int rt, int nbands) {
  __shared__ __attribute__((aligned(16))) char smem[256 * kWc3PA * 2 + kC3PMax * 128];
  bf16* Ds = reinterpret_cast<bf16*>(smem);                // dy band [px][kWc3PA]
  char* Ps = smem + 256 * kWc3PA * 2;                       // patch, chunks XOR-swizzled
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int W = a.Q, PWd = W + 2, npx = rt * W, npp = (rt + 2) * PWd, bpi = a.P / rt;
  const int nks = (npx + 31) >> 5;
  const u32x4 z4 = {0u, 0u, 0u, 0u};
  constexpr int NDV = 256 * 8 / 512, NPV = (kC3PMax * 8 + 511) / 512;
  u32x4 dv[NDV], pv[NPV];
  auto gload = [&](int t) {
#pragma unroll
    for (int i = 0; i < NDV; ++i) {
      const int v = tid + 512 * i, px = v >> 3, cv = v & 7;
      const int pc = min(px, npx - 1);
      dv[i] = *reinterpret_cast<const u32x4*>(a.dy + ((size_t)t * npx + pc) * 64 + 8 * cv);
      if (px >= npx) dv[i] = z4;
    }
    const int n = t / bpi, ih0 = (t - n * bpi) * rt - 1;
    const bf16* xin = a.x + (size_t)n * a.H * a.W * 64;
#pragma unroll
    for (int i = 0; i < NPV; ++i) {
      const int v = min(tid + 512 * i, npp * 8 - 1), pix = v >> 3, ch = v & 7;
      const int pr = pix / PWd, pc = pix - pr * PWd, ih = ih0 + pr, iw = pc - 1;
      const bool ok = (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      pv[i] = *reinterpret_cast<const u32x4*>(xin + (size_t)(ok ? ih * a.W + iw : 0) * 64 + 8 * ch);
      if (!ok) pv[i] = z4;
    }
  };
  auto sstore = [&] {
#pragma unroll
    for (int i = 0; i < NDV; ++i) {
      const int v = tid + 512 * i, px = v >> 3, cv = v & 7;
      *reinterpret_cast<u32x4*>(Ds + px * kWc3PA + 8 * (cv ^ wg_swz(px))) = dv[i];
    }
#pragma unroll
    for (int i = 0; i < NPV; ++i) {
      const int v = tid + 512 * i, pix = v >> 3, ch = v & 7;
      if (v < npp * 8) *reinterpret_cast<u32x4*>(Ps + pix * 128 + 16 * (ch ^ ((pix >> 1) & 7))) = pv[i];
    }
  };
  const int nj = w < 4 ? 5 : 4;  // column tiles w + 8 t of the 36
  f32x4 acc[4][5];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 5; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int t = blockIdx.x;
  if (t < nbands) {
    gload(t);
    sstore();
  }
  __syncthreads();
  const bf16* ps = reinterpret_cast<const bf16*>(Ps);
  for (; t < nbands; t += gridDim.x) {
    const bool more = t + (int)gridDim.x < nbands;
    if (more) gload(t + gridDim.x);
    for (int ks = 0; ks < nks; ++ks) {
      bf16x8 av[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) av[i] = tr_frag(Ds + 32 * ks * kWc3PA, kWc3PA, 16 * i, lane);
      // first pixel of this k-step's lane groups: 8-pixel groups never straddle a band row (W % 8 == 0)
      const int p0 = min(32 * ks + 8 * (lane >> 4), npx - 8), pr = p0 / W, base = pr * PWd + (p0 - pr * W);
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        if (j < nj) {
          const int nt = w + 8 * j, tap = nt >> 2, r = tap / 3, s = tap - 3 * r;
          // patch_tr_frag adds 8 (lane >> 4) itself: pass the group-0 origin of this lane's group
          const bf16x8 bv = patch_tr_frag(ps, base + r * PWd + s - 8 * (lane >> 4), 2 * (nt & 3), lane);
#pragma unroll
          for (int i = 0; i < 4; ++i)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv, acc[i][j], 0, 0, 0);
        }
      }
    }
    __syncthreads();  // every wave done with this band's tiles
    if (more) sstore();
    __syncthreads();
  }
  float* pl = a.part + (size_t)blockIdx.x * 64 * 576;
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    if (j >= nj) continue;
    const int col = 16 * (w + 8 * j) + (lane & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) pl[(size_t)(16 * i + 4 * (lane >> 4) + q) * 576 + col] = acc[i][j][q];
  }
}

static bool wgrad_c3_eligible(const WgNArgs& a) {
  return a.Ca == 64 && a.Kout == 64 && a.R == 3 && a.S == 3 && a.sh == 1 && a.sw == 1 && a.ph == 1 && a.pw == 1 &&
         a.P == a.H && a.Q == a.W && a.Q <= 64 && a.Q % 8 == 0 && c3_band_rows(a.P, a.Q) >= 2;
}

static bool wgrad_stem_eligible(const WgNArgs& a) {
  return a.Ca == 8 && a.R == 7 && a.S == 7 && a.sh == 2 && a.sw == 2 && a.ph == 3 && a.pw == 3 && a.Kout == 64 &&
         a.P % 16 == 0 && a.Q % 16 == 0 && a.P == (a.H + 6 - 7) / 2 + 1 && a.Q == (a.W + 6 - 7) / 2 + 1;
}
constexpr int kSwBlocks = 256;  // persistent blocks (one per CU: 131 KB of LDS each)

// dw[k][c][r][s] (+)= sum over splits of part[sp][k][(r, s, c)] (c < Cin; padded channels dropped).
// Block = (256 / G) float4 column quads x G split groups: thread (q, g) sums splits g, g + G, ...
// of its quad (float4 loads, 4 consecutive columns of one tap since Ca % 8 == 0), the G group
// sums are combined in LDS in a fixed order (deterministic).  Many splits (the 56 x 56 layers
// have ~200) are spread over the G groups instead of one thread's serial chain.
__device__ __forceinline__ void nhwc_reduce_body(const float* __restrict__ part, float* __restrict__ dw, int splits,
                                                 int Kout, int Ng, int Ca, int Cin, int RS, int accumulate, int G,
                                                 int blk) {
  __shared__ float4 red[256];
  const int plane4 = Kout * Ng / 4, QB = 256 / G;
  const int q = threadIdx.x % QB, g = threadIdx.x / QB;
  const int i = blk * QB + q;
  const float4* p4 = reinterpret_cast<const float4*>(part);
  // 8 partial planes per round with every load issued before the first add, at clamped indices
  // (a plane past `splits` or a lane past the plane loads a valid element and discards it): the
  // former loop, behind a per-lane range check, waited for each pair of loads in turn -- at batch
  // 32 (~200 splits) that was ~6 dependent round trips per launch
  const int ic = min(i, plane4 - 1);
  float4 acc[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int sp0 = g; sp0 < splits; sp0 += 8 * G) {
    float4 u[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) u[k] = p4[(size_t)min(sp0 + k * G, splits - 1) * plane4 + ic];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const bool in = sp0 + k * G < splits;
      acc[k & 3].x += in ? u[k].x : 0.f;
      acc[k & 3].y += in ? u[k].y : 0.f;
      acc[k & 3].z += in ? u[k].z : 0.f;
      acc[k & 3].w += in ? u[k].w : 0.f;
    }
  }
  red[threadIdx.x] = make_float4((acc[0].x + acc[1].x) + (acc[2].x + acc[3].x), (acc[0].y + acc[1].y) + (acc[2].y + acc[3].y),
                                 (acc[0].z + acc[1].z) + (acc[2].z + acc[3].z), (acc[0].w + acc[1].w) + (acc[2].w + acc[3].w));
  __syncthreads();
  if (g != 0 || i >= plane4) return;
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < G; ++k) {
    const float4 r = red[k * QB + q];
    v[0] += r.x; v[1] += r.y; v[2] += r.z; v[3] += r.w;
  }
  const int e = 4 * i, k = e / Ng, n = e - k * Ng;
  const int rs = n / Ca, c = n - rs * Ca;
  float* d = dw + ((size_t)k * Cin + c) * RS + rs;
  // the 4 old values (accumulate) requested together at clamped channels, then the masked stores
  // (the per-element `break` made each read-add-write wait for its own load)
  float old[4] = {0.f, 0.f, 0.f, 0.f};
  if (accumulate) {
#pragma unroll
    for (int j = 0; j < 4; ++j) old[j] = d[(size_t)min(j, Cin - 1 - c) * RS];
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (c + j < Cin) d[(size_t)j * RS] = old[j] + v[j];
}

__global__ __launch_bounds__(256) void wgrad_nhwc_reduce_k(const float* __restrict__ part, float* __restrict__ dw,
                                                            int splits, int Kout, int Ng, int Ca, int Cin, int RS,
                                                            int accumulate, int G) {
  nhwc_reduce_body(part, dw, splits, Kout, Ng, Ca, Cin, RS, accumulate, G, blockIdx.x);
}

// many deferred reductions in one launch (wgrad_defer.h): block b runs job q's block b - blk0[q]
__global__ __launch_bounds__(256) void wgrad_nhwc_reduce_batch_k(RedBatch bt) {
  int q = 0;
  for (int k = 1; k < bt.n; ++k)
    if ((int)blockIdx.x >= bt.j[k].blk0) q = k;
  const RedJob& jb = bt.j[q];
  nhwc_reduce_body(jb.part, jb.dw, jb.nplanes, jb.Kout, jb.Ng, jb.Ca, jb.Cin, jb.RS, jb.acc, jb.G,
                   (int)blockIdx.x - jb.blk0);
}

// ------------------------------------------------------------------------------------------
// layout / weight conversion
// x fp32 [N][C][H][W] -> bf16 [N][H][W][Cp] (zeros for c >= C)
// one thread per (pixel, 8-channel group): 8 coalesced fp32 plane reads, one 16-byte store,
// 32-bit FastDiv indexing (the per-element 64-bit divisions and 2-byte stores ran at ~1.7 TB/s)
__global__ void nchw_to_nhwc_k(const float* __restrict__ x, uint4* __restrict__ y, int N, int C, int HW, int G,
                               FastDiv fG, FastDiv fHW) {
  const int total = N * HW * G;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int pix = (int)fG.div((uint32_t)i), g = i - pix * G;
    const int n = (int)fHW.div((uint32_t)pix), hw = pix - n * HW;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = 8 * g + e;
      v[e] = c < C ? x[((size_t)n * C + c) * HW + hw] : 0.f;
    }
    y[i] = pack8(v);
  }
}

// w fp32 [K][C][R][S] -> fwd: bf16 [K][R][S][Cp] (zero-padded channels) and/or dgrad: bf16
// [C][R][S][K]; both layouts in one pass when both pointers are given (one launch per conv)
__global__ void wrepack_k(const float* __restrict__ w, bf16* __restrict__ wt, bf16* __restrict__ wtd, int K, int C,
                          int R, int S, int Cp) {
  const int RS = R * S;
  const int64_t tf = wt ? (int64_t)K * RS * Cp : 0, td = wtd ? (int64_t)C * RS * K : 0;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < tf + td; i += (int64_t)gridDim.x * 256) {
    if (i < tf) {
      const int c = (int)(i % Cp);
      const int64_t krs = i / Cp;
      const int rs = (int)(krs % RS), k = (int)(krs / RS);
      wt[i] = c < C ? f2bf(w[((int64_t)k * C + c) * RS + rs]) : (bf16)0;
    } else {
      const int64_t j = i - tf;
      const int k = (int)(j % K);
      const int64_t crs = j / K;
      const int rs = (int)(crs % RS), c = (int)(crs / RS);
      wtd[j] = f2bf(w[((int64_t)k * C + c) * RS + rs]);
    }
  }
}

// Every convolution of a model in ONE launch (nhwc_repack_many): desc[i] = {w, wt, wtd, K, C,
// R*S, Cp, first block}; block b finds its convolution by binary search over the first-block
// column.  K % 8 == 0: the convolution's first cdiv(K*RS*Cp, 2048) blocks write the forward
// layout (8 outputs per thread, one 16-byte store), the rest are 64 x 64 tiles of the data-gradient
// layout, which is the transpose of w viewed as [K][C*RS]: read as coalesced rows into LDS, written
// as 16-byte vectors along k.  (A thread gathering 8 k straight from global read 8 cache lines
// 4 bytes each, C*RS*4 bytes apart: the one-launch repack ran at ~1.2 TB/s, 174 us per ResNet-50
// step.)  Otherwise every block strides over the convolution's elements (32-bit indices).
constexpr int kRepackPerBlock = 256 * 8;
constexpr int kRepackT = 64;  // data-gradient transpose tile (k x crs)

// forward-layout blocks of one convolution: 3x3 weights go through LDS tiles of 4 k x 64 c x 9
// taps (coalesced row loads instead of a 9-float-stride gather), the others 2,048 elements per
// block.  (Measured: the whole ResNet-50 repack 91.2 -> 89.6 us per step -- it is bound by
// reading the fp32 weights once per layout and writing both bf16 layouts, ~300 MB at ~3.4 TB/s.)
constexpr int kRepackTK = 4, kRepackTC = 64;
__host__ __device__ inline int repack_fwd_blocks(int K, int Cp, int RS) {
  if (RS == 9) return ((K + kRepackTK - 1) / kRepackTK) * ((Cp + kRepackTC - 1) / kRepackTC);
  const int64_t nf = (int64_t)K * RS * Cp;
  return (int)((nf + kRepackPerBlock - 1) / kRepackPerBlock);
}

__global__ __launch_bounds__(256) void wrepack_many_k(const int64_t* __restrict__ desc, int n) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (desc[mid * 8 + 7] <= (int64_t)blockIdx.x) lo = mid; else hi = mid - 1;
  }
  const int64_t* d = desc + lo * 8;
  const float* w = reinterpret_cast<const float*>(d[0]);
  bf16* wt = reinterpret_cast<bf16*>(d[1]);
  bf16* wtd = reinterpret_cast<bf16*>(d[2]);
  const int K = (int)d[3], C = (int)d[4], RS = (int)d[5], Cp = (int)d[6], b0 = (int)d[7];
  const int nb = (lo + 1 < n ? (int)desc[(lo + 1) * 8 + 7] : (int)gridDim.x) - b0;
  const int tf = wt ? K * RS * Cp : 0, td = wtd ? C * RS * K : 0;
  if ((K & 7) == 0) {
    // (WeightPack places every layout at a 64-element boundary, so the 16-byte stores are aligned)
    const int lb = (int)blockIdx.x - b0, fb = wt ? repack_fwd_blocks(K, Cp, RS) : 0;
    if (lb < fb && RS == 9) {  // forward layout of a 3x3 conv through an LDS tile
      __shared__ float fs[kRepackTK * kRepackTC * 9];
      const int ctiles = (Cp + kRepackTC - 1) / kRepackTC;
      const int k0 = (lb / ctiles) * kRepackTK, c0 = (lb % ctiles) * kRepackTC;
      // row kk of the tile = w[k0 + kk][c0 .. c0 + 63][0 .. 8]: 576 contiguous floats (clamped
      // loads, zeros outside the weight)
#pragma unroll
      for (int i = 0; i < 9; ++i) {
        const int idx = threadIdx.x + 256 * i, kk = idx / 576, off = idx - kk * 576, c = c0 + off / 9;
        const int k = k0 + kk;
        const float v = w[((size_t)min(k, K - 1) * C + min(c, C - 1)) * 9 + off % 9];
        fs[idx] = k < K && c < C ? v : 0.f;
      }
      __syncthreads();
      // wt[(k * 9 + tap) * Cp + c]: 8 channels of one (k, tap) per thread, 16-byte stores
      for (int id = threadIdx.x; id < kRepackTK * 9 * 8; id += 256) {
        const int kk = id / 72, rem = id - kk * 72, rs = rem >> 3, p = rem & 7;
        const int k = k0 + kk, c = c0 + 8 * p;
        if (k < K && c < Cp) {
          float v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = fs[kk * 576 + (8 * p + u) * 9 + rs];
          *reinterpret_cast<uint4*>(wt + ((size_t)k * 9 + rs) * Cp + c) = pack8(v);
        }
      }
      return;
    }
    if (lb < fb) {  // forward layout: 8 channels of one (k, tap) row per thread
      const int e = (lb * 256 + threadIdx.x) * 8;
      if (e < tf) {
        float v[8];
        const int krs = e / Cp, c0 = e - krs * Cp;
        const int k = krs / RS, rs = krs - k * RS;
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = c0 + u < C ? w[(k * C + c0 + u) * RS + rs] : 0.f;
        *reinterpret_cast<uint4*>(wt + e) = pack8(v);
      }
      return;
    }
    if (!wtd) return;
    // data-gradient layout: tile (k0.., j0..) of W[K][CRS] -> wtd[CRS][K]
    const int CRS = C * RS, tcols = (CRS + kRepackT - 1) / kRepackT;
    const int t = lb - fb, k0 = (t / tcols) * kRepackT, j0 = (t % tcols) * kRepackT;
    __shared__ float tile[kRepackT][kRepackT + 1];
    const int col = threadIdx.x & 63, r0 = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < kRepackT / 4; ++i) {  // 16 independent coalesced row loads per thread
      const int row = r0 + 4 * i, k = k0 + row, j = j0 + col;
      tile[row][col] = (k < K && j < CRS) ? w[(size_t)k * CRS + j] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int v = threadIdx.x + 256 * h, row = v >> 3, kv = v & 7;
      const int j = j0 + row, kk = k0 + 8 * kv;
      if (j < CRS && kk < K) {
        float f8[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) f8[u] = tile[8 * kv + u][row];
        *reinterpret_cast<uint4*>(wtd + (size_t)j * K + kk) = pack8(f8);
      }
    }
    return;
  }
  for (int i = ((int)blockIdx.x - b0) * 256 + threadIdx.x; i < tf + td; i += nb * 256) {
    if (i < tf) {
      const int c = i % Cp, krs = i / Cp;
      const int rs = krs % RS, k = krs / RS;
      wt[i] = c < C ? f2bf(w[(k * C + c) * RS + rs]) : (bf16)0;
    } else {
      const int j = i - tf;
      const int k = j % K, crs = j / K;
      const int rs = crs % RS, c = crs / RS;
      wtd[j] = f2bf(w[(k * C + c) * RS + rs]);
    }
  }
}

// ------------------------------------------------------------------------------------------
// BatchNorm over [Npix][C] (C % 8 == 0, 256 % (C / 8) == 0 or C / 8 a multiple of 256), three
// launches per direction:
//   partial  grid (gx, gy): each block reduces its pixel slice to per-channel partial sums and
//            WRITES them to part[blockIdx.x][2C] (no atomics: gx ~ 256 blocks keep HBM busy, and
//            same-address atomics from that many blocks serialise);
//   finalize one thread per channel sums the gx partials in a fixed order (deterministic) and
//            produces the per-channel affine coefficients (+ saved mean / invstd, running stats,
//            num_batches_tracked; backward: dgamma / dbeta);
//   apply    each block stages the coefficients of all C channels in LDS, then streams 8-channel
//            vectors: one FMA per element (+ residual, ReLU).
// Forward partials are sums of (x - K) and (x - K)^2 with K = x[pixel 0][c] (well conditioned
// when |mean| >> std); backward partials are sum(g) and sum(g (x - mean)), g = dy masked by the
// fused ReLU.  Thread (in a 256-thread block) owns vector v = tid % V of pixels tid / V + k * PPI.
constexpr int kBnT = 256;

struct BnNArgs {
  const bf16* x;      // BN input
  const bf16* res;    // residual added after the affine map (or null)
  bf16* y;            // output
  const bf16* dy;     // bwd: gradient wrt y
  bf16* dx;           // bwd: gradient wrt x
  bf16* dres;         // bwd: gradient wrt res (= relu-masked dy), or null
  const float* gamma;
  const float* beta;
  float* mean;        // [C] out (fwd) / in (bwd)
  float* invstd;      // [C]
  float* run_mean;
  float* run_var;
  float* part;        // [gx][2C] partial sums
  float* coef;        // fwd [C][2] (scale, shift); bwd [C][3] (A, D, B): dx = A g + D x + B
  float* dgamma;
  float* dbeta;
  int64_t* num_batches;
  int Npix, C, relu, gx, acc_params;
  const float* fcoef;  // bwd, ReLU without residual: the forward's [C][2] (scale, shift); the mask
                       // is then (x * scale + shift > 0) and y is not read (one tensor less)
  uint8_t* mask;       // ReLU mask bits [Npix * C / 8] (bit e of byte i: element e of vector i > 0):
                       // written by the forward apply, read by the backward instead of y
  const float* kshift;  // fwd, partials precomputed by the conv epilogue: their per-channel shift
  int pre;              // fwd: part already holds gx partial rows (no statistics pass)
  int wt;               // apply passes: outputs stored write-through (g_bn_wt)
  float momentum, eps;
};

template <bool BWD>
__global__ __launch_bounds__(kBnT) void bn_nhwc_partial_k(BnNArgs a) {
  const int V = a.C >> 3;
  const int vv = V >= kBnT ? kBnT : V;
  const int ppi = kBnT / vv;
  const int vbase = (V >= kBnT) ? blockIdx.y * kBnT : 0;
  const int v = vbase + threadIdx.x % vv, pr = threadIdx.x / vv;
  float s1[8], s2[8], K[8], mc[16];
#pragma unroll
  for (int e = 0; e < 8; ++e) s1[e] = s2[e] = 0.f;
  if (!BWD) {
    unpack8(*reinterpret_cast<const uint4*>(a.x + 8 * v), K);
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) K[e] = a.mean[8 * v + e];
    if (a.fcoef) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 q = reinterpret_cast<const float4*>(a.fcoef + 16 * v)[j];
        mc[4 * j] = q.x; mc[4 * j + 1] = q.y; mc[4 * j + 2] = q.z; mc[4 * j + 3] = q.w;
      }
    }
  }
  const bool ymask = BWD && a.relu && !a.fcoef && !a.mask;
  const bool bmask = BWD && a.relu && !a.fcoef && a.mask;
  // UNR pixel rows per iteration with all their loads issued before any use: one 16-byte load
  // in flight per thread cannot cover HBM latency with ~256 blocks
  constexpr int UNR = BWD ? 2 : 4;
  const int pstep = gridDim.x * ppi;
  struct Buf {
    uint4 x[UNR], g[UNR], y[UNR];
    uint32_t m[UNR];
  };
  // loads at clamped rows issued unconditionally (the rows past Npix are skipped below): a
  // per-lane `ok ? load : 0` would branch around each load and drain with a vmcnt(0) per row
  auto load = [&](int p0, Buf& b) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int p = min(p0 + u * pstep, a.Npix - 1);
      const size_t o = (size_t)p * a.C + 8 * v;
      b.x[u] = *reinterpret_cast<const uint4*>(a.x + o);
      if (BWD) {
        b.g[u] = *reinterpret_cast<const uint4*>(a.dy + o);
        if (ymask) b.y[u] = *reinterpret_cast<const uint4*>(a.y + o);
        if (bmask) b.m[u] = a.mask[o >> 3];
      }
    }
  };
  auto accumulate = [&](int p0, const Buf& b) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      if (p0 + u * pstep >= a.Npix) break;
      const uint4* xr = b.x;
      const uint4* gr = b.g;
      const uint4* yr = b.y;
      const uint32_t* mb = b.m;
      float xv[8];
      unpack8(xr[u], xv);
      if (!BWD) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = xv[e] - K[e];
          s1[e] += d;
          s2[e] = fmaf(d, d, s2[e]);
        }
      } else {
        float g[8];
        unpack8(gr[u], g);
        if (bmask) {
#pragma unroll
          for (int e = 0; e < 8; ++e) g[e] = (mb[u] >> e) & 1u ? g[e] : 0.f;
        } else if (ymask) {
          float yv[8];
          unpack8(yr[u], yv);
#pragma unroll
          for (int e = 0; e < 8; ++e) g[e] = yv[e] > 0.f ? g[e] : 0.f;
        } else if (a.relu) {  // the forward's exact fp32 pre-activation (same fmaf, same operands)
#pragma unroll
          for (int e = 0; e < 8; ++e) g[e] = fmaf(xv[e], mc[2 * e], mc[2 * e + 1]) > 0.f ? g[e] : 0.f;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          s1[e] += g[e];
          s2[e] = fmaf(g[e], xv[e] - K[e], s2[e]);
        }
      }
    }
  };
  // the next rows' loads are in flight while this iteration's are summed (ping-pong buffers);
  // unpipelined, every iteration paid a full load round trip (2.4 TB/s, profiles/r4_pmc)
  Buf ba, bb;
  int p0 = blockIdx.x * ppi + pr;
  if (p0 < a.Npix) load(p0, ba);
  while (p0 < a.Npix) {
    const int p1 = p0 + UNR * pstep;
    load(p1, bb);
    accumulate(p0, ba);
    if (p1 >= a.Npix) break;
    const int p2 = p1 + UNR * pstep;
    load(p2, ba);
    accumulate(p1, bb);
    p0 = p2;
  }
  // planar [16][kBnT] (thread-fastest): a thread-major [kBnT][16] layout put 16 threads on one
  // bank for every store and read (counters: 3.5x more conflict than LDS-active cycles)
  __shared__ float red[16 * kBnT];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[e * kBnT + threadIdx.x] = s1[e];
    red[(8 + e) * kBnT + threadIdx.x] = s2[e];
  }
  __syncthreads();
  if (pr == 0) {
    for (int k = 1; k < ppi; ++k) {
      const int o = threadIdx.x + k * vv;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s1[e] += red[e * kBnT + o];
        s2[e] += red[(8 + e) * kBnT + o];
      }
    }
    float* dst = a.part + (size_t)blockIdx.x * 2 * a.C + 16 * v;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      dst[2 * e] = s1[e];
      dst[2 * e + 1] = s2[e];
    }
  }
}

template <bool BWD>
__global__ __launch_bounds__(1024) void bn_nhwc_finalize_k(BnNArgs a) {
  // block = 8 channels as 4 pairs (one 16-byte (s1, s2, s1', s2') load per thread per row) x 256
  // row groups: each thread sums <= 16 rows per pass of 4,096 with every load issued up front (one
  // memory round trip per pass; the 128-pixel conv tiles give a batch-256 56 x 56 layer 6,272
  // rows: 2 passes, 4 with the former 8-byte / 128-group layout), the 256 group sums are
  // combined in a fixed order (deterministic): lane shuffles, then one LDS step.  The per-channel inputs of the
  // finalize (gamma, beta, running stats, x[0][c]) are loaded by 8 owner threads before the
  // reduction so their latency overlaps it.
  constexpr int RG = 256, MAXR = 16, NW = 1024 / 64;
  __shared__ float red[NW][4][4];
  const int cp = threadIdx.x & 3, rg = threadIdx.x >> 2, c2 = blockIdx.x * 8 + 2 * cp;
  const bool pok = c2 + 1 < a.C;  // C % 8 == 0 (checked on the host): always true
  const size_t pitch = 2 * (size_t)a.C;
  float s1a = 0.f, s2a = 0.f, s1b = 0.f, s2b = 0.f;
  for (int base = 0; pok && base < a.gx; base += RG * MAXR) {
    float4 t[MAXR];
#pragma unroll
    for (int u = 0; u < MAXR; ++u) {
      const int b = base + rg + RG * u;
      const bool ok = b < a.gx;
      const float4 v = *reinterpret_cast<const float4*>(a.part + (size_t)(ok ? b : 0) * pitch + 2 * c2);
      t[u] = ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < MAXR; ++u) {
      s1a += t[u].x;
      s2a += t[u].y;
      s1b += t[u].z;
      s2b += t[u].w;
    }
  }
  // per-channel inputs of the finalize (threads 0..7 own channels blockIdx.x * 8 + tid), fetched
  // while the reduction runs
  const int cl = threadIdx.x, c = blockIdx.x * 8 + cl;
  const bool own = cl < 8 && c < a.C;
  float gm = 1.f, bt = 0.f, rm = 0.f, rv = 0.f, K0 = 0.f, mu = 0.f, inv = 0.f, dg0 = 0.f, db0 = 0.f;
  if (own) {
    gm = a.gamma ? a.gamma[c] : 1.f;
    if (!BWD) {
      bt = a.beta ? a.beta[c] : 0.f;
      rm = a.run_mean ? a.run_mean[c] : 0.f;
      rv = a.run_var ? a.run_var[c] : 0.f;
      K0 = a.pre ? (a.kshift ? a.kshift[c] : 0.f) : bf2f(a.x[c]);
    } else {
      mu = a.mean[c];
      inv = a.invstd[c];
      if (a.acc_params) {
        dg0 = a.dgamma ? a.dgamma[c] : 0.f;
        db0 = a.dbeta ? a.dbeta[c] : 0.f;
      }
    }
  }
  // the 16 row groups of a wave are combined with lane shuffles (xor 4..32 keeps cp), then the 16
  // wave sums through LDS behind ONE barrier (the former 8-level LDS tree paid 9 barriers)
#pragma unroll
  for (int m = 4; m < 64; m <<= 1) {
    s1a += __shfl_xor(s1a, m);
    s2a += __shfl_xor(s2a, m);
    s1b += __shfl_xor(s1b, m);
    s2b += __shfl_xor(s2b, m);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane < 4) {
    red[wv][lane][0] = s1a;
    red[wv][lane][1] = s2a;
    red[wv][lane][2] = s1b;
    red[wv][lane][3] = s2b;
  }
  __syncthreads();
  if (!own) return;
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int w = 0; w < NW; ++w) {  // fixed order: deterministic
    s1 += red[w][cl >> 1][2 * (cl & 1)];
    s2 += red[w][cl >> 1][2 * (cl & 1) + 1];
  }
  const float cnt = (float)a.Npix;
  if (!BWD) {
    if (a.num_batches && c == 0) *a.num_batches += 1;
    const float m1 = s1 / cnt;
    const float var = fmaxf(s2 / cnt - m1 * m1, 0.f);
    const float mean = K0 + m1, iv = rsqrtf(var + a.eps);
    a.mean[c] = mean;
    a.invstd[c] = iv;
    if (a.run_mean) a.run_mean[c] = (1.f - a.momentum) * rm + a.momentum * mean;
    if (a.run_var) a.run_var[c] = (1.f - a.momentum) * rv + a.momentum * var * cnt / fmaxf(cnt - 1.f, 1.f);
    const float sc = iv * gm;
    a.coef[2 * c] = sc;
    a.coef[2 * c + 1] = bt - mean * sc;
  } else {
    const float db = s1, dg = s2 * inv;
    if (a.dgamma) a.dgamma[c] = dg0 + dg;
    if (a.dbeta) a.dbeta[c] = db0 + db;
    // dx = k (cnt g - db - (x - mu) inv dg), k = gamma inv / cnt
    const float k = gm * inv / cnt;
    a.coef[3 * c] = k * cnt;
    a.coef[3 * c + 1] = -k * inv * dg;
    a.coef[3 * c + 2] = -k * db + k * inv * dg * mu;
  }
}

// forward apply: y = relu?(x * scale + shift (+ res)).  32-bit indices (checked on the host),
// U vectors per iteration with their loads issued first (g_bn_unroll).  The grid stride is a multiple of
// 256 and V = C / 8 divides 256 for every channel count up to 2048, so a thread's channel vector
// v never changes: its 16 coefficients are loaded once into registers (the LDS copy indexed per
// element cost 16-way bank conflicts: 9x more conflict than LDS-active cycles).
// PIPE: the next iteration's loads are issued before this iteration's stores, into the other
// of two register buffers.  Without it the loop head waited (vmcnt) for the previous
// iteration's stores to be acknowledged before issuing its loads -- the loaded registers were the
// stores' data registers -- so every iteration paid a store round trip plus a load round trip
// (the apply kernels streamed at ~3.4 TB/s, profiles/r4_pmc/pmc_rn.txt).
template <int U, bool PIPE>
__global__ __launch_bounds__(kBnT) void bn_nhwc_apply_k(BnNArgs a, FastDiv fV) {
  const int V = a.C >> 3;
  const int total = a.Npix * V, step = gridDim.x * kBnT;
  const uint4 z = make_uint4(0u, 0u, 0u, 0u);
  const int i00 = blockIdx.x * kBnT + threadIdx.x;
  const int v = i00 - (int)fV.div((uint32_t)i00) * V;  // fixed for this thread (step % V == 0)
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float4 q = reinterpret_cast<const float4*>(a.coef + 16 * v)[j];
    sc[2 * j] = q.x;
    sh[2 * j] = q.y;
    sc[2 * j + 1] = q.z;
    sh[2 * j + 1] = q.w;
  }
  // loads at clamped indices, issued unconditionally (a per-lane `i < total ? load : 0` makes
  // hipcc branch around each load and split it into dwords with a vmcnt(0) per element); only
  // the stores are masked
  const uint4* x4 = reinterpret_cast<const uint4*>(a.x);
  const uint4* r4 = reinterpret_cast<const uint4*>(a.res);
  auto load = [&](int i0, uint4 (&xr)[U], uint4 (&rr)[U]) {
    int ic[U];
#pragma unroll
    for (int u = 0; u < U; ++u) ic[u] = min(i0 + u * step, total - 1);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      xr[u] = x4[ic[u]];
      rr[u] = z;
    }
    if (r4) {
#pragma unroll
      for (int u = 0; u < U; ++u) rr[u] = r4[ic[u]];
    }
  };
  auto apply = [&](int i0, const uint4 (&xr)[U], const uint4 (&rr)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * step;
      if (i >= total) break;
      float xv[8], rv[8];
      unpack8(xr[u], xv);
      if (a.res) unpack8(rr[u], rv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float o = fmaf(xv[e], sc[e], sh[e]);
        if (a.res) o += rv[e];
        xv[e] = a.relu ? fmaxf(o, 0.f) : o;
      }
      const uint4 yo = pack8(xv);
      st16(reinterpret_cast<uint4*>(a.y) + i, yo, a.wt);
      if (a.mask) a.mask[i] = (uint8_t)pos_bits8(yo);
    }
  };
  if constexpr (!PIPE) {
    for (int i0 = i00; i0 < total; i0 += U * step) {
      uint4 xr[U], rr[U];
      load(i0, xr, rr);
      apply(i0, xr, rr);
    }
  } else {
    // ping-pong: (xa, ra) hold iteration i0, (xb, rb) the next one; the prefetch past the end
    // re-reads the last valid vectors (clamped) and is not used
    uint4 xa[U], ra[U], xb[U], rb[U];
    int i0 = i00;
    if (i0 < total) load(i0, xa, ra);
    while (i0 < total) {
      const int i1 = i0 + U * step;
      load(i1, xb, rb);
      apply(i0, xa, ra);
      if (i1 >= total) break;
      const int i2 = i1 + U * step;
      load(i2, xa, ra);
      apply(i1, xb, rb);
      i0 = i2;
    }
  }
}

// backward apply: dx = A g + D x + B; dres = g (the residual branch gradient).  XM: the ReLU mask
// from x and the forward's (scale, shift) (no residual), else from y.  Coefficients in registers
// as in the forward apply (fixed channel vector per thread).
template <bool XM, int U, bool PIPE>
__global__ __launch_bounds__(kBnT) void bn_nhwc_bwd_apply_k(BnNArgs a, FastDiv fV) {
  const int V = a.C >> 3;
  const int total = a.Npix * V, step = gridDim.x * kBnT;
  const uint4 z = make_uint4(0u, 0u, 0u, 0u);
  const int i00 = blockIdx.x * kBnT + threadIdx.x;
  const int v = i00 - (int)fV.div((uint32_t)i00) * V;
  float kc[24], mc[16];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const float4 q = reinterpret_cast<const float4*>(a.coef + 24 * v)[j];
    kc[4 * j] = q.x;
    kc[4 * j + 1] = q.y;
    kc[4 * j + 2] = q.z;
    kc[4 * j + 3] = q.w;
  }
  if (XM) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float4 q = reinterpret_cast<const float4*>(a.fcoef + 16 * v)[j];
      mc[4 * j] = q.x;
      mc[4 * j + 1] = q.y;
      mc[4 * j + 2] = q.z;
      mc[4 * j + 3] = q.w;
    }
  }
  const bool bmask = !XM && a.relu && a.mask;
  const bool ymask = !XM && a.relu && !a.mask;
  // clamped, unconditional loads (see bn_nhwc_apply_k); the mask source is a uniform branch
  const uint4 *g4 = reinterpret_cast<const uint4*>(a.dy), *x4 = reinterpret_cast<const uint4*>(a.x),
              *y4 = reinterpret_cast<const uint4*>(a.y);
  struct Buf {
    uint4 g[U], x[U], y[U];
    uint32_t m[U];
  };
  auto load = [&](int i0, Buf& b) {
    int ic[U];
#pragma unroll
    for (int u = 0; u < U; ++u) ic[u] = min(i0 + u * step, total - 1);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      b.g[u] = g4[ic[u]];
      b.x[u] = x4[ic[u]];
      b.y[u] = z;
      b.m[u] = 0u;
    }
    if (bmask) {
#pragma unroll
      for (int u = 0; u < U; ++u) b.m[u] = a.mask[ic[u]];
    } else if (ymask) {
#pragma unroll
      for (int u = 0; u < U; ++u) b.y[u] = y4[ic[u]];
    }
  };
  auto apply = [&](int i0, const Buf& b) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * step;
      if (i >= total) break;
      float g[8], xv[8];
      unpack8(b.g[u], g);
      unpack8(b.x[u], xv);
      if (XM) {
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = fmaf(xv[e], mc[2 * e], mc[2 * e + 1]) > 0.f ? g[e] : 0.f;
      } else if (bmask) {
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = (b.m[u] >> e) & 1u ? g[e] : 0.f;
      } else if (a.relu) {
        float yv[8];
        unpack8(b.y[u], yv);
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = yv[e] > 0.f ? g[e] : 0.f;
      }
      if (a.dres) st16(reinterpret_cast<uint4*>(a.dres) + i, pack8(g), a.wt);
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = fmaf(kc[3 * e], g[e], fmaf(kc[3 * e + 1], xv[e], kc[3 * e + 2]));
      st16(reinterpret_cast<uint4*>(a.dx) + i, pack8(o), a.wt);
    }
  };
  if constexpr (!PIPE) {
    for (int i0 = i00; i0 < total; i0 += U * step) {
      Buf b;
      load(i0, b);
      apply(i0, b);
    }
  } else {  // ping-pong as in bn_nhwc_apply_k
    Buf ba, bb;
    int i0 = i00;
    if (i0 < total) load(i0, ba);
    while (i0 < total) {
      const int i1 = i0 + U * step;
      load(i1, bb);
      apply(i0, ba);
      if (i1 >= total) break;
      const int i2 = i1 + U * step;
      load(i2, ba);
      apply(i1, bb);
      i0 = i2;
    }
  }
}

// ------------------------------------------------------------------------------------------
// max pool (k x k, stride, pad) with uint8 argmax tap; backward gathers over covering windows.
// 32-bit indices through FastDiv (sizes checked on the host), the 8 taps of a channel vector
// loaded / stored as one 8-byte word, and the window loops unrolled for the ResNet stem pool
// (KS = 3; KS = 0: runtime k).
template <int KS>
__global__ void maxpool_nhwc_k(const bf16* __restrict__ x, bf16* __restrict__ y, uint8_t* __restrict__ arg, int N,
                               int H, int W, int C, int P, int Q, int kr, int st, int pd, FastDiv fV, FastDiv fQ,
                               FastDiv fP) {
  const int k = KS ? KS : kr;
  const int V = C >> 3;
  const int total = N * P * Q * V;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int pix = (int)fV.div((uint32_t)i), v = i - pix * V;
    const int pq = (int)fQ.div((uint32_t)pix), q = pix - pq * Q;
    const int n = (int)fP.div((uint32_t)pq), p = pq - n * P;
    float best[8];
    uint32_t b0 = 0, b1 = 0;  // argmax taps, 4 per word
#pragma unroll
    for (int e = 0; e < 8; ++e) best[e] = -INFINITY;
#pragma unroll
    for (int r = 0; r < (KS ? KS : 1); ++r) {
      for (int rr = (KS ? r : 0); rr < (KS ? r + 1 : k); ++rr) {
#pragma unroll
        for (int s = 0; s < (KS ? KS : 1); ++s) {
          for (int ss = (KS ? s : 0); ss < (KS ? s + 1 : k); ++ss) {
            const int h = p * st - pd + rr, w = q * st - pd + ss;
            if ((unsigned)h >= (unsigned)H || (unsigned)w >= (unsigned)W) continue;
            float xv[8];
            unpack8(*reinterpret_cast<const uint4*>(x + ((size_t)(n * H + h) * W + w) * C + 8 * v), xv);
            const uint32_t tap = (uint32_t)(rr * k + ss);
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (xv[e] > best[e]) {
                best[e] = xv[e];
                if (e < 4) b0 = (b0 & ~(0xffu << (8 * e))) | (tap << (8 * e));
                else b1 = (b1 & ~(0xffu << (8 * (e - 4)))) | (tap << (8 * (e - 4)));
              }
          }
        }
      }
    }
    reinterpret_cast<uint4*>(y)[i] = pack8(best);
    reinterpret_cast<uint2*>(arg)[i] = make_uint2(b0, b1);
  }
}

// 3x3 / stride 2 / pad 1 (ResNet's stem pool): input row h is covered by window row h / 2 (tap 1)
// when h is even, by rows (h + 1) / 2 (tap 0) and (h - 1) / 2 (tap 2) when odd; the same for
// columns.  All four candidate windows' (dy, argmax) loads are issued unconditionally (clamped
// indices, validity as a mask) -- the generic kernel's loads sat behind data-dependent branches,
// one round trip each (250 us per step at batch 256).
__global__ void maxpool_nhwc_bwd_s2_k(const bf16* __restrict__ dy, const uint8_t* __restrict__ arg,
                                      bf16* __restrict__ dx, int N, int H, int W, int C, int P, int Q, FastDiv fV,
                                      FastDiv fW, FastDiv fH) {
  const int V = C >> 3;
  const int total = N * H * W * V;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int pix = (int)fV.div((uint32_t)i), v = i - pix * V;
    const int hw = (int)fW.div((uint32_t)pix), w = pix - hw * W;
    const int n = (int)fH.div((uint32_t)hw), h = hw - n * H;
    int pr[2], tr[2], qc[2], tc[2];
    bool okr[2], okc[2];
    if (h & 1) {
      pr[0] = (h + 1) >> 1; tr[0] = 0; okr[0] = pr[0] < P;
      pr[1] = (h - 1) >> 1; tr[1] = 2; okr[1] = true;
    } else {
      pr[0] = h >> 1; tr[0] = 1; okr[0] = pr[0] < P;
      pr[1] = 0; tr[1] = 0; okr[1] = false;
    }
    if (w & 1) {
      qc[0] = (w + 1) >> 1; tc[0] = 0; okc[0] = qc[0] < Q;
      qc[1] = (w - 1) >> 1; tc[1] = 2; okc[1] = true;
    } else {
      qc[0] = w >> 1; tc[0] = 1; okc[0] = qc[0] < Q;
      qc[1] = 0; tc[1] = 0; okc[1] = false;
    }
    uint4 d4[4];
    uint2 a4[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int a = c >> 1, b = c & 1;
      const int o = ((n * P + min(pr[a], P - 1)) * Q + min(qc[b], Q - 1)) * V + v;
      d4[c] = reinterpret_cast<const uint4*>(dy)[o];
      a4[c] = reinterpret_cast<const uint2*>(arg)[o];
    }
    float g[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int a = c >> 1, b = c & 1;
      const bool ok = okr[a] && okc[b];
      const uint32_t tap = (uint32_t)(tr[a] * 3 + tc[b]);
      float dv[8];
      unpack8(d4[c], dv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t t = ((e < 4 ? a4[c].x : a4[c].y) >> (8 * (e & 3))) & 0xffu;
        g[e] += (ok && t == tap) ? dv[e] : 0.f;
      }
    }
    reinterpret_cast<uint4*>(dx)[i] = pack8(g);
  }
}

template <int KS>
__global__ void maxpool_nhwc_bwd_k(const bf16* __restrict__ dy, const uint8_t* __restrict__ arg, bf16* __restrict__ dx,
                                   int N, int H, int W, int C, int P, int Q, int kr, int st, int pd, FastDiv fV,
                                   FastDiv fW, FastDiv fH, FastDiv fS) {
  const int k = KS ? KS : kr;
  const int V = C >> 3;
  const int total = N * H * W * V;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int pix = (int)fV.div((uint32_t)i), v = i - pix * V;
    const int hw = (int)fW.div((uint32_t)pix), w = pix - hw * W;
    const int n = (int)fH.div((uint32_t)hw), h = hw - n * H;
    float g[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] = 0.f;
#pragma unroll
    for (int r = 0; r < (KS ? KS : 1); ++r) {
      for (int rr = (KS ? r : 0); rr < (KS ? r + 1 : k); ++rr) {
        const int tp = h + pd - rr;
        if (tp < 0) continue;
        const int p = (int)fS.div((uint32_t)tp);
        if (p * st != tp || p >= P) continue;
#pragma unroll
        for (int s = 0; s < (KS ? KS : 1); ++s) {
          for (int ss = (KS ? s : 0); ss < (KS ? s + 1 : k); ++ss) {
            const int tq = w + pd - ss;
            if (tq < 0) continue;
            const int q = (int)fS.div((uint32_t)tq);
            if (q * st != tq || q >= Q) continue;
            const int o = ((n * P + p) * Q + q) * V + v;
            float dv[8];
            unpack8(reinterpret_cast<const uint4*>(dy)[o], dv);
            const uint2 a2 = reinterpret_cast<const uint2*>(arg)[o];
            const uint32_t tap = (uint32_t)(rr * k + ss);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const uint32_t t = ((e < 4 ? a2.x : a2.y) >> (8 * (e & 3))) & 0xffu;
              if (t == tap) g[e] += dv[e];
            }
          }
        }
      }
    }
    reinterpret_cast<uint4*>(dx)[i] = pack8(g);
  }
}

// global average pool: bf16 [N][HW][C] -> fp32 [N][C]; backward broadcasts dy / HW
__global__ void gap_nhwc_k(const bf16* __restrict__ x, float* __restrict__ y, int N, int HW, int C) {
  const int n = blockIdx.y;
  for (int c = blockIdx.x * 256 + threadIdx.x; c < C; c += gridDim.x * 256) {
    float s = 0.f;
    for (int p = 0; p < HW; ++p) s += bf2f(x[((size_t)n * HW + p) * C + c]);
    y[(size_t)n * C + c] = s / (float)HW;
  }
}

__global__ void gap_nhwc_bwd_k(const float* __restrict__ dy, bf16* __restrict__ dx, int N, int HW, int C) {
  const int64_t total = (int64_t)N * HW * C;
  const float inv = 1.f / (float)HW;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % C);
    const int n = (int)(i / ((int64_t)HW * C));
    dx[i] = f2bf(dy[(size_t)n * C + c] * inv);
  }
}

int grid_for(int64_t n, int cap = 4096) {
  const int64_t g = (n + 255) / 256;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}

// grid of a streaming grid-stride kernel over n items (256-thread blocks): ~6 items per thread,
// at least 2,048 blocks (or one item per thread), at most `cap`.  Measured on the BN apply kernels
// (scripts/bench_bn.py, profiles/r4_j..l): 2,048-block grids capped a 411 MB stream at 4.8 TB/s,
// 8-32 k blocks reach 5.6-5.9; a flat 65,536 made the mid-sized layers dispatch-bound.
static int g_stream_cap = 32768;
static int stream_blocks(int64_t n) {
  const int64_t nb = std::max<int64_t>((n + 256 * 6 - 1) / (256 * 6), std::min<int64_t>(2048, (n + 255) / 256));
  return (int)std::max<int64_t>(1, std::min<int64_t>(nb, g_stream_cap));
}

}  // namespace

// ------------------------------------------------------------------------------------------
void nhwc_from_nchw(const float* x, uint16_t* y, int N, int C, int H, int W, int Cp, hipStream_t st) {
  MX_CHECK(Cp % 8 == 0 && C <= Cp && (int64_t)N * H * W * Cp / 8 < (1ll << 31), "nhwc_from_nchw: Cp % 8, 32-bit indices");
  const int G = Cp / 8;
  MX_LAUNCH(nchw_to_nhwc_k, dim3(grid_for((int64_t)N * H * W * G)), dim3(256), 0, st, x, reinterpret_cast<uint4*>(y), N,
            C, H * W, G, FastDiv(G), FastDiv(H * W));
}

void nhwc_repack_weight(const float* w, uint16_t* wt, uint16_t* wtd, int K, int C, int R, int S, int Cp,
                        hipStream_t st) {
  const int64_t total = (wt ? (int64_t)K * Cp * R * S : 0) + (wtd ? (int64_t)K * C * R * S : 0);
  MX_LAUNCH(wrepack_k, dim3(grid_for(total)), dim3(256), 0, st, w, wt, wtd, K, C, R, S, Cp);
}

int nhwc_repack_blocks(int K, int C, int R, int S, int Cp, bool fwd, bool dgrad) {
  const int64_t nf = fwd ? (int64_t)K * R * S * Cp : 0, nd = dgrad ? (int64_t)K * C * R * S : 0;
  MX_CHECK(nf + nd < (1ll << 31), "nhwc repack: weight too large for 32-bit indices");
  if (K % 8 == 0)  // forward blocks, then the data-gradient transpose tiles (wrepack_many_k)
    return std::max(1, (fwd ? repack_fwd_blocks(K, Cp, R * S) : 0) +
                           (dgrad ? cdiv(K, kRepackT) * cdiv(C * R * S, kRepackT) : 0));
  return std::max(1, (int)((nf + nd + kRepackPerBlock - 1) / kRepackPerBlock));
}

void nhwc_repack_many(const int64_t* desc, int n, int total_blocks, hipStream_t st) {
  if (n <= 0) return;
  MX_LAUNCH(wrepack_many_k, dim3(total_blocks), dim3(256), 0, st, desc, n);
}

struct ConvPlan {
  int tm, tn, blocks, splits, kt_per_split;
};

// largest tile whose grid still gives every CU two blocks (layer3/4 of ResNet-50 have only
// 1.5k-6k output pixels at batch 32): 128 x 128, then 64 x 128, then 64 x 64; when even 64 x 64
// leaves the chip under-filled, split the reduction (k-tiles) over blockIdx.y with fp32
// partials (>= 8 k-tiles per split)
// split-K only below this many blocks (A/B: nhwc_conv_set_split_blocks; each split adds a reduce
// launch, ~5-6 us at batch 32).  ResNet-50 (profiles/r4_w/, two runs each): batch 32 5,368 / 5,370
// img/s at 512, 5,400 / 5,405 at 256, 5,399 / 5,410 at 384, 5,390 / 5,387 at 128; batch 256 equal
static int g_split_blocks = 256;
void nhwc_conv_set_split_blocks(int n) { g_split_blocks = n; }
static ConvPlan conv_plan(int M, int Ng, int Kg) {
  ConvPlan p{};
  const int b128 = cdiv(Ng, 128) * cdiv(M, 128), b64 = cdiv(Ng, 64) * cdiv(M, 128);
  if (Ng > 64 && b128 >= 512) {
    p.tm = 128; p.tn = 128; p.blocks = b128;
  } else if (b64 >= 512 || (Ng <= 64 && M >= 128 * 256)) {
    p.tm = 64; p.tn = 128; p.blocks = b64;
  } else {
    p.tm = 64; p.tn = 64; p.blocks = cdiv(Ng, 64) * cdiv(M, 64);
  }
  const int nkt = cdiv(Kg, 64);
  p.splits = 1;
  if (p.blocks < g_split_blocks) p.splits = std::max(1, std::min(cdiv(512, p.blocks), nkt / 8));
  p.kt_per_split = cdiv(nkt, p.splits);
  p.splits = cdiv(nkt, p.kt_per_split);
  return p;
}

// kernel variant, parity mode and tile plan of one convolution (shared by the launch and the
// scratch-size queries, so the caller's split-K buffer always matches the launch)
struct ConvSetup {
  ConvPlan p;
  bool wide, par;
};

static ConvSetup conv_setup(const ConvNArgs& a) {
  ConvSetup c{};
  // wide path: whole 64-k stages inside one tap, and every byte offset fits 32 bits
  c.wide = a.Ca % 64 == 0 && a.Kg % 64 == 0 &&
           (int64_t)a.IH * a.IW * a.Ca * (a.M / (a.OH * a.OW) + 1) < (1ll << 30) &&
           (int64_t)a.Ng * a.Kg < (1ll << 30);
  c.par = c.wide && a.dgrad && a.sh == 2 && a.sw == 2 && a.OH % 2 == 0 && a.OW % 2 == 0;
  // parity classes: a quarter of the pixels each, at most ceil(R/2) x ceil(S/2) taps
  c.p = c.par ? conv_plan(a.M / 4, a.Ng, ((a.R + 1) / 2) * ((a.S + 1) / 2) * a.Ca) : conv_plan(a.M, a.Ng, a.Kg);
  return c;
}


// LDS-DMA kernel selection: 0 = never, 1 = large layers (default), 2 = wherever eligible (tests)
static int g_conv_glds = -1;
void nhwc_conv_set_glds(int mode) { g_conv_glds = mode; }
static int conv_glds_mode() {
  if (g_conv_glds < 0) {
    g_conv_glds = 1;  // nhwc_conv_set_glds() overrides (tests, A/B runs)
  }
  return g_conv_glds;
}

// the LDS-DMA kernel: wide path, forward or stride-1 data gradient, and (mode 1) enough
// 256-pixel tiles for ~3/4 of the CUs
struct GldsPlan {
  int tm, splits, kt_per_split;  // tm == 0: not used
};

static GldsPlan glds_plan_mnk(int M, int Ng, int Kg) {
  GldsPlan g{};
  g.tm = Ng >= 128 ? 128 : 64;
  const int tiles = cdiv(Ng, g.tm) * cdiv(M, 256);
  const int nkt = Kg / 64;
  // split the reduction (>= 8 k-tiles per split) until ~one block per CU
  g.splits = std::max(1, std::min(cdiv(256, tiles), nkt / 8));
  g.kt_per_split = cdiv(nkt, g.splits);
  g.splits = cdiv(nkt, g.kt_per_split);
  // measured per layer at batch 32 / 64 (scripts/gpu_glds_sweep.sh, bench_nhwc_layers.py): a
  // win from ~200 blocks up (0.75 of the 256 CUs), a loss at <= 112; with split-K a win only when
  // the layer has few tiles (<= 50: long per-split reductions), a loss at ~100 tiles x 2 splits
  if (conv_glds_mode() == 1 && (tiles * g.splits < 192 || (g.splits > 1 && tiles > 64))) g.tm = 0;
  return g;
}

// the LDS-DMA kernel: wide path, forward or stride-1 data gradient
static GldsPlan glds_plan(const ConvNArgs& a, bool wide, bool par) {
  if (conv_glds_mode() == 0 || !wide || par || (a.dgrad && (a.sh != 1 || a.sw != 1))) return GldsPlan{};
  return glds_plan_mnk(a.M, a.Ng, a.Kg);
}

// the 256 x 256 tile (conv_nhwc_glds256_kernel): 0 = never, 1 = where it fills the chip with a
// reduction of >= 4 k-tiles (default), 2 = wherever Ng % 256 == 0 (tests)
static int g_conv_glds256 = 1;
// the two-stage 128-pixel variant of the LDS-DMA kernel (conv_nhwc_glds_kernel<TM, STATS, 128, 2>)
// for layers of <= 2 k-tiles with >= 512 tiles: 0 = never, 1 = there (default)
static int g_conv_glds_short = 1;
void nhwc_conv_set_glds_short(int mode) { g_conv_glds_short = mode; }
// 128 x 128 tiles of the two-stage LDS-DMA variant (two blocks per CU, the whole reduction per
// block) for reductions of >= 4 k-tiles.  Measured per layer (profiles/r5_deep/): on the layers
// whose 256-pixel tiles under-fill the chip (the 7 x 7 stage at batch 256: 4 x 49 tiles) they
// replace split-K / the generic kernel (3x3 512 -> 512 150 -> 66 us); with >= ~200 such tiles they
// also beat the three-stage 256-pixel and the 256 x 256 tiles on most layers (28 x 28 3x3 97 -> 72
// us, 14 x 14 1024 -> 256 data gradient 58 -> 43 us), and lose below ~100 tiles (batch 32's
// 7 x 7 stage: 24 -> 47 us at 52 tiles).  0 = never, 1 = >= 192 tiles (default), 2 = every
// eligible layer, 3 = only where the 256-pixel tiles would under-fill the chip (the first rule)
static int g_conv_glds_deep = 1;
void nhwc_conv_set_glds_deep(int mode) { g_conv_glds_deep = mode; }
// stride-2 data gradients (parity classes, blockIdx.z) on the same tiles: 1 = on, 0 = the generic
// kernel's parity classes
static int g_conv_glds_par = 1;
void nhwc_conv_set_glds_par(int on) { g_conv_glds_par = on; }
// the two-stage 128 x 128 tiles as conv_nhwc_gk2_kernel (64 x 64 wave tiles, two k-groups): 0 =
// conv_nhwc_glds_kernel<128, *, 128, 2> (8 waves of 64 x 32), 1 = gk2 on 16x16x32 MFMAs, 2 = gk2 on
// 32x32x16 MFMAs
static int g_conv_gk2 = 0;
void nhwc_conv_set_gk2(int mode) { g_conv_gk2 = mode; }
static void launch_tile128(ConvNArgs& a, dim3 grid, bool stats, hipStream_t st) {
  if (g_conv_gk2 == 2) {
    if (stats) MX_LAUNCH((conv_nhwc_gk2_kernel<true, true>), grid, dim3(512), 0, st, a);
    else MX_LAUNCH((conv_nhwc_gk2_kernel<false, true>), grid, dim3(512), 0, st, a);
  } else if (g_conv_gk2 == 1) {
    if (stats) MX_LAUNCH((conv_nhwc_gk2_kernel<true, false>), grid, dim3(512), 0, st, a);
    else MX_LAUNCH((conv_nhwc_gk2_kernel<false, false>), grid, dim3(512), 0, st, a);
  } else {
    if (stats) MX_LAUNCH((conv_nhwc_glds_kernel<128, true, 128, 2>), grid, dim3(512), 0, st, a);
    else MX_LAUNCH((conv_nhwc_glds_kernel<128, false, 128, 2>), grid, dim3(512), 0, st, a);
  }
}
static bool glds_deep_fits(const ConvNArgs& a, bool wide, bool par) {
  if (!g_conv_glds_deep || conv_glds_mode() == 0 || !wide) return false;
  if (a.dgrad && (a.sh != 1 || a.sw != 1) && !(par && g_conv_glds_par)) return false;
  if (a.Kg % 64 != 0 || a.Kg < 256 || a.Ng < 128) return false;
  const int64_t mc = par ? a.M / 4 : a.M, cls = par ? 4 : 1;
  const int64_t t256 = cls * cdiv(a.Ng, 128) * cdiv(mc, 256), t128 = cls * cdiv(a.Ng, 128) * cdiv(mc, 128);
  switch (g_conv_glds_deep) {
    case 2: return true;
    case 3: return t256 < 256 && t128 >= 256;
    default: return t128 >= 192;
  }
}
// The BN apply kernels run U = 2 vectors per iteration, software-pipelined (4 vectors measured
// ~1 % slower, the unpipelined loop equal: profiles/r4_ab2, r4_g).
// blocks of the BN apply kernels (any multiple of 256 threads keeps each thread's channel vector
// fixed): stream_blocks; ResNet-50 9,981 -> 10,218 img/s against the old 2,048-block cap
// (profiles/r4_l/)
static int g_bn_wt = 1;  // ResNet-50 b32 5,682 -> 5,772 img/s with g_conv_wt (profiles/r5_nhwcwt)
void nhwc_bn_set_wt(int on) { g_bn_wt = on; }
void nhwc_bn_set_grid_cap(int cap) {  // cap of stream_blocks (2048 = the round-3 grids)
  MX_CHECK(cap >= 256, "nhwc_bn_set_grid_cap: >= 256");
  g_stream_cap = cap;
}
void nhwc_conv_set_glds256(int mode) { g_conv_glds256 = mode; }
static bool glds256_fits(const ConvNArgs& a) {
  if (g_conv_glds256 == 0 || a.Ng % 256 != 0 || a.Kg % 64 != 0) return false;
  const int64_t tiles = (int64_t)(a.Ng / 256) * cdiv(a.M, 256);
  // mode 1: enough tiles to fill the chip and a reduction of >= 4 k-tiles -- measured per layer at
  // batch 256 (profiles/r4_i/rn_layers_t256.log): a win on every such layer (e.g. 512 -> 2048
  // forward 51.8 -> 43.4 us, 1024 -> 512 84.1 -> 68.4 us), a loss on the 1-2 k-tile layers, which
  // the two-stage 128-pixel variant serves better
  return g_conv_glds256 == 2 || (tiles >= 256 && a.Kg >= 256);
}

size_t nhwc_conv_scratch_floats(int M, int Ng, int Kg) {
  // either kernel may run (the LDS-DMA one needs a wide layer: Kg % 64 == 0 is necessary)
  const ConvPlan p = conv_plan(M, Ng, Kg);
  size_t n = p.splits > 1 ? (size_t)p.splits * M * Ng : 0;
  if (Kg % 64 == 0) {
    const GldsPlan g = glds_plan_mnk(M, Ng, Kg);
    if (g.tm && g.splits > 1) n = std::max(n, (size_t)g.splits * M * Ng);
  }
  return n;
}

// forward BN statistics in the split-K reduce: one row per `bpr` blocks (>= 8 pixels per row,
// <= 2,048 blocks); the channel quads must tile the grid stride (ResNet's power-of-two widths)
static int splitk_bn_bpr(int Ng) { return std::max(1, Ng / 1024); }
static int splitk_bn_rows(int M, int Ng) { return std::min(cdiv(M, 8), 2048 / splitk_bn_bpr(Ng)); }
static bool splitk_bn_ok(int Ng) {
  const int q4 = Ng / 4;
  return Ng % 4 == 0 && q4 > 0 && (q4 <= 256 ? 256 % q4 == 0 : q4 % 256 == 0);
}

// sums the split-K partials into a.out; fpart (forward only): the consuming BN's partial rows are
// written there too.  Returns their count (0: none)
static int launch_splitk_reduce(const ConvNArgs& a, float* scratch, int splits, float* fpart, hipStream_t st) {
  const int64_t n4 = (int64_t)a.M * a.Ng / 4;
  if (fpart && !a.dgrad && !a.addend && splitk_bn_ok(a.Ng)) {
    const int rows = splitk_bn_rows(a.M, a.Ng);
    MX_LAUNCH(conv_nhwc_splitk_reduce_k<true>, dim3(rows * splitk_bn_bpr(a.Ng)), dim3(256), 0, st, scratch, a.out, n4,
              splits, a.addend, a.amask, fpart, a.bnshift, a.Ng, (a.owt >> 2) & 1);
    return rows;
  }
  MX_LAUNCH(conv_nhwc_splitk_reduce_k<false>, dim3(grid_for(n4, 2048)), dim3(256), 0, st, scratch, a.out, n4, splits,
            a.addend, a.amask, nullptr, nullptr, a.Ng, (a.owt >> 2) & 1);
  return 0;
}

// returns the number of BN partial rows the epilogue wrote to a.bnpart (0: none, the BN runs its
// own statistics pass)
// bit 0 the tile kernels' bf16 epilogue: ResNet-50 b256 11,037 -> 11,055 (noise level), with the
// BN stores b32 5,682 -> 5,772 img/s (profiles/r5_nhwcwt/); bit 1 the split-K fp32 partials: b32
// 5,774 -> 5,816, b256 neutral (profiles/r5_splitwt/); bit 2 the split-K reduce's output (neutral, off: b_* logs)
static int g_conv_wt = 3;
void nhwc_conv_set_wt(int on) { g_conv_wt = on; }
static int launch_conv(ConvNArgs& a, float* scratch, hipStream_t st) {
  a.owt = g_conv_wt;
  MX_CHECK(a.Kg % 8 == 0 && a.Ca % 8 == 0 && a.Ng % 8 == 0, "nhwc conv: channels must be multiples of 8");
  a.fOW = FastDiv(a.OW);
  a.fOHW = FastDiv(a.OH * a.OW);
  a.fCa = FastDiv(a.Ca);
  a.fS = FastDiv(a.S);
  // a half-resolution addend is mapped only by the tile epilogue (epi_vectors), not by the
  // split-K reduce (full-resolution indices): no partial buffer, so no plan splits the reduction
  if (a.asub) scratch = nullptr;
  if (c3_eligible(a)) {  // persistent band kernel (forward or data gradient)
    const int rt = c3_band_rows(a.OH, a.OW), nb = a.M / (rt * a.OW);
    // BN rows: one per band (nhwc_conv_bn_rows sized the buffer for them); no backward statistics
    if (!(a.bnpart && !a.dgrad && nb <= 16384)) a.bnpart = nullptr;
    a.bx = nullptr;
    const int blocks = std::min(nb, 256);
    if (a.bnpart) MX_LAUNCH(conv3x3_s1_c64_kernel<true>, dim3(blocks), dim3(512), 0, st, a, rt, nb);
    else MX_LAUNCH(conv3x3_s1_c64_kernel<false>, dim3(blocks), dim3(512), 0, st, a, rt, nb);
    return a.bnpart ? nb : 0;
  }
  if (stem_eligible(a)) {  // 16 x 16 output tiles: M / 256 blocks
    const int gx = a.M / 256;
    if (!(a.bnpart && gx <= 16384)) a.bnpart = nullptr;
    if (a.bnpart) MX_LAUNCH(conv_nhwc_stem_kernel<true>, dim3(gx), dim3(512), 0, st, a);
    else MX_LAUNCH(conv_nhwc_stem_kernel<false>, dim3(gx), dim3(512), 0, st, a);
    return a.bnpart ? gx : 0;
  }
  const ConvSetup cs = conv_setup(a);
  ConvPlan p = cs.p;
  const bool wide = cs.wide;
  const GldsPlan gp = glds_plan(a, wide, cs.par);
  if (glds_deep_fits(a, wide, cs.par)) {  // 128 x 128 tiles, two blocks per CU, no split-K
    const bool par = cs.par;  // stride-2 data gradient: one grid slice per output parity class
    a.par = par ? 1 : 0;
    if (par) {
      a.Hc = a.OH / 2;
      a.Wc = a.OW / 2;
      a.fWc = FastDiv(a.Wc);
      a.fHWc = FastDiv(a.Hc * a.Wc);
    }
    a.part = nullptr;
    a.kt_per_split = a.Kg / 64;  // >= every class's k-tiles
    const int gx = cdiv(par ? a.M / 4 : a.M, 128), rows = (par ? 4 : 1) * gx;
    const bool bst = a.dgrad && a.bx && a.bnpart && rows <= 16384;  // backward BN statistics epilogue
    if (!bst) a.bx = nullptr;
    if (!(a.bnpart && (bst || !a.dgrad) && rows <= 16384)) a.bnpart = nullptr;
    const dim3 grid(cdiv(a.Ng, 128) * gx, 1, par ? 4 : 1);
    launch_tile128(a, grid, a.bnpart && !bst, st);
    return a.bnpart ? rows : 0;
  }
  if (gp.tm && glds256_fits(a)) {  // 256 x 256 tiles, no split-K
    a.par = 0;
    a.part = nullptr;
    const int gx = cdiv(a.M, 256);
    const bool bst = a.dgrad && a.bx && a.bnpart && gx <= 16384;
    if (!bst) a.bx = nullptr;
    if (!(a.bnpart && (bst || !a.dgrad) && gx <= 16384)) a.bnpart = nullptr;
    const dim3 grid((a.Ng / 256) * gx);
    if (a.bnpart && !bst) MX_LAUNCH(conv_nhwc_glds256_kernel<true>, grid, dim3(512), 0, st, a);
    else MX_LAUNCH(conv_nhwc_glds256_kernel<false>, grid, dim3(512), 0, st, a);
    return a.bnpart ? gx : 0;
  }
  if (gp.tm && (gp.splits == 1 || scratch)) {
    a.par = 0;
    a.kt_per_split = gp.kt_per_split;
    a.part = gp.splits > 1 ? scratch : nullptr;
    // short reductions (<= 2 k-tiles) with enough tiles for two blocks per CU: 128-pixel tiles,
    // two stages
    const bool shrt = g_conv_glds_short && gp.splits == 1 && a.Kg <= 128 &&
                      (int64_t)cdiv(a.Ng, gp.tm) * cdiv(a.M, 128) >= 512;
    const int tn = shrt ? 128 : 256, gx = cdiv(a.M, tn);
    // epilogue BN statistics (forward: bnpart / bnshift; data gradient: bx, see ConvNArgs) need
    // the whole reduction in one block: no split-K
    const bool bst = a.dgrad && a.bx && a.bnpart && gp.splits == 1 && gx <= 16384;
    float* const fpart = (!a.dgrad && gp.splits > 1) ? a.bnpart : nullptr;  // statistics in the reduce
    if (!bst) a.bx = nullptr;
    if (!(a.bnpart && (bst || (!a.dgrad && gp.splits == 1)) && gx <= 16384)) a.bnpart = nullptr;
    const dim3 grid(cdiv(a.Ng, gp.tm) * gx, gp.splits);
    if (shrt) {
      if (gp.tm == 128) launch_tile128(a, grid, a.bnpart && !bst, st);
      else if (a.bnpart && !bst) MX_LAUNCH((conv_nhwc_glds_kernel<64, true, 128, 2>), grid, dim3(512), 0, st, a);
      else MX_LAUNCH((conv_nhwc_glds_kernel<64, false, 128, 2>), grid, dim3(512), 0, st, a);
    } else if (a.bnpart && !bst) {
      if (gp.tm == 128) MX_LAUNCH((conv_nhwc_glds_kernel<128, true>), grid, dim3(512), 0, st, a);
      else MX_LAUNCH((conv_nhwc_glds_kernel<64, true>), grid, dim3(512), 0, st, a);
    } else {
      if (gp.tm == 128) MX_LAUNCH((conv_nhwc_glds_kernel<128>), grid, dim3(512), 0, st, a);
      else MX_LAUNCH((conv_nhwc_glds_kernel<64>), grid, dim3(512), 0, st, a);
    }
    if (gp.splits > 1) return launch_splitk_reduce(a, scratch, gp.splits, fpart, st);
    return a.bnpart ? gx : 0;
  }
  a.par = cs.par ? 1 : 0;
  if (cs.par) {
    a.Hc = a.OH / 2;
    a.Wc = a.OW / 2;
    a.fWc = FastDiv(a.Wc);
    a.fHWc = FastDiv(a.Hc * a.Wc);
  }
  if (!scratch) {  // no partial buffer: no split
    p.splits = 1;
    p.kt_per_split = cdiv(a.Kg, 64);
  }
  a.kt_per_split = p.kt_per_split;
  a.part = p.splits > 1 ? scratch : nullptr;
  // backward BN statistics in the epilogue: one partial row per (parity class, pixel tile)
  const int Mc = cs.par ? a.M / 4 : a.M, brows = (cs.par ? 4 : 1) * cdiv(Mc, p.tn);
  const bool bst = a.dgrad && a.bx && a.bnpart && p.splits == 1 && brows <= 16384;
  float* const fpart = (!a.dgrad && p.splits > 1) ? a.bnpart : nullptr;  // statistics in the reduce
  if (!bst) {
    a.bx = nullptr;
    a.bnpart = nullptr;
  }
  const dim3 grid(p.blocks, p.splits, cs.par ? 4 : 1);
  if (p.tm == 128) {
    if (wide) MX_LAUNCH((conv_nhwc_kernel<128, 128, true>), grid, dim3(256), 0, st, a);
    else MX_LAUNCH((conv_nhwc_kernel<128, 128, false>), grid, dim3(256), 0, st, a);
  } else if (p.tn == 128) {
    if (wide) MX_LAUNCH((conv_nhwc_kernel<64, 128, true>), grid, dim3(256), 0, st, a);
    else MX_LAUNCH((conv_nhwc_kernel<64, 128, false>), grid, dim3(256), 0, st, a);
  } else {
    if (wide) MX_LAUNCH((conv_nhwc_kernel<64, 64, true>), grid, dim3(256), 0, st, a);
    else MX_LAUNCH((conv_nhwc_kernel<64, 64, false>), grid, dim3(256), 0, st, a);
  }
  if (p.splits > 1) return launch_splitk_reduce(a, scratch, p.splits, fpart, st);
  return bst ? brows : 0;
}

int nhwc_conv_fwd(const uint16_t* x, const uint16_t* wt, uint16_t* y, int N, int H, int W, int Cp, int K, int R,
                  int S, int sh, int sw, int ph, int pw, int P, int Q, float* scratch, hipStream_t st, float* bnpart,
                  const float* bnshift) {
  ConvNArgs a{};
  a.act = x;
  a.wt = wt;
  a.out = y;
  a.M = N * P * Q;
  a.Ng = K;
  a.Kg = R * S * Cp;
  a.Ca = Cp;
  a.OH = P;
  a.OW = Q;
  a.IH = H;
  a.IW = W;
  a.R = R;
  a.S = S;
  a.sh = sh;
  a.sw = sw;
  a.ph = ph;
  a.pw = pw;
  a.dgrad = 0;
  a.bnpart = bnpart;
  a.bnshift = bnshift;
  return launch_conv(a, scratch, st);
}

int nhwc_conv_bn_rows(int N, int H, int W, int Cp, int K, int R, int S, int sh, int sw, int ph, int pw, int P, int Q) {
  // upper bound: one per 128-pixel tile (the LDS-DMA kernel's two-stage variant; 256-pixel tiles
  // elsewhere -- the launch returns the rows it wrote), or the split-K reduce's rows
  int rows = std::max(cdiv(N * P * Q, 128), splitk_bn_rows(N * P * Q, K));  // or the split-K reduce's
  if (Cp == 64 && K == 64 && R == 3 && S == 3 && sh == 1 && sw == 1 && ph == 1 && pw == 1 && P == H && Q == W &&
      W <= 64) {  // the band kernel writes one row per band
    const int rt = c3_band_rows(P, Q);
    if (rt >= 2) rows = std::max(rows, N * P / rt);
  }
  return rows;
}

static ConvNArgs dgrad_args(const uint16_t* dy, const uint16_t* wt_d, uint16_t* dx, int N, int H, int W, int C, int K,
                            int R, int S, int sh, int sw, int ph, int pw, int P, int Q) {
  MX_CHECK((sh == 1 || sh == 2) && (sw == 1 || sw == 2), "nhwc dgrad: stride 1 or 2");
  ConvNArgs a{};
  a.act = dy;
  a.wt = wt_d;
  a.out = dx;
  a.M = N * H * W;
  a.Ng = C;
  a.Kg = R * S * K;
  a.Ca = K;
  a.OH = H;
  a.OW = W;
  a.IH = P;
  a.IW = Q;
  a.R = R;
  a.S = S;
  a.sh = sh;
  a.sw = sw;
  a.ph = ph;
  a.pw = pw;
  a.dgrad = 1;
  return a;
}

size_t nhwc_conv_dgrad_scratch_floats(int N, int H, int W, int C, int K, int R, int S, int sh, int sw, int ph, int pw,
                                      int P, int Q) {
  const ConvNArgs a = dgrad_args(nullptr, nullptr, nullptr, N, H, W, C, K, R, S, sh, sw, ph, pw, P, Q);
  const ConvSetup cs = conv_setup(a);
  const GldsPlan g = glds_plan(a, cs.wide, cs.par);
  const int splits = g.tm ? g.splits : cs.p.splits;
  return splits > 1 ? (size_t)splits * a.M * a.Ng : 0;
}

int nhwc_conv_dgrad(const uint16_t* dy, const uint16_t* wt_d, uint16_t* dx, int N, int H, int W, int C, int K, int R,
                    int S, int sh, int sw, int ph, int pw, int P, int Q, float* scratch, hipStream_t st,
                    const uint16_t* addend, float* bnpart, const uint16_t* bx, const float* bmean,
                    const float* bfcoef, const uint8_t* bmask, bool brelu, const uint8_t* amask, bool addend_sub) {
  ConvNArgs a = dgrad_args(dy, wt_d, dx, N, H, W, C, K, R, S, sh, sw, ph, pw, P, Q);
  a.addend = addend;
  a.amask = addend ? amask : nullptr;
  if (addend && addend_sub) {
    // the implicit-GEMM kernels' shared epilogue (epi_vectors) maps it; the 3x3 band and stem
    // kernels are never chosen for a 1x1 layer
    MX_CHECK(R == 1 && S == 1 && sh == 1 && sw == 1 && H % 2 == 0 && W % 2 == 0 && !amask,
             "nhwc dgrad: a half-resolution addend needs a 1x1 stride-1 layer of even size, no mask");
    a.asub = 1;
  }
  if (bnpart && bx && bmean) {
    MX_CHECK(!brelu || bfcoef || bmask, "nhwc dgrad BN statistics: a ReLU needs the forward's coefficients or mask");
    a.bnpart = bnpart;
    a.bx = reinterpret_cast<const bf16*>(bx);
    a.bmean = bmean;
    a.bfcoef = brelu ? bfcoef : nullptr;
    a.bmask = (brelu && !bfcoef) ? bmask : nullptr;
    a.brelu = brelu ? 1 : 0;
  }
  return launch_conv(a, scratch, st);
}

int nhwc_conv_dgrad_bn_rows(int N, int H, int W, int C, int K, int R, int S, int sh, int sw, int ph, int pw, int P,
                            int Q) {
  // upper bound of the partial rows the data gradient's epilogue writes (the LDS-DMA kernel: one
  // per 256-pixel tile; the generic kernel: one per (parity class, pixel tile) of >= 64 pixels)
  const int M = N * H * W;
  return std::max(cdiv(M, 256), cdiv(M, 64) + 4);
}

// 256 x 256 weight-gradient tiles where both GEMM dimensions reach 256 and the layer is a 3x3
// with > 12,544 pixels or has >= 96 K pixels (A/B: nhwc_wgrad_set_tile256).  (The two 3x3 layers
// of exactly 12,544 output pixels at batch 256 -- the 7 x 7 stage -- moved to the 8-wave 128 x 128
// tile once it existed: 141 -> 129 and 140 -> 130 us, profiles/r5_wtile/.)  Per layer at batch
// 256 (profiles/r5_wgrad/): the 3x3 layers 395 -> 585, 402 -> 585 TF/s, 28 x 28 1x1 412 -> 482;
// the 1x1 layers of 14 x 14 and 7 x 7 (<= 50 K pixels, one block per CU with few stages each)
// 3-14 % slower.  At batch 32 (<= 6,272 pixels per layer) every 3x3 layer lost 17-22 % and the
// step 1.6 % (5,345 vs 5,429 img/s, profiles/r5_wgrad/rn32_*), so small layers keep 128 x 128.
static int g_wgrad_tile256 = 1;
void nhwc_wgrad_set_tile256(int on) { g_wgrad_tile256 = on; }
static void wgrad_tile(int K, int Ng, int Npix, int RS, int& tm, int& tn) {
  if (g_wgrad_tile256 && K >= 256 && Ng >= 256 && ((RS > 1 && Npix > 12544) || Npix >= 96 * 1024)) {
    tm = tn = 256;
    return;
  }
  tm = K <= 64 ? 64 : 128;
  tn = Ng <= 64 ? 64 : 128;
}

// weight-gradient blocks aimed at (A/B: nhwc_wgrad_set_target; 256 and 1,024 measured no better,
// profiles/r4_y/); half that for the one-block-per-CU 256 x 256 tile
static int g_wgrad_target = 512;
// 128 x 128 (and 128 x 64) weight-gradient tiles over 8 waves (wave tile 64 x 32) instead of 4:
// four waves per SIMD at two blocks per CU.  ResNet-50 batch 32 5,568-5,582 vs 5,514-5,536 img/s,
// batch 256 +0.2 % (noise); with 1,024 blocks aimed at instead of 512, batch 256 lost 2.5 %
// (profiles/r5_w8/).  A/B: nhwc_wgrad_set_waves8
static int g_wgrad_w8 = 1;
void nhwc_wgrad_set_waves8(int on) { g_wgrad_w8 = on; }
void nhwc_wgrad_set_target(int n) { g_wgrad_target = n; }
// Layers of at most this many output pixels that would split into >= 32 planes aim at half the
// blocks: their split-K planes (written, then read back by the reduction) cost more than the
// extra blocks gain.  ResNet-50 batch 32, on one box: all layers at target 512 / 256 / 128 =
// 5,850 / 5,883 / 5,631 img/s; half the target below 6,272 / 25,088 / 100,352 pixels 5,905 /
// 5,924 / 5,922 vs 5,897 (the 28 x 28 stage's 49-plane layers carry the gain); batch 256 lost
// 1.2 % / 0.7 % with the 100,352 / 25,088 pixel rule alone (its 7 x 7 and 14 x 14 layers split
// into 4-15 planes), so the plane count gates it too (profiles/r6_wtarget/).  A/B:
// nhwc_wgrad_set_small_npix (0 = off)
static int g_wgrad_small_npix = 25088;
void nhwc_wgrad_set_small_npix(int n) { g_wgrad_small_npix = n; }
static int wgrad_splits_for(int Npix, int K, int Ng, int tiles, int target) {
  // ~2 blocks per CU (1 for the 256 tile), >= 512 pixels (8 stages) per block, partial planes
  // <= 32M floats
  int splits = std::max(1, cdiv(target, tiles));
  splits = std::min(splits, std::max(1, Npix / 512));
  splits = std::min(splits, std::max(1, (int)((32ll << 20) / ((int64_t)K * Ng))));
  const int chunk = cdiv(cdiv(Npix, splits), 64) * 64;
  return cdiv(Npix, chunk);
}
static int wgrad_splits(int Npix, int K, int Ng, int RS) {
  int tm, tn;
  wgrad_tile(K, Ng, Npix, RS, tm, tn);
  const int tiles = cdiv(K, tm) * cdiv(Ng, tn);
  const int target = tm == 256 ? g_wgrad_target / 2 : g_wgrad_target;
  const int splits = wgrad_splits_for(Npix, K, Ng, tiles, target);
  if (Npix <= g_wgrad_small_npix && splits >= 32) return wgrad_splits_for(Npix, K, Ng, tiles, target / 2);
  return splits;
}

size_t nhwc_wgrad_scratch_floats(int N, int Cp, int K, int R, int S, int P, int Q) {
  const int Ng = R * S * Cp;
  size_t n = (size_t)wgrad_splits(N * P * Q, K, Ng, R * S) * K * Ng;
  if (Cp == 8 && R == 7 && S == 7 && K == 64 && P % 16 == 0 && Q % 16 == 0)  // the stem kernel may run
    n = std::max(n, (size_t)kSwBlocks * K * Ng);
  if (Cp == 64 && K == 64 && R == 3 && S == 3 && Q <= 64 && Q % 8 == 0 && c3_band_rows(P, Q) >= 2)  // band kernel
    n = std::max(n, (size_t)kSwBlocks * K * Ng);
  return n;
}

// the weight gradient's split reduction: launched now, or recorded for the optimizer's batched
// flush (wgrad_defer.h) when the caller opted this call in
static void nhwc_wgrad_reduce(const float* part, float* dw, int splits, int K, int Ng, int Cp, int Cin, int RS,
                              bool accumulate, int G, hipStream_t st) {
  const int plane4 = K * Ng / 4, blocks = cdiv(plane4, 256 / G);
  if (wgrad_defer_active()) {
    RedJob j{};
    j.part = part;
    j.dw = dw;
    j.plane = plane4;
    j.nplanes = splits;
    j.G = G;
    j.acc = accumulate ? 1 : 0;
    j.kind = 1;
    j.Kout = K;
    j.Ng = Ng;
    j.Ca = Cp;
    j.Cin = Cin;
    j.RS = RS;
    j.blocks = blocks;
    wgrad_defer_push(j);
    return;
  }
  MX_LAUNCH(wgrad_nhwc_reduce_k, dim3(blocks), dim3(256), 0, st, part, dw, splits, K, Ng, Cp, Cin, RS,
            accumulate ? 1 : 0, G);
}

void nhwc_reduce_batch_launch(const RedBatch& b, int blocks, hipStream_t st) {
  MX_LAUNCH(wgrad_nhwc_reduce_batch_k, dim3(blocks), dim3(256), 0, st, b);
}

void nhwc_conv_wgrad(const uint16_t* dy, const uint16_t* x, float* dw, int N, int H, int W, int Cin, int Cp, int K,
                     int R, int S, int sh, int sw, int ph, int pw, int P, int Q, bool accumulate, float* scratch,
                     hipStream_t st) {
  MX_CHECK(Cp % 8 == 0 && K % 8 == 0, "nhwc wgrad: channels must be multiples of 8");
  WgNArgs a{};
  a.dy = dy;
  a.x = x;
  a.part = scratch;
  a.Npix = N * P * Q;
  a.Kout = K;
  a.Ca = Cp;
  a.Cin = Cin;
  a.H = H;
  a.W = W;
  a.P = P;
  a.Q = Q;
  a.R = R;
  a.S = S;
  a.sh = sh;
  a.sw = sw;
  a.ph = ph;
  a.pw = pw;
  a.Ng = R * S * Cp;
  a.fQ = FastDiv(Q);
  a.fPQ = FastDiv(P * Q);
  a.fCa = FastDiv(Cp);
  a.fS = FastDiv(S);
  MX_CHECK((int64_t)K * a.Ng < (1ll << 31), "nhwc wgrad: weight too large for 32-bit indices");
  if (wgrad_c3_eligible(a)) {  // persistent band kernel, one plane per block
    const int rt = c3_band_rows(P, Q);
    MX_LAUNCH(wgrad_c3_kernel, dim3(kSwBlocks), dim3(512), 0, st, a, rt, N * (P / rt));
    nhwc_wgrad_reduce(scratch, dw, kSwBlocks, K, a.Ng, Cp, Cin, R * S, accumulate, 16, st);
    return;
  }
  if (wgrad_stem_eligible(a)) {  // persistent LDS-patch kernel, one plane per block
    MX_LAUNCH(wgrad_stem_kernel, dim3(kSwBlocks), dim3(512), 0, st, a, N * (P / 16) * (Q / 16));
    nhwc_wgrad_reduce(scratch, dw, kSwBlocks, K, a.Ng, Cp, Cin, R * S, accumulate, 16, st);
    return;
  }
  int tm, tn;
  wgrad_tile(K, a.Ng, a.Npix, R * S, tm, tn);
  const int tiles = cdiv(K, tm) * cdiv(a.Ng, tn);
  const int splits = wgrad_splits(a.Npix, K, a.Ng, R * S);
  a.chunk = cdiv(cdiv(a.Npix, splits), 64) * 64;
  const dim3 grid(tiles * splits);
  if (tm == 256) MX_LAUNCH((wgrad_nhwc_kernel<256, 256, 2, 4>), grid, dim3(512), 0, st, a);
  else if (tm == 128 && tn == 128 && g_wgrad_w8) MX_LAUNCH((wgrad_nhwc_kernel<128, 128, 2, 4>), grid, dim3(512), 0, st, a);
  else if (tm == 128 && tn == 128) MX_LAUNCH((wgrad_nhwc_kernel<128, 128>), grid, dim3(256), 0, st, a);
  else if (tm == 128 && g_wgrad_w8) MX_LAUNCH((wgrad_nhwc_kernel<128, 64, 2, 4>), grid, dim3(512), 0, st, a);
  else if (tm == 128) MX_LAUNCH((wgrad_nhwc_kernel<128, 64>), grid, dim3(256), 0, st, a);
  else if (tn == 128) MX_LAUNCH((wgrad_nhwc_kernel<64, 128>), grid, dim3(256), 0, st, a);
  else MX_LAUNCH((wgrad_nhwc_kernel<64, 64>), grid, dim3(256), 0, st, a);
  MX_CHECK((int64_t)K * a.Ng < (1ll << 31), "nhwc wgrad: weight too large for 32-bit indices");
  int G = 1;  // split groups per reduce block: enough that each thread sums <= ~8 splits
  while (G < 16 && G * 8 < splits) G *= 2;
  nhwc_wgrad_reduce(scratch, dw, splits, K, a.Ng, Cp, Cin, R * S, accumulate, G, st);
}

static dim3 bn_grid(int Npix, int C) {
  const int V = C / 8, vv = V >= kBnT ? kBnT : V, ppi = kBnT / vv;
  const int gy = V >= kBnT ? V / kBnT : 1;
  // ~1024 blocks in total (one partial row each; 2,048 - 8,192 measured slower on a 411 MB
  // tensor, profiles/r4_k/bench_bn.log), at least 8 pixel rows per thread
  const int gx = std::max(1, std::min(cdiv(Npix, ppi * 8), std::max(1, 1024 / gy)));
  return dim3(gx, gy);
}

size_t nhwc_bn_scratch_floats(int Npix, int C) {
  const dim3 g = bn_grid(Npix, C);
  return (size_t)g.x * 2 * C + 3 * (size_t)C;  // partials + coefficients
}

void nhwc_bn_fwd(const uint16_t* x, const uint16_t* res, uint16_t* y, const float* gamma, const float* beta,
                 float* mean, float* invstd, float* run_mean, float* run_var, int64_t* num_batches, int Npix, int C,
                 float momentum, float eps, bool relu, float* scratch, hipStream_t st, float* coef_out,
                 uint8_t* mask_out, const float* pre_part, int pre_gx, const float* kshift) {
  const int V = C / 8;
  MX_CHECK(C % 8 == 0 && C <= 2048 && (V >= kBnT ? V % kBnT == 0 : kBnT % V == 0),
           "nhwc bn: unsupported channel count");
  const dim3 g = bn_grid(Npix, C);
  BnNArgs a{};
  a.Npix = Npix;
  a.C = C;
  a.x = x;
  a.res = res;
  a.y = y;
  a.gamma = gamma;
  a.beta = beta;
  a.mean = mean;
  a.invstd = invstd;
  a.run_mean = run_mean;
  a.run_var = run_var;
  a.part = scratch;
  a.coef = coef_out ? coef_out : scratch + (size_t)g.x * 2 * C;  // kept for the backward's ReLU mask
  a.gx = g.x;
  a.num_batches = num_batches;
  a.relu = relu;
  a.mask = relu ? mask_out : nullptr;
  a.momentum = momentum;
  a.eps = eps;
  if (pre_part) {  // the producing conv's epilogue already wrote the partial sums
    MX_CHECK(pre_gx >= 1 && pre_gx <= 16384, "nhwc bn: precomputed partial rows out of range");
    a.part = const_cast<float*>(pre_part);
    a.gx = pre_gx;
    a.pre = 1;
    a.kshift = kshift;
  } else {
    MX_LAUNCH(bn_nhwc_partial_k<false>, g, dim3(kBnT), 0, st, a);
  }
  MX_LAUNCH(bn_nhwc_finalize_k<false>, dim3(cdiv(C, 8)), dim3(1024), 0, st, a);
  MX_CHECK((int64_t)Npix * V < (1ll << 31), "nhwc bn: tensor too large for 32-bit indices");
  const dim3 agrid(stream_blocks((int64_t)Npix * V));
  a.wt = g_bn_wt;
  MX_LAUNCH((bn_nhwc_apply_k<2, true>), agrid, dim3(kBnT), 0, st, a, FastDiv(V));
}

void nhwc_bn_bwd(const uint16_t* dy, const uint16_t* x, const uint16_t* y, const float* gamma, const float* mean,
                 const float* invstd, uint16_t* dx, uint16_t* dres, float* dgamma, float* dbeta, int Npix, int C,
                 bool relu, bool accumulate_params, float* scratch, hipStream_t st, const float* fcoef,
                 const uint8_t* mask, const float* pre_part, int pre_gx) {
  const int V = C / 8;
  MX_CHECK(C % 8 == 0 && C <= 2048 && (V >= kBnT ? V % kBnT == 0 : kBnT % V == 0),
           "nhwc bn: unsupported channel count");
  const dim3 g = bn_grid(Npix, C);
  BnNArgs a{};
  a.Npix = Npix;
  a.C = C;
  a.dy = dy;
  a.x = x;
  a.y = const_cast<uint16_t*>(y);
  a.gamma = gamma;
  a.mean = const_cast<float*>(mean);
  a.invstd = const_cast<float*>(invstd);
  a.dx = dx;
  a.dres = dres;
  a.dgamma = dgamma;
  a.dbeta = dbeta;
  a.part = scratch;
  a.coef = scratch + (size_t)g.x * 2 * C;
  a.gx = g.x;
  a.relu = relu;
  a.acc_params = accumulate_params;
  a.fcoef = (relu && fcoef && C <= 512) ? fcoef : nullptr;
  a.mask = (relu && !a.fcoef) ? const_cast<uint8_t*>(mask) : nullptr;
  MX_CHECK(!relu || a.fcoef || a.mask || y, "nhwc bn bwd: ReLU needs y, the forward's mask or its coefficients");
  if (pre_part) {  // the consuming conv's data-gradient epilogue wrote the partial sums
    MX_CHECK(pre_gx >= 1 && pre_gx <= 16384, "nhwc bn bwd: precomputed partial rows out of range");
    a.part = const_cast<float*>(pre_part);
    a.gx = pre_gx;
  } else {
    MX_LAUNCH(bn_nhwc_partial_k<true>, g, dim3(kBnT), 0, st, a);
  }
  MX_LAUNCH(bn_nhwc_finalize_k<true>, dim3(cdiv(C, 8)), dim3(1024), 0, st, a);
  MX_CHECK((int64_t)Npix * V < (1ll << 31), "nhwc bn: tensor too large for 32-bit indices");
  const dim3 agrid(stream_blocks((int64_t)Npix * V));
  a.wt = g_bn_wt;
  if (a.fcoef) MX_LAUNCH((bn_nhwc_bwd_apply_k<true, 2, true>), agrid, dim3(kBnT), 0, st, a, FastDiv(V));
  else MX_LAUNCH((bn_nhwc_bwd_apply_k<false, 2, true>), agrid, dim3(kBnT), 0, st, a, FastDiv(V));
}

void nhwc_maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* arg, int N, int H, int W, int C, int P, int Q, int k,
                      int s, int p, hipStream_t st) {
  MX_CHECK(C % 8 == 0 && (int64_t)N * H * W * C / 8 < (1ll << 31), "nhwc maxpool: C % 8 and 32-bit indices");
  const dim3 g(grid_for((int64_t)N * P * Q * (C / 8))), b(256);  // (stream_blocks: 133 -> 147 us)
  const FastDiv fV(C / 8), fQ(Q), fP(P);
  if (k == 3) MX_LAUNCH(maxpool_nhwc_k<3>, g, b, 0, st, x, y, arg, N, H, W, C, P, Q, k, s, p, fV, fQ, fP);
  else MX_LAUNCH(maxpool_nhwc_k<0>, g, b, 0, st, x, y, arg, N, H, W, C, P, Q, k, s, p, fV, fQ, fP);
}

void nhwc_maxpool_bwd(const uint16_t* dy, const uint8_t* arg, uint16_t* dx, int N, int H, int W, int C, int P, int Q,
                      int k, int s, int p, hipStream_t st) {
  MX_CHECK(C % 8 == 0 && (int64_t)N * H * W * C / 8 < (1ll << 31), "nhwc maxpool: C % 8 and 32-bit indices");
  const dim3 g(grid_for((int64_t)N * H * W * (C / 8))), b(256);  // (stream_blocks: no change)
  const FastDiv fV(C / 8), fW(W), fH(H), fS(s);
  if (k == 3 && s == 2 && p == 1)
    MX_LAUNCH(maxpool_nhwc_bwd_s2_k, g, b, 0, st, dy, arg, dx, N, H, W, C, P, Q, fV, fW, fH);
  else if (k == 3) MX_LAUNCH(maxpool_nhwc_bwd_k<3>, g, b, 0, st, dy, arg, dx, N, H, W, C, P, Q, k, s, p, fV, fW, fH, fS);
  else MX_LAUNCH(maxpool_nhwc_bwd_k<0>, g, b, 0, st, dy, arg, dx, N, H, W, C, P, Q, k, s, p, fV, fW, fH, fS);
}

void nhwc_gap_fwd(const uint16_t* x, float* y, int N, int HW, int C, hipStream_t st) {
  MX_LAUNCH(gap_nhwc_k, dim3(cdiv(C, 256), N), dim3(256), 0, st, x, y, N, HW, C);
}

void nhwc_gap_bwd(const float* dy, uint16_t* dx, int N, int HW, int C, hipStream_t st) {
  MX_LAUNCH(gap_nhwc_bwd_k, dim3(grid_for((int64_t)N * HW * C)), dim3(256), 0, st, dy, dx, N, HW, C);
}

}  // namespace mx
