// Direct-LDS 3x3 / stride-1 / pad-1 convolution on fp32 MFMA (v_mfma_f32_16x16x4_f32), gfx950.
//
// The generic implicit GEMM (igemm.h) gathers every im2col element with its own index
// arithmetic and 4-byte load.  For the 3x3 s1 p1 convolutions that make up almost all of
// PyramidNet (and most 3x3s of ResNet) this kernel instead stages, per chunk of 8 input
// channels, ONE zero-padded input patch [8][TH+2][W+2] (full image rows, coalesced) and the
// weight slab [64 couts][8 x 9] in LDS, then forms the im2col operand straight from the patch:
// with K ordered k = tap*8 + ci, MFMA k-step s reads tap s/2 and channels 4*(s&1)+g, so each
// lane's B address is a per-lane base + a compile-time offset (no index math in the loop).
//
// GEMM per block: M = 64 output channels (A = weights), N = 64 output positions (B = patch
// im2col; TH = 64/W full rows; W is a template parameter so all patch index math divides by
// constants), K = 9*C in chunks of 72.  4 waves in 2 x 2, each 32 x 32 = 2 x 2 MFMA tiles.
// Output positions are the MFMA columns, so the epilogue writes 16 consecutive pixels per lane
// group (coalesced NCHW stores).  Fused epilogue: bias, ReLU, mask (dx *= mask > 0), accumulate.
// Global loads of chunk c+1 are issued into registers before chunk c's MFMAs.
//
// The data gradient of a 3x3 s1 p1 conv is the same convolution of dy with the weights
// transposed/flipped (w'[ci][co][8-tap]): conv3x3_dgrad runs a tiny transpose then this kernel.
//
// Replaces (reference): cuDNN conv fwd / bwd-data for pytorch/model.py:28-32 (PyramidNet).
#include "common.h"
#include "ops.h"

#include <algorithm>

namespace mx {

namespace {

constexpr int kCi = 8, kKK = kCi * 9, kLDA = 80;  // As [72][80]: k rows, 16 mod 32 pitch

struct C3Args {
  const float* x;     // [N][C][H][W]
  const float* w;     // [K][C][3][3]
  const float* bias;  // [K] or null
  const float* mask;  // [N][K][H][W] or null
  float* y;           // [N][K][H][W]
  int N, C, H, K;
  int tiles_h, ktiles;
  int relu, accumulate;
};

constexpr int round16(int v) { return (v + 15) / 16 * 16; }
constexpr int pad16mod32(int v) { return round16(v) % 32 == 0 ? round16(v) + 16 : round16(v); }

template <int W>
struct C3Geom {
  static constexpr int TH = 64 / W, PW = W + 2, PR = TH + 2, RP = PW, CHP = pad16mod32(PR * PW);
  static constexpr int pelems = kCi * PR * PW, EP = (pelems + 255) / 256, EW = 64 * kKK / 256;
  static constexpr size_t lds = sizeof(float) * ((size_t)kKK * kLDA + (size_t)kCi * CHP);
};

template <int W>
__global__ __launch_bounds__(256) void conv3x3_kernel(C3Args a) {
  using G = C3Geom<W>;
  constexpr int TH = G::TH, PW = G::PW, PR = G::PR, RP = G::RP, CHP = G::CHP;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* As = sm;               // [72][80]
  float* Ps = sm + kKK * kLDA;  // [8][CHP]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave >> 1, wn = wave & 1;
  const int g = lane >> 4, l16 = lane & 15;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);  // blocks sharing an input patch share an XCD
  const int kt = bid % a.ktiles, rest = bid / a.ktiles;
  const int th = rest % a.tiles_h, n = rest / a.tiles_h;
  const int co0 = kt * 64, h0 = th * TH;
  const size_t HW = (size_t)a.H * W;
  const float* xb = a.x + (size_t)n * a.C * HW;

  int bbase[2];  // per-lane B base: output position p -> patch offset of its (0,0) tap
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int p = min(wn * 32 + 16 * j + l16, TH * W - 1);
    const int pr = p / W, pc = p - pr * W;
    bbase[j] = g * CHP + pr * RP + pc;
  }

  // weight slab: thread t loads row m = t/4 (output channel), 18 consecutive (ci, tap) values
  // starting at ci = 2*(t%4): one base pointer + immediate offsets
  const int wm_row = tid >> 2, wq = tid & 3;
  const bool wrow_ok = co0 + wm_row < a.K;
  const float* wrow = a.w + (size_t)min(co0 + wm_row, a.K - 1) * a.C * 9 + wq * 18;
  float rw[G::EW], rp[G::EP];
  auto gload = [&](int c0) {
    const int lim = (a.C - c0) * 9 - wq * 18;  // valid (ci, tap) values left in this row segment
#pragma unroll
    for (int i = 0; i < G::EW; ++i) rw[i] = (wrow_ok && i < lim) ? wrow[c0 * 9 + i] : 0.f;
#pragma unroll
    for (int i = 0; i < G::EP; ++i) {
      const int e = tid + 256 * i;
      float v = 0.f;
      if (e < G::pelems) {
        const int ci = e / (PR * PW), rem = e - ci * (PR * PW), r = rem / PW, c = rem - r * PW;
        const int h = h0 + r - 1, ww = c - 1;
        if (c0 + ci < a.C && (unsigned)h < (unsigned)a.H && (unsigned)ww < (unsigned)W)
          v = xb[(size_t)(c0 + ci) * HW + (size_t)h * W + ww];
      }
      rp[i] = v;
    }
  };
  auto sstore = [&]() {
#pragma unroll
    for (int i = 0; i < G::EW; ++i) As[((i % 9) * kCi + 2 * wq + i / 9) * kLDA + wm_row] = rw[i];
#pragma unroll
    for (int i = 0; i < G::EP; ++i) {
      const int e = tid + 256 * i;
      if (e < G::pelems) {
        const int ci = e / (PR * PW), rem = e - ci * (PR * PW), r = rem / PW, c = rem - r * PW;
        Ps[ci * CHP + r * RP + c] = rp[i];
      }
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nchunks = (a.C + kCi - 1) / kCi;
  gload(0);
  const float* ap = As + g * kLDA + wm * 32 + l16;
  for (int ch = 0; ch < nchunks; ++ch) {
    if (ch) __syncthreads();  // previous chunk's LDS reads are done
    sstore();
    __syncthreads();
    if (ch + 1 < nchunks) gload((ch + 1) * kCi);
#pragma unroll
    for (int s = 0; s < 18; ++s) {
      const int tap = s >> 1, ky = tap / 3, kx = tap - 3 * ky;
      const int koff = 4 * (s & 1) * CHP + ky * RP + kx;
      float av[2], bv[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) av[i] = ap[4 * s * kLDA + 16 * i];
#pragma unroll
      for (int j = 0; j < 2; ++j) bv[j] = Ps[bbase[j] + koff];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
  }

  // epilogue: MFMA row = output channel, column = output position
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int p = wn * 32 + 16 * j + l16;
    const int pr = p / W, pc = p - pr * W, h = h0 + pr;
    if (p >= TH * W || h >= a.H) continue;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wm * 32 + 16 * i + 4 * g + r;
        if (co >= a.K) continue;
        const size_t o = ((size_t)n * a.K + co) * HW + (size_t)h * W + pc;
        float v = acc[i][j][r];
        if (a.bias) v += a.bias[co];
        if (a.relu) v = fmaxf(v, 0.f);
        if (a.mask && !(a.mask[o] > 0.f)) v = 0.f;
        if (a.accumulate) v += a.y[o];
        a.y[o] = v;
      }
  }
}

// ------------------------------------------------------------------------------------------
// Weight gradient of a 3x3 s1 p1 conv: dw[co][ci][tap] += sum_{n,h,w} dy[n][co][h][w] *
// x[n][ci][h+ky-1][w+kx-1].  GEMM: M = 64 output channels (A = dy tile in LDS), N = 16 input
// channels x 9 taps = 144 columns (B = im2col of the x patch in LDS, per-lane constant (ci, tap)
// offset + a compile-time position offset), K = output positions, walked one 64-position tile
// (TH full rows) at a time over a group of G images.  Wave w owns output channels 16w..16w+15
// x all 9 column tiles (9 accumulators).  W % 4 == 0 so a 4-position k-group never straddles a
// row.  Block results are atomically added into dw (G images per block bound the contention).
struct C3WArgs {
  const float* dy;  // [N][K][H][W]
  const float* x;   // [N][C][H][W]
  float* dw;        // [K][C][3][3]
  int N, C, H, K;
  int tiles_h, ktiles, cchunks, G, ngroups;
};
constexpr int kWCi = 16, kDP = 66;  // dy tile pitch: 16 co rows x 2 lane groups -> distinct banks

template <int W>
struct C3WGeom {
  static constexpr int TH = 64 / W, NP = TH * W, PW = W + 2, PR = TH + 2, RP = PW, CHP = pad16mod32(PR * PW);
  static constexpr int pelems = kWCi * PR * PW, EP = (pelems + 255) / 256;
  static constexpr size_t lds = sizeof(float) * ((size_t)64 * kDP + (size_t)kWCi * CHP);
};

template <int W>
__global__ __launch_bounds__(256) void conv3x3_wgrad_kernel(C3WArgs a) {
  using G = C3WGeom<W>;
  static_assert(W % 4 == 0, "k-groups of 4 positions must not straddle rows");
  constexpr int TH = G::TH, NP = G::NP, PW = G::PW, PR = G::PR, RP = G::RP, CHP = G::CHP;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Ds = sm;               // [64 co][66]
  float* Ps = sm + 64 * kDP;    // [16 ci][CHP]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, l16 = lane & 15;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int kt = bid % a.ktiles, r1 = bid / a.ktiles;
  const int cc = r1 % a.cchunks, ng = r1 / a.cchunks;
  const int co0 = kt * 64, c0 = cc * kWCi;
  const int n_beg = ng * a.G, n_end = min(a.N, n_beg + a.G);
  const size_t HW = (size_t)a.H * W;

  int bo[9];  // per-lane B offset of column 16j + l16 = (ci, tap)
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    const int c = 16 * j + l16, ci = c / 9, tap = c - 9 * ci;
    bo[j] = ci * CHP + (tap / 3) * RP + (tap % 3) + g;
  }
  // dy tile: thread t -> co row t/4, 16 consecutive positions from (t%4)*16 (float4 x 4)
  const int drow = tid >> 2, dq = tid & 3;
  const bool drow_ok = co0 + drow < a.K;
  float4 rd[4];
  float rp[G::EP];
  auto gload = [&](int n, int th) {
    const int h0 = th * TH;
    const float* dyp = a.dy + ((size_t)n * a.K + min(co0 + drow, a.K - 1)) * HW + (size_t)h0 * W;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = dq * 16 + 4 * i;
      rd[i] = (drow_ok && p < NP && h0 + p / W < a.H) ? *reinterpret_cast<const float4*>(dyp + p)
                                                       : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const float* xb = a.x + ((size_t)n * a.C + c0) * HW;
#pragma unroll
    for (int i = 0; i < G::EP; ++i) {
      const int e = tid + 256 * i;
      float v = 0.f;
      if (e < G::pelems) {
        const int ci = e / (PR * PW), rem = e - ci * (PR * PW), r = rem / PW, c = rem - r * PW;
        const int h = h0 + r - 1, ww = c - 1;
        if (c0 + ci < a.C && (unsigned)h < (unsigned)a.H && (unsigned)ww < (unsigned)W)
          v = xb[(size_t)ci * HW + (size_t)h * W + ww];
      }
      rp[i] = v;
    }
  };
  auto sstore = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<float4*>(Ds + drow * kDP + dq * 16 + 4 * i) = rd[i];
#pragma unroll
    for (int i = 0; i < G::EP; ++i) {
      const int e = tid + 256 * i;
      if (e < G::pelems) {
        const int ci = e / (PR * PW), rem = e - ci * (PR * PW), r = rem / PW, c = rem - r * PW;
        Ps[ci * CHP + r * RP + c] = rp[i];
      }
    }
  };

  f32x4 acc[9];
#pragma unroll
  for (int j = 0; j < 9; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ntiles = (n_end - n_beg) * a.tiles_h;
  gload(n_beg, 0);
  const float* ap = Ds + (16 * w + l16) * kDP + g;
  for (int t = 0; t < ntiles; ++t) {
    if (t) __syncthreads();
    sstore();
    __syncthreads();
    if (t + 1 < ntiles) gload(n_beg + (t + 1) / a.tiles_h, (t + 1) % a.tiles_h);
#pragma unroll
    for (int s = 0; s < NP / 4; ++s) {
      const int pr = (4 * s) / W, pc = (4 * s) % W;  // position 4s + g -> (pr, pc + g)
      const float av = ap[4 * s];
#pragma unroll
      for (int j = 0; j < 9; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, Ps[bo[j] + pr * RP + pc], acc[j], 0, 0, 0);
    }
  }
  // C: row = co (16w + 4g + r), column = 16j + l16 -> (ci, tap)
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    const int c = 16 * j + l16, ci = c / 9, tap = c - 9 * ci;
    if (c0 + ci >= a.C) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = co0 + 16 * w + 4 * g + r;
      if (co < a.K) atomicAdd(a.dw + ((size_t)co * a.C + c0 + ci) * 9 + tap, acc[j][r]);
    }
  }
}

template <int W>
void launch_wgrad_w(const C3WArgs& a, hipStream_t st) {
  const int blocks = a.ngroups * a.cchunks * a.ktiles;
  MX_LAUNCH(conv3x3_wgrad_kernel<W>, dim3(blocks), dim3(256), C3WGeom<W>::lds, st, a);
}

// w'[ci][co][8 - tap] = w[co][ci][tap]: weights of the equivalent forward conv for dgrad.
__global__ void flip_transpose_k(const float* __restrict__ w, float* __restrict__ wt, int K, int C) {
  const int total = K * C * 9;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int tap = i % 9, kc = i / 9, c = kc % C, k = kc / C;
    wt[((size_t)c * K + k) * 9 + (8 - tap)] = w[i];
  }
}

template <int W>
void launch_w(const C3Args& a, hipStream_t st) {
  const int blocks = a.N * a.tiles_h * a.ktiles;
  MX_LAUNCH(conv3x3_kernel<W>, dim3(blocks), dim3(256), C3Geom<W>::lds, st, a);
}

void launch(const float* x, const float* w, const float* bias, const float* mask, float* y, int N, int C, int H,
            int W, int K, bool relu, bool accumulate, hipStream_t st) {
  C3Args a{};
  a.x = x;
  a.w = w;
  a.bias = bias;
  a.mask = mask;
  a.y = y;
  a.N = N;
  a.C = C;
  a.H = H;
  a.K = K;
  a.tiles_h = cdiv(H, 64 / W);
  a.ktiles = cdiv(K, 64);
  a.relu = relu;
  a.accumulate = accumulate;
  switch (W) {
    case 7: return launch_w<7>(a, st);
    case 8: return launch_w<8>(a, st);
    case 14: return launch_w<14>(a, st);
    case 16: return launch_w<16>(a, st);
    case 28: return launch_w<28>(a, st);
    case 32: return launch_w<32>(a, st);
    case 56: return launch_w<56>(a, st);
    default: MX_CHECK(false, "conv3x3: unsupported width");
  }
}

}  // namespace

bool conv3x3_eligible(const ConvShape& s) {
  return s.R == 3 && s.S == 3 && s.str_h == 1 && s.str_w == 1 && s.pad_h == 1 && s.pad_w == 1 && s.dil_h == 1 &&
         s.dil_w == 1 && s.P == s.H && s.Q == s.W &&
         (s.W == 7 || s.W == 8 || s.W == 14 || s.W == 16 || s.W == 28 || s.W == 32 || s.W == 56);
}

void conv3x3_fwd(const float* x, const float* w, const float* bias, float* y, const ConvShape& s, bool relu,
                 hipStream_t st) {
  launch(x, w, bias, nullptr, y, s.N, s.C, s.H, s.W, s.K, relu, false, st);
}

bool conv3x3_wgrad_eligible(const ConvShape& s) {
  return conv3x3_eligible(s) && s.W % 4 == 0;
}

void conv3x3_wgrad(const float* dy, const float* x, float* dw, const ConvShape& s, bool accumulate, hipStream_t st) {
  if (!accumulate) zero_fill(dw, (int64_t)s.K * s.C * 9, st);
  C3WArgs a{};
  a.dy = dy;
  a.x = x;
  a.dw = dw;
  a.N = s.N;
  a.C = s.C;
  a.H = s.H;
  a.K = s.K;
  a.tiles_h = cdiv(s.H, 64 / s.W);
  a.ktiles = cdiv(s.K, 64);
  a.cchunks = cdiv(s.C, kWCi);
  // images per block: enough blocks to fill the chip (~768), as few atomics per address as that allows
  const int per_img = a.ktiles * a.cchunks;
  a.G = std::max(1, (s.N * per_img) / 768);
  a.ngroups = cdiv(s.N, a.G);
  switch (s.W) {
    case 8: return launch_wgrad_w<8>(a, st);
    case 16: return launch_wgrad_w<16>(a, st);
    case 28: return launch_wgrad_w<28>(a, st);
    case 32: return launch_wgrad_w<32>(a, st);
    case 56: return launch_wgrad_w<56>(a, st);
    default: MX_CHECK(false, "conv3x3_wgrad: unsupported width");
  }
}

void conv3x3_dgrad(const float* dy, const float* w, float* dx, const ConvShape& s, const float* relu_mask,
                   bool accumulate, float* wt_scratch, hipStream_t st) {
  const int total = s.K * s.C * 9;
  MX_LAUNCH(flip_transpose_k, dim3(cdiv(total, 256) < 1024 ? cdiv(total, 256) : 1024), dim3(256), 0, st, w,
            wt_scratch, s.K, s.C);
  // forward conv of dy (K channels) with w' -> C channels
  launch(dy, wt_scratch, nullptr, relu_mask, dx, s.N, s.K, s.H, s.W, s.C, false, accumulate, st);
}

}  // namespace mx
