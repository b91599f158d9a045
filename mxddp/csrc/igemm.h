// Implicit-GEMM engine on fp32-input MFMA (v_mfma_f32_16x16x4_f32), gfx950.
//
// One templated kernel drives every GEMM-shaped op of the framework (conv fwd /
// dgrad / wgrad in NCHW, linear fwd / dgrad / wgrad).  An "Op" describes how to
// gather the A[m][k] and B[k][n] operands from global memory (im2col on the fly,
// nothing materialised) and how to store C[m][n] (bias / ReLU / mask / split-K
// atomics fused into the epilogue).
//
// Block = 256 threads = 4 waves in a WM x WN grid; block tile BM x BN, k-tile BK.
// Operand tiles are staged global -> registers -> LDS (k-major, rows padded so the
// two 16-lane groups of a ds_read_b32 half-wave hit disjoint banks), double-buffered
// with one barrier per k-tile; global loads run two k-tiles ahead (two register sets).  Columns are XOR-swizzled by (k & 14): an operand gathered
// k-fast (weights along K, dy along pixels) stores 16 k-rows x 2 columns per 32-lane group,
// and with the 16-mod-32 row pitch the even rows shared one bank (8-way conflicts: the
// counters showed 2-4x more conflict cycles than LDS-active cycles); the XOR only permutes
// columns inside each 16-aligned group, so the MFMA operand reads stay conflict-free.  Each wave owns (BM/WM) x (BN/WN) outputs as
// TM x TN MFMA 16x16 accumulators.  fp32 in, fp32 accumulate: exact fp32 numerics
// (gfx950 has no xf32), at the f32 matrix rate.
//
// Reference behaviour being replaced: cuDNN conv / cuBLAS GEMM reached through
// nn.Conv2d / nn.Linear in pytorch/model.py:28-32,62-63,77 and the Keras/Chainer
// layers (tensorflow2/mnist_single.py:17-26, chainer/train_mnist.py:19-21).
#pragma once
#include "common.h"

namespace mx {

// Epilogue shared by the fp32 and bf16 engines.  Phase 1 requests every output's operands (bias,
// mask, accumulate source: Op::spre, clamped indices) for all of the lane's TM x TN x 4 outputs;
// phase 2 stores.  (store() loading its own operands was one dependent round trip per output.)
// C/D map of the 16x16 MFMA tiles: col = lane & 15, row = (lane >> 4) * 4 + reg.
template <class Op, int BM, int BN, int WM, int WN, int TM, int TN>
__device__ __forceinline__ void igemm_epilogue(const Op& op, const f32x4 (&acc)[TM][TN], int m0, int n0, int wm,
                                               int wn, int lane) {
  typename Op::SP sp[TM][TN][4];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = min(n0 + wn * (BN / WN) + j * 16 + (lane & 15), op.N - 1);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = min(m0 + wm * (BM / WM) + i * 16 + (lane >> 4) * 4 + r, op.M - 1);
        sp[i][j][r] = op.spre(m, n, blockIdx.z);
      }
    }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * (BN / WN) + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * (BM / WM) + i * 16 + (lane >> 4) * 4 + r;
        if (m < op.M && n < op.N) op.store(m, n, acc[i][j][r], blockIdx.z, sp[i][j][r]);
      }
    }
}

template <class Op, int BM, int BN, int BK, int WM, int WN>
__global__ __launch_bounds__(256) void igemm_f32_kernel(Op op, int k_split_len) {
  static_assert(WM * WN == 4, "4 waves per block");
  static_assert(BM % (16 * WM) == 0 && BN % (16 * WN) == 0, "wave tile must be 16-multiple");
  static_assert((BM * BK) % 256 == 0 && (BN * BK) % 256 == 0, "tile loads must split evenly");
  static_assert(BK % 4 == 0, "BK multiple of MFMA K (4)");
  constexpr int LDA = BM + 16, LDB = BN + 16;  // (LD % 32 == 16): k-row groups on disjoint banks
  constexpr int EA = BM * BK / 256, EB = BN * BK / 256;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;

  __shared__ float As[2][BK * LDA];
  __shared__ float Bs[2][BK * LDB];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_n = (op.N + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (bid / tiles_n) * BM, n0 = (bid % tiles_n) * BN;
  const int kbeg = blockIdx.z * k_split_len;
  const int kend = min(op.K, kbeg + k_split_len);
  if (kbeg >= kend) return;

  typename Op::APre apre[EA];
  typename Op::BPre bpre[EB];
  int a_kl[EA], a_ml[EA], b_kl[EB], b_nl[EB];
#pragma unroll
  for (int i = 0; i < EA; ++i) {
    const int e = tid + 256 * i;
    if constexpr (Op::A_MFAST) { a_ml[i] = e % BM; a_kl[i] = e / BM; }
    else { a_kl[i] = e % BK; a_ml[i] = e / BK; }
    apre[i] = op.a_pre(m0 + a_ml[i]);
  }
#pragma unroll
  for (int i = 0; i < EB; ++i) {
    const int e = tid + 256 * i;
    if constexpr (Op::B_NFAST) { b_nl[i] = e % BN; b_kl[i] = e / BN; }
    else { b_kl[i] = e % BK; b_nl[i] = e / BK; }
    bpre[i] = op.b_pre(n0 + b_nl[i]);
  }

  // two register sets of prefetched k-tiles: a tile's global loads are issued two k-tiles
  // before it is stored to LDS (one k-tile of MFMAs was too little to cover the load latency
  // on the long-K, few-block shapes: ~1 us per k-tile)
  // Loads are branch-free: the op reads a clamped address and reports the element's validity
  // (k, bounds, padding) as a bit; the zero is selected only at LDS-store time.  (A load behind a
  // per-element test is a branch, and a select right after the load waits for it: either way the
  // ISA showed s_waitcnt vmcnt(0) after every load, so the two prefetched register sets never
  // actually overlapped the MFMAs.)
  static_assert(EA <= 32 && EB <= 32, "validity bits");
  float ra0[EA], rb0[EB], ra1[EA], rb1[EB];
  uint32_t va0 = 0, vb0 = 0, va1 = 0, vb1 = 0;
  auto gload = [&](float (&ra)[EA], float (&rb)[EB], uint32_t& va, uint32_t& vb, int k0) {
    va = vb = 0;
#pragma unroll
    for (int i = 0; i < EA; ++i) {
      const int k = k0 + a_kl[i];
      bool ok;
      ra[i] = op.a_load(apre[i], min(k, kend - 1), ok);
      va |= (ok && k < kend ? 1u : 0u) << i;
    }
#pragma unroll
    for (int i = 0; i < EB; ++i) {
      const int k = k0 + b_kl[i];
      bool ok;
      rb[i] = op.b_load(bpre[i], min(k, kend - 1), ok);
      vb |= (ok && k < kend ? 1u : 0u) << i;
    }
  };
  static_assert(BK <= 16, "column swizzle assumes k-tile rows < 16");
  auto sstore = [&](int buf, const float (&ra)[EA], const float (&rb)[EB], uint32_t va, uint32_t vb) {
#pragma unroll
    for (int i = 0; i < EA; ++i) As[buf][a_kl[i] * LDA + (a_ml[i] ^ (a_kl[i] & 14))] = (va >> i) & 1u ? ra[i] : 0.f;
#pragma unroll
    for (int i = 0; i < EB; ++i) Bs[buf][b_kl[i] * LDB + (b_nl[i] ^ (b_kl[i] & 14))] = (vb >> i) & 1u ? rb[i] : 0.f;
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nt = (kend - kbeg + BK - 1) / BK;
  const int g = lane >> 4, l16 = lane & 15;
  const int a_off = g * LDA + wm * (BM / WM);
  const int b_off = g * LDB + wn * (BN / WN);
  auto mfma_tile = [&](int cur) {
    const float* as = &As[cur][a_off];
    const float* bs = &Bs[cur][b_off];
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      const int lx = l16 ^ ((4 * kk + (g & 2)) & 14);  // swizzled column of k-row 4kk + g
      float a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = as[kk * 4 * LDA + i * 16 + lx];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = bs[kk * 4 * LDB + j * 16 + lx];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  };
  gload(ra0, rb0, va0, vb0, kbeg);
  sstore(0, ra0, rb0, va0, vb0);
  __syncthreads();
  if (nt > 1) gload(ra0, rb0, va0, vb0, kbeg + BK);      // k-tile 1 -> set 0
  if (nt > 2) gload(ra1, rb1, va1, vb1, kbeg + 2 * BK);  // k-tile 2 -> set 1
  // invariant at even t: LDS buffer 0 holds k-tile t, set 0 k-tile t + 1, set 1 k-tile t + 2
  for (int t = 0; t < nt; t += 2) {
    mfma_tile(0);
    if (t + 1 < nt) sstore(1, ra0, rb0, va0, vb0);
    __syncthreads();
    if (t + 3 < nt) gload(ra0, rb0, va0, vb0, kbeg + (t + 3) * BK);
    if (t + 1 >= nt) break;
    mfma_tile(1);
    if (t + 2 < nt) sstore(0, ra1, rb1, va1, vb1);
    __syncthreads();
    if (t + 4 < nt) gload(ra1, rb1, va1, vb1, kbeg + (t + 4) * BK);
  }
  igemm_epilogue<Op, BM, BN, WM, WN, TM, TN>(op, acc, m0, n0, wm, wn, lane);
}

// Host-side launcher.  `splits` > 1 splits the reduction dimension over gridDim.z;
// the Op's store() must then accumulate atomically (output pre-zeroed).
template <class Op, int BM, int BN, int BK, int WM, int WN>
inline void igemm_launch(const Op& op, int splits, hipStream_t st) {
  if (op.M <= 0 || op.N <= 0) return;
  const int tiles = cdiv(op.M, BM) * cdiv(op.N, BN);
  if (op.K <= 0) return;
  splits = splits < 1 ? 1 : splits;
  int klen = cdiv(cdiv(op.K, splits), BK) * BK;
  splits = cdiv(op.K, klen);
  dim3 grid(tiles, 1, splits);
  MX_LAUNCH((igemm_f32_kernel<Op, BM, BN, BK, WM, WN>), grid, dim3(256), 0, st, op, klen);
  MX_HIP_CHECK(hipGetLastError());
}

// Choose a split-K factor so that the grid roughly fills the chip (256 CUs) without
// making each split shorter than `min_k` reduction elements.
inline int pick_splits(int tiles, int K, int min_k = 256, int target_blocks = 512) {
  if (tiles >= target_blocks) return 1;
  int s = target_blocks / (tiles > 0 ? tiles : 1);
  int max_s = K / min_k;
  if (s > max_s) s = max_s;
  return s < 1 ? 1 : s;
}

}  // namespace mx
