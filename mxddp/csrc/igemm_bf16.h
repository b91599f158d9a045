// bf16-operand / fp32-accumulate variant of the implicit-GEMM engine (igemm.h), for the
// mixed-precision path (--dtype bf16: ResNet-50 config of BASELINE.json).  Same Op interface:
// operands are gathered in fp32 from the fp32 tensors, rounded to bf16 (RNE) while being
// staged into LDS, and multiplied on v_mfma_f32_16x16x32_bf16 (16x the f32 MFMA rate).
//
// LDS tiles are row-major with K contiguous ([BM][BK+8] / [BN][BK+8] bf16): each lane's MFMA
// fragment (8 consecutive k of one row) is ONE ds_read_b128; the +8 element pad makes the row
// pitch 144 B (9 x 16 B, odd) so the 16 rows read by a 16-lane group hit 16 distinct 16-B slots.
#pragma once
#include "common.h"

namespace mx {

typedef short bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ unsigned short f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);  // round to nearest even
  return (unsigned short)(u >> 16);
}

template <class Op, int BM, int BN, int BK, int WM, int WN>
__global__ __launch_bounds__(256) void igemm_bf16_kernel(Op op, int k_split_len) {
  static_assert(WM * WN == 4, "4 waves per block");
  static_assert(BK % 32 == 0, "BK multiple of the MFMA K (32)");
  static_assert((BM * BK) % 256 == 0 && (BN * BK) % 256 == 0, "tile loads must split evenly");
  constexpr int LD = BK + 8;  // bf16 elements per LDS row
  constexpr int EA = BM * BK / 256, EB = BN * BK / 256;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  __shared__ __attribute__((aligned(16))) unsigned short As[2][BM * LD];
  __shared__ __attribute__((aligned(16))) unsigned short Bs[2][BN * LD];

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
  // raw values + validity bits, converted / zeroed at LDS-store time (see igemm.h)
  static_assert(EA <= 32 && EB <= 32, "validity bits");
  float ra[EA], rb[EB];
  uint32_t va = 0, vb = 0;
  auto gload = [&](int k0) {
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
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < EA; ++i) As[buf][a_ml[i] * LD + a_kl[i]] = f2bf((va >> i) & 1u ? ra[i] : 0.f);
#pragma unroll
    for (int i = 0; i < EB; ++i) Bs[buf][b_nl[i] * LD + b_kl[i]] = f2bf((vb >> i) & 1u ? rb[i] : 0.f);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nt = (kend - kbeg + BK - 1) / BK;
  gload(kbeg);
  sstore(0);
  __syncthreads();
  const int a_row = wm * (BM / WM) + (lane & 15), b_row = wn * (BN / WN) + (lane & 15);
  const int koff = 8 * (lane >> 4);
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    if (t + 1 < nt) gload(kbeg + (t + 1) * BK);
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        a[i] = *reinterpret_cast<const bf16x8*>(&As[cur][(a_row + 16 * i) * LD + kk * 32 + koff]);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        b[j] = *reinterpret_cast<const bf16x8*>(&Bs[cur][(b_row + 16 * j) * LD + kk * 32 + koff]);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (t + 1 < nt) sstore(cur ^ 1);
    __syncthreads();
  }
  igemm_epilogue<Op, BM, BN, WM, WN, TM, TN>(op, acc, m0, n0, wm, wn, lane);
}

template <class Op, int BM, int BN, int BK, int WM, int WN>
inline void igemm_bf16_launch(const Op& op, int splits, hipStream_t st) {
  if (op.M <= 0 || op.N <= 0 || op.K <= 0) return;
  const int tiles = cdiv(op.M, BM) * cdiv(op.N, BN);
  splits = splits < 1 ? 1 : splits;
  int klen = cdiv(cdiv(op.K, splits), BK) * BK;
  splits = cdiv(op.K, klen);
  MX_LAUNCH((igemm_bf16_kernel<Op, BM, BN, BK, WM, WN>), dim3(tiles, 1, splits), dim3(256), 0, st, op,
                     klen);
  MX_HIP_CHECK(hipGetLastError());
}

}  // namespace mx
