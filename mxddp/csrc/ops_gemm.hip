// Conv2d / Linear forward + backward as Ops of the MFMA implicit-GEMM engine.
// NCHW fp32, arbitrary stride / padding / dilation and non-tile-multiple channel
// counts (PyramidNet-110 has 103 distinct (C_in, C_out) pairs).
#include <algorithm>
#include <mutex>
#include <vector>

#include "igemm.h"
#include "igemm_bf16.h"
#include "ops.h"

namespace mx {
namespace {

enum StoreMode { kStore = 0, kAccum = 1, kAtomic = 2 };

__device__ __forceinline__ void emit(float* out, int64_t idx, float v, int mode) {
  if (mode == kStore) out[idx] = v;
  else if (mode == kAccum) out[idx] += v;
  else atomicAdd(out + idx, v);
}
// Epilogue operands of one output, requested for ALL of a lane's outputs before any is stored
// (igemm epilogue phase 1): bias, ReLU / mask source, accumulate source.  A load inside store()
// was a branch + load + wait per output -- 16 to 32 dependent round trips per lane.
struct SPre {
  float b = 0.f, mk = 1.f, old = 0.f;
};
__device__ __forceinline__ void emit2(float* out, int64_t idx, float v, int mode, float old) {
  if (mode == kStore) out[idx] = v;
  else if (mode == kAccum) out[idx] = old + v;
  else atomicAdd(out + idx, v);
}

// ------------------------------------------------------------------ conv geometry
struct ConvG {
  int N, C, H, W, K, R, S, P, Q, sh, sw, ph, pw, dh, dw;
  int PQ, RS, HW;
  FastDiv fPQ, fQ, fRS, fS, fHW, fW;
  explicit ConvG(const ConvShape& s)
      : N(s.N), C(s.C), H(s.H), W(s.W), K(s.K), R(s.R), S(s.S), P(s.P), Q(s.Q), sh(s.str_h),
        sw(s.str_w), ph(s.pad_h), pw(s.pad_w), dh(s.dil_h), dw(s.dil_w) {
    PQ = P * Q;
    RS = R * S;
    HW = H * W;
    fPQ = FastDiv(PQ);
    fQ = FastDiv(Q);
    fRS = FastDiv(RS);
    fS = FastDiv(S);
    fHW = FastDiv(HW);
    fW = FastDiv(W);
  }
};

// Forward: C[m=(n,p,q)][kout] = sum_{k=(c,r,s)} x[n,c,p*sh-ph+r*dh, q*sw-pw+s*dw] * w[kout,c,r,s]
struct ConvFwdOp {
  using SP = SPre;
  static constexpr bool A_MFAST = true;   // consecutive q -> coalesced input rows
  static constexpr bool B_NFAST = false;  // weights read along (c,r,s)
  int M, N, K;
  ConvG g;
  const float* x;
  const float* w;
  const float* bias;
  float* y;
  bool relu;
  float* part = nullptr;  // split-K: raw partial sums part[split][y index] (finished by splitk_finish_k)
  int64_t ptotal = 0;
  struct APre { int64_t base; int h0, w0; bool ok; };
  struct BPre { int64_t base; bool ok; };
  __device__ APre a_pre(int m) const {
    APre a;
    a.ok = m < M;
    const int mm = a.ok ? m : 0;
    const int n = g.fPQ.div(mm), pq = mm - n * g.PQ;
    const int p = g.fQ.div(pq), q = pq - p * g.Q;
    a.h0 = p * g.sh - g.ph;
    a.w0 = q * g.sw - g.pw;
    a.base = (int64_t)n * g.C * g.HW;
    return a;
  }
  __device__ float a_load(const APre& a, int k, bool& ok) const {
    const int c = g.fRS.div(k), rs = k - c * g.RS;
    const int r = g.fS.div(rs), s = rs - r * g.S;
    const int h = a.h0 + r * g.dh, ww = a.w0 + s * g.dw;
    ok = a.ok && (unsigned)h < (unsigned)g.H && (unsigned)ww < (unsigned)g.W;
    // clamped address, validity returned: the select happens at LDS-store time (a load behind the
    // bounds test is a branch, and a select right after it waits for the load)
    return x[a.base + (int64_t)c * g.HW + min(max(h, 0), g.H - 1) * g.W + min(max(ww, 0), g.W - 1)];
  }
  __device__ BPre b_pre(int n) const { return BPre{(int64_t)(n < N ? n : 0) * K, n < N}; }
  __device__ float b_load(const BPre& b, int k, bool& ok) const {
    ok = b.ok;
    return w[b.base + k];
  }
  __device__ SPre spre(int, int n, int) const {
    SPre p;
    if (!part && bias) p.b = bias[n];
    return p;
  }
  __device__ void store(int m, int n, float v, int split, const SPre& p) const {
    const int nb = g.fPQ.div(m), pq = m - nb * g.PQ;
    const int64_t idx = ((int64_t)nb * g.K + n) * g.PQ + pq;
    if (part) {
      part[split * ptotal + idx] = v;
      return;
    }
    v += p.b;
    if (relu) v = fmaxf(v, 0.f);
    y[idx] = v;
  }
};

// Data gradient: C[m=(n,h,w)][c] = sum_{k=(kout,r,s)} dy[n,kout,p,q] * w[kout,c,r,s]
//   with p = (h + ph - r*dh)/sh when divisible and in range.
struct ConvDgradOp {
  using SP = SPre;
  static constexpr bool A_MFAST = true;
  static constexpr bool B_NFAST = true;
  int M, N, K;
  ConvG g;
  const float* dy;
  const float* w;
  float* dx;
  const float* mask;
  int mode;
  struct APre { int64_t base; int h, w; bool ok; };
  struct BPre { int n; bool ok; };
  __device__ APre a_pre(int m) const {
    APre a;
    a.ok = m < M;
    const int mm = a.ok ? m : 0;
    const int n = g.fHW.div(mm), hw = mm - n * g.HW;
    a.h = g.fW.div(hw);
    a.w = hw - a.h * g.W;
    a.base = (int64_t)n * g.K * g.PQ;
    return a;
  }
  __device__ float a_load(const APre& a, int k, bool& ok) const {
    const int ko = g.fRS.div(k), rs = k - ko * g.RS;
    const int r = g.fS.div(rs), s = rs - r * g.S;
    const int ph_ = a.h + g.ph - r * g.dh, pw_ = a.w + g.pw - s * g.dw;
    const int p = ph_ >= 0 ? ph_ / g.sh : -1, q = pw_ >= 0 ? pw_ / g.sw : -1;
    ok = a.ok && ph_ >= 0 && pw_ >= 0 && p * g.sh == ph_ && q * g.sw == pw_ && p < g.P && q < g.Q;
    return dy[a.base + (int64_t)ko * g.PQ + min(max(p, 0), g.P - 1) * g.Q + min(max(q, 0), g.Q - 1)];
  }
  __device__ BPre b_pre(int n) const { return BPre{n, n < N}; }
  __device__ float b_load(const BPre& b, int k, bool& ok) const {
    const int ko = g.fRS.div(k), rs = k - ko * g.RS;
    ok = b.ok;
    return w[((int64_t)ko * g.C + (b.ok ? b.n : 0)) * g.RS + rs];
  }
  __device__ int64_t oidx(int m, int n) const {
    const int nb = g.fHW.div(m), hw = m - nb * g.HW;
    return ((int64_t)nb * g.C + n) * g.HW + hw;
  }
  __device__ SPre spre(int m, int n, int) const {
    SPre p;
    const int64_t idx = oidx(m, n);
    if (mask) p.mk = mask[idx];
    if (mode == kAccum) p.old = dx[idx];
    return p;
  }
  __device__ void store(int m, int n, float v, int, const SPre& p) const {
    if (mask && !(p.mk > 0.f)) v = 0.f;
    emit2(dx, oidx(m, n), v, mode, p.old);
  }
};

// Weight gradient: C[kout][n=(c,r,s)] = sum_{k=(n,p,q)} dy[n,kout,p,q] * x[n,c,h,w]
struct ConvWgradOp {
  using SP = SPre;
  static constexpr bool A_MFAST = false;  // consecutive k = consecutive q: coalesced dy rows
  static constexpr bool B_NFAST = false;  // consecutive k: coalesced x rows
  int M, N, K;
  ConvG g;
  const float* dy;
  const float* x;
  float* dw;
  int mode;
  // db != null: GEMM column nw (= C*R*S) is a column of ones, so the same reduction over the
  // B*P*Q pixels also produces the bias gradient (no separate bias_grad launch); N = nw + 1
  float* db = nullptr;
  int nw = 0;
  struct APre { int m; bool ok; };
  struct BPre { int64_t coff; int r, s; bool ok, one; };
  __device__ APre a_pre(int m) const { return APre{m, m < M}; }
  __device__ float a_load(const APre& a, int k, bool& ok) const {
    const int nb = g.fPQ.div(k), pq = k - nb * g.PQ;
    ok = a.ok;
    return dy[((int64_t)nb * g.K + (a.ok ? a.m : 0)) * g.PQ + pq];
  }
  __device__ BPre b_pre(int n) const {
    BPre b;
    b.one = db != nullptr && n == nw;
    b.ok = n < nw;
    const int nn = b.ok ? n : 0;
    const int c = g.fRS.div(nn), rs = nn - c * g.RS;
    b.r = g.fS.div(rs);
    b.s = rs - b.r * g.S;
    b.r *= g.dh;
    b.s *= g.dw;
    b.coff = (int64_t)c * g.HW;
    return b;
  }
  __device__ float b_load(const BPre& b, int k, bool& ok) const {
    const int nb = g.fPQ.div(k), pq = k - nb * g.PQ;
    const int p = g.fQ.div(pq), q = pq - p * g.Q;
    const int h = p * g.sh - g.ph + b.r, ww = q * g.sw - g.pw + b.s;
    ok = b.one || (b.ok && (unsigned)h < (unsigned)g.H && (unsigned)ww < (unsigned)g.W);
    const float v = x[(int64_t)nb * g.C * g.HW + b.coff + min(max(h, 0), g.H - 1) * g.W + min(max(ww, 0), g.W - 1)];
    return b.one ? 1.f : v;
  }
  __device__ SPre spre(int m, int n, int) const {
    SPre p;
    if (mode == kAccum) p.old = (db != nullptr && n == nw) ? db[m] : dw[(int64_t)m * nw + min(n, nw - 1)];
    return p;
  }
  __device__ void store(int m, int n, float v, int, const SPre& p) const {
    if (n == nw) emit2(db, m, v, mode, p.old);  // only reached when db is set (n < N = nw + 1)
    else emit2(dw, (int64_t)m * nw + n, v, mode, p.old);
  }
};

// ------------------------------------------------------------------ 1x1 stride-1 convs
// (ResNet bottlenecks): plain batched GEMMs over (n, hw) with channel-strided operands; no
// im2col index math per element.
struct Conv1x1FwdOp {  // y[n,k,hw] = sum_c x[n,c,hw] w[k,c]
  using SP = SPre;
  static constexpr bool A_MFAST = true;   // consecutive m = consecutive hw
  static constexpr bool B_NFAST = false;  // w rows contiguous along c
  int M, N, K;
  int HW;
  FastDiv fHW;
  const float* x;
  const float* w;
  const float* bias;
  float* y;
  bool relu;
  struct APre { int64_t base; bool ok; };
  struct BPre { int64_t base; bool ok; };
  __device__ APre a_pre(int m) const {
    const int mm = m < M ? m : 0, nb = fHW.div(mm), hw = mm - nb * HW;
    return APre{(int64_t)nb * K * HW + hw, m < M};
  }
  __device__ float a_load(const APre& a, int k, bool& ok) const {
    ok = a.ok;
    return x[a.base + (int64_t)k * HW];
  }
  __device__ BPre b_pre(int n) const { return BPre{(int64_t)(n < N ? n : 0) * K, n < N}; }
  __device__ float b_load(const BPre& b, int k, bool& ok) const {
    ok = b.ok;
    return w[b.base + k];
  }
  __device__ SPre spre(int, int n, int) const {
    SPre p;
    if (bias) p.b = bias[n];
    return p;
  }
  __device__ void store(int m, int n, float v, int, const SPre& p) const {
    const int nb = fHW.div(m), hw = m - nb * HW;
    v += p.b;
    if (relu) v = fmaxf(v, 0.f);
    y[((int64_t)nb * N + n) * HW + hw] = v;
  }
};

struct Conv1x1DgradOp {  // dx[n,c,hw] = sum_k dy[n,k,hw] w[k,c]
  using SP = SPre;
  static constexpr bool A_MFAST = true;
  static constexpr bool B_NFAST = true;   // w[k, c]: consecutive c contiguous
  int M, N, K;
  int HW;
  FastDiv fHW;
  const float* dy;
  const float* w;
  float* dx;
  const float* mask;
  int mode;
  struct APre { int64_t base; bool ok; };
  struct BPre { int n; bool ok; };
  __device__ APre a_pre(int m) const {
    const int mm = m < M ? m : 0, nb = fHW.div(mm), hw = mm - nb * HW;
    return APre{(int64_t)nb * K * HW + hw, m < M};
  }
  __device__ float a_load(const APre& a, int k, bool& ok) const {
    ok = a.ok;
    return dy[a.base + (int64_t)k * HW];
  }
  __device__ BPre b_pre(int n) const { return BPre{n < N ? n : 0, n < N}; }
  __device__ float b_load(const BPre& b, int k, bool& ok) const {
    ok = b.ok;
    return w[(int64_t)k * N + b.n];
  }
  __device__ int64_t oidx(int m, int n) const {
    const int nb = fHW.div(m), hw = m - nb * HW;
    return ((int64_t)nb * N + n) * HW + hw;
  }
  __device__ SPre spre(int m, int n, int) const {
    SPre p;
    const int64_t idx = oidx(m, n);
    if (mask) p.mk = mask[idx];
    if (mode == kAccum) p.old = dx[idx];
    return p;
  }
  __device__ void store(int m, int n, float v, int, const SPre& p) const {
    if (mask && !(p.mk > 0.f)) v = 0.f;
    emit2(dx, oidx(m, n), v, mode, p.old);
  }
};

bool is_1x1_s1(const ConvShape& s) {
  return s.R == 1 && s.S == 1 && s.str_h == 1 && s.str_w == 1 && s.pad_h == 0 && s.pad_w == 0;
}

// ------------------------------------------------------------------ linear
struct LinFwdOp {  // y[M,N] = x[M,K] w[N,K]^T + b
  using SP = SPre;
  static constexpr bool A_MFAST = false;
  static constexpr bool B_NFAST = false;
  int M, N, K;
  const float* x;
  const float* w;
  const float* b;
  float* y;
  bool relu;
  int mode;
  float* part = nullptr;  // split-K partials (see ConvFwdOp)
  int64_t ptotal = 0;
  struct Pre { int64_t base; bool ok; };
  using APre = Pre;
  using BPre = Pre;
  __device__ Pre a_pre(int m) const { return Pre{(int64_t)(m < M ? m : 0) * K, m < M}; }
  __device__ float a_load(const Pre& a, int k, bool& ok) const {
    ok = a.ok;
    return x[a.base + k];
  }
  __device__ Pre b_pre(int n) const { return Pre{(int64_t)(n < N ? n : 0) * K, n < N}; }
  __device__ float b_load(const Pre& p, int k, bool& ok) const {
    ok = p.ok;
    return w[p.base + k];
  }
  __device__ SPre spre(int m, int n, int split) const {
    SPre p;
    if (part) return p;
    if (b && split == 0) p.b = b[n];
    if (mode == kAccum) p.old = y[(int64_t)m * N + n];
    return p;
  }
  __device__ void store(int m, int n, float v, int split, const SPre& p) const {
    if (part) {
      part[split * ptotal + (int64_t)m * N + n] = v;
      return;
    }
    v += p.b;
    if (relu) v = fmaxf(v, 0.f);
    emit2(y, (int64_t)m * N + n, v, mode, p.old);
  }
};

struct LinDgradOp {  // dx[M,Kin] = dy[M,Nout] w[Nout,Kin]; GEMM N=Kin, K=Nout
  using SP = SPre;
  static constexpr bool A_MFAST = false;
  static constexpr bool B_NFAST = true;
  int M, N, K;
  const float* dy;
  const float* w;
  float* dx;
  const float* mask;
  int mode;
  float* part = nullptr;  // split-K partials (see ConvFwdOp)
  int64_t ptotal = 0;
  const float* amask = nullptr;  // dy masked on load by (amask > 0): the layer's own fused ReLU
  struct APre { int64_t base; bool ok; };
  struct BPre { int n; bool ok; };
  __device__ APre a_pre(int m) const { return APre{(int64_t)(m < M ? m : 0) * K, m < M}; }
  __device__ float a_load(const APre& a, int k, bool& ok) const {
    ok = a.ok && (!amask || amask[a.base + k] > 0.f);  // (amask: off by default)
    return dy[a.base + k];
  }
  __device__ BPre b_pre(int n) const { return BPre{n < N ? n : 0, n < N}; }
  __device__ float b_load(const BPre& b, int k, bool& ok) const {
    ok = b.ok;
    return w[(int64_t)k * N + b.n];
  }
  __device__ SPre spre(int m, int n, int) const {
    SPre p;
    if (part) return p;
    const int64_t idx = (int64_t)m * N + n;
    if (mask) p.mk = mask[idx];
    if (mode == kAccum) p.old = dx[idx];
    return p;
  }
  __device__ void store(int m, int n, float v, int split, const SPre& p) const {
    const int64_t idx = (int64_t)m * N + n;
    if (part) {
      part[split * ptotal + idx] = v;
      return;
    }
    if (mask && !(p.mk > 0.f)) v = 0.f;
    emit2(dx, idx, v, mode, p.old);
  }
};

struct LinWgradOp {  // dw[Nout,Kin] = dy[B,Nout]^T x[B,Kin]; GEMM M=Nout, N=Kin, K=B
  using SP = SPre;
  static constexpr bool A_MFAST = true;
  static constexpr bool B_NFAST = true;
  int M, N, K;
  const float* dy;
  const float* x;
  float* dw;
  int mode;
  const float* amask = nullptr;  // dy masked on load by (amask > 0) (see LinDgradOp)
  struct APre { int m; bool ok; };
  struct BPre { int n; bool ok; };
  __device__ APre a_pre(int m) const { return APre{m < M ? m : 0, m < M}; }
  __device__ float a_load(const APre& a, int k, bool& ok) const {
    ok = a.ok && (!amask || amask[(int64_t)k * M + a.m] > 0.f);  // (amask: off by default)
    return dy[(int64_t)k * M + a.m];
  }
  __device__ BPre b_pre(int n) const { return BPre{n < N ? n : 0, n < N}; }
  __device__ float b_load(const BPre& b, int k, bool& ok) const {
    ok = b.ok;
    return x[(int64_t)k * N + b.n];
  }
  __device__ SPre spre(int m, int n, int) const {
    SPre p;
    if (mode == kAccum) p.old = dw[(int64_t)m * N + n];
    return p;
  }
  __device__ void store(int m, int n, float v, int, const SPre& p) const { emit2(dw, (int64_t)m * N + n, v, mode, p.old); }
};

int g_gemm_precision = 0;  // 0 = fp32 MFMA (exact), 1 = bf16 operands / fp32 accumulate

template <class Op>
void run(Op& op, int splits, hipStream_t st) {
  if (g_gemm_precision == 1) igemm_bf16_launch<Op, 64, 64, 32, 2, 2>(op, splits, st);
  else igemm_launch<Op, 64, 64, 16, 2, 2>(op, splits, st);
}

// ---------------------------------------------------------------- split-K with partial planes
// Few output tiles over a long reduction (the Keras / MLP layers at batch 64: 9-25 tiles x
// 36-63 k-tiles) leave most CUs idle and serialise the k-loop's load latency (~1 us per k-tile).
// Such GEMMs run split-K: every split stores its raw partial sums to plane part[split][out
// index], and splitk_finish_k sums the planes in a fixed order (deterministic) and applies the
// epilogue (bias, ReLU, ReLU mask, accumulate).  The planes live in one fixed buffer per
// STREAM, allocated on first use and never freed or moved: captured hipGraphs bake its address
// into their kernel arguments (a grow-and-free buffer left replays of an earlier capture
// reading freed memory), and GEMMs issued on two streams at once must not share planes (the
// round-2 side-stream weight-gradient experiment did exactly that with one buffer per device).
// A GEMM whose planes would not fit, or a stream beyond the first kMaxPlaneStreams of a
// device, runs unsplit.
int effective_splits(int K, int splits) {  // what igemm_*_launch will run (every split non-empty)
  const int BK = g_gemm_precision == 1 ? 32 : 16;
  if (splits <= 1) return 1;
  const int klen = cdiv(cdiv(K, splits), BK) * BK;
  return cdiv(K, klen);
}

constexpr size_t kPlaneFloats = size_t(3) << 20;  // 12 MB per stream
constexpr int kMaxPlaneStreams = 8;                // per device

float* splitk_planes(size_t floats, hipStream_t st) {
  static std::mutex mu;
  struct Planes {
    hipStream_t st;
    int dev;
    float* p;
  };
  static std::vector<Planes> bufs;  // never freed (a handle reused by a new stream reuses them)
  if (floats > kPlaneFloats) return nullptr;
  int dev = 0;
  MX_HIP_CHECK(hipStreamGetDevice(st, &dev));
  std::lock_guard<std::mutex> lk(mu);
  int on_dev = 0;
  for (const auto& b : bufs) {
    if (b.st == st && b.dev == dev) return b.p;
    on_dev += b.dev == dev;
  }
  if (on_dev >= kMaxPlaneStreams) return nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  MX_HIP_CHECK(hipStreamIsCapturing(st, &cs));
  if (cs != hipStreamCaptureStatusNone) return nullptr;  // no allocation inside a capture
  int cur = 0;
  float* p = nullptr;
  MX_HIP_CHECK(hipGetDevice(&cur));
  MX_HIP_CHECK(hipSetDevice(dev));
  MX_HIP_CHECK(hipMalloc(&p, kPlaneFloats * sizeof(float)));
  MX_HIP_CHECK(hipSetDevice(cur));
  bufs.push_back({st, dev, p});
  return p;
}

// out[i] = epilogue(sum_s part[s][i]); bias channel of i = (i / inner) % C
__global__ void splitk_finish_k(const float* __restrict__ part, int splits, int total, float* __restrict__ out,
                                const float* __restrict__ bias, int C, int inner, int relu,
                                const float* __restrict__ mask, int accumulate) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    // four independent partial sums (loads in flight together), combined in a fixed order
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int sp = 0;
    for (; sp + 4 <= splits; sp += 4) {
      a0 += part[(int64_t)sp * total + i];
      a1 += part[(int64_t)(sp + 1) * total + i];
      a2 += part[(int64_t)(sp + 2) * total + i];
      a3 += part[(int64_t)(sp + 3) * total + i];
    }
    for (; sp < splits; ++sp) a0 += part[(int64_t)sp * total + i];
    float v = (a0 + a1) + (a2 + a3);
    if (bias) v += bias[(i / inner) % C];
    if (relu) v = fmaxf(v, 0.f);
    if (mask && !(mask[i] > 0.f)) v = 0.f;
    if (accumulate) v += out[i];
    out[i] = v;
  }
}

// Split factor for a GEMM of `tiles` output tiles over K: only when the tiles alone leave the
// chip mostly idle and each split keeps >= 64 reduction elements (4 f32 k-tiles).
int partial_splits(int tiles, int K) {
  if (tiles >= 192 || K < 128) return 1;
  return pick_splits(tiles, K, 64, 512);
}

// Runs `op` split-K into partial planes and finishes into `out` (total outputs); false if no
// split applies or no planes are available (the caller then runs it unsplit).
template <class Op>
bool run_partial(Op& op, int64_t total, float* out, const float* bias, int C, int inner, bool relu,
                 const float* mask, bool accumulate, hipStream_t st) {
  const int tiles = cdiv(op.M, 64) * cdiv(op.N, 64);
  // <= ~1 M partial floats (a plane per split is written and read once more by the finish
  // pass) and <= max(16, total / 256) planes (each finish thread sums the planes of one output:
  // MNIST fc1's 8 K outputs over 128 planes left the finish 32 blocks with long loops, 13 us)
  const int cap = (int)std::max<int64_t>(
      2, std::min<int64_t>((1 << 20) / std::max<int64_t>(total, 1), std::max<int64_t>(16, total / 256)));
  const int splits = effective_splits(op.K, std::min(cap, partial_splits(tiles, op.K)));
  if (splits <= 1 || total >= (1ll << 31) || total * splits > (1ll << 28)) return false;
  float* part = splitk_planes((size_t)total * splits, st);
  if (!part) return false;
  op.part = part;
  op.ptotal = total;
  run(op, splits, st);
  MX_LAUNCH(splitk_finish_k, dim3((unsigned)std::min<int64_t>((total + 255) / 256, 1024)), dim3(256), 0, st,
            part, splits, (int)total, out, bias, C, inner, relu ? 1 : 0, mask, accumulate ? 1 : 0);
  return true;
}

}  // namespace

// Allocate the split-K partial planes of `st` now (outside any capture): a stream that will
// capture a hipGraph gets its planes before the capture, so the captured GEMMs run split.
void reserve_splitk_planes(hipStream_t st) { (void)splitk_planes(kPlaneFloats, st); }

namespace {
int g_conv_algo = 0;  // set_conv_algo(): 0 = Winograd where eligible, 1 = direct
bool use_wino(const ConvShape& s) { return g_gemm_precision == 0 && g_conv_algo == 0 && wino_eligible(s); }
}  // namespace

void set_conv_algo(int a) {
  MX_CHECK(a == 0 || a == 1, "conv algo: 0 (auto: Winograd where eligible) or 1 (direct)");
  g_conv_algo = a;
}
int conv_algo() { return g_conv_algo; }

// dgrad of a stride-1 convolution = forward convolution of dy with the flipped, transposed
// filters w'[c][k][R-1-r][S-1-s] and padding R-1-p (conv2d_dgrad uses it when it is allowed a
// scratch buffer and needs no ReLU mask / accumulation): the forward gather is much cheaper
// than the generic dgrad gather with its stride / divisibility tests.
bool dgrad_as_fwd(const ConvShape& s) {
  return s.str_h == 1 && s.str_w == 1 && s.dil_h == 1 && s.dil_w == 1 && !(s.R == 1 && s.S == 1) &&
         s.pad_h <= s.R - 1 && s.pad_w <= s.S - 1;
}

__global__ void flip_transpose_any_k(const float* __restrict__ w, float* __restrict__ wt, int K, int C, int RS) {
  const int64_t total = (int64_t)K * C * RS;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int tap = (int)(i % RS);
    const int64_t kc = i / RS;
    const int c = (int)(kc % C), k = (int)(kc / C);
    wt[((int64_t)c * K + k) * RS + (RS - 1 - tap)] = w[i];
  }
}

// dgrad of a 3x3 / stride-2 / pad-1 conv = the stride-1 transposed conv of dy zero-inserted to
// the input resolution (u[2p][2q] = dy[p][q], zeros elsewhere):
//   dx[h] = sum_r dy[(h + 1 - r) / 2] w[r] = sum_r' u[h - 1 + r'] w[2 - r'],
// i.e. exactly the stride-1 Winograd data gradient of shape (N, C, H, W, K) run on u.  4x the
// ideal MFMA work, but through the 2.25x-cheaper Winograd kernel instead of the generic dgrad
// gather that multiplies 3 of every 4 taps by zero anyway.
ConvShape s2_as_s1(const ConvShape& s) { return ConvShape::make(s.N, s.C, s.H, s.W, s.K, 3, 3, 1, 1, 1, 1); }

bool wino_s2_dgrad(const ConvShape& s) {
  return g_gemm_precision == 0 && g_conv_algo == 0 && s.R == 3 && s.S == 3 && s.str_h == 2 && s.str_w == 2 &&
         s.pad_h == 1 && s.pad_w == 1 && s.dil_h == 1 && s.dil_w == 1 && s.H == s.W && s.H % 2 == 0 &&
         s.P * 2 == s.H && s.Q * 2 == s.W && wino_eligible(s2_as_s1(s));
}

__global__ void zero_insert2_k(const float* __restrict__ dy, float* __restrict__ u, int64_t planes, int P, int Q) {
  const int H = 2 * P, W = 2 * Q;
  const int64_t total = planes * H * W;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int w = (int)(i % W);
    const int64_t r = i / W;
    const int h = (int)(r % H);
    const int64_t pl = r / H;
    u[i] = ((h | w) & 1) ? 0.f : dy[(pl * P + (h >> 1)) * Q + (w >> 1)];
  }
}

size_t conv_scratch_floats(const ConvShape& s) {
  size_t n = dgrad_as_fwd(s) ? (size_t)s.K * s.C * s.R * s.S : 0;
  if (wino_s2_dgrad(s)) {
    const ConvShape t = s2_as_s1(s);
    n = std::max(n, wino_scratch_floats(t) + (size_t)s.N * s.K * s.H * s.W);
  }
  if (g_gemm_precision != 0) return n;
  if (wino_eligible(s)) n = std::max(n, wino_scratch_floats(s));
  if (conv3x3_eligible(s)) n = std::max(n, (size_t)s.K * s.C * 9);
  return n;
}

size_t conv_dgrad_filter_floats(const ConvShape& s) { return use_wino(s) ? wino_dgrad_filter_floats(s) : 0; }
size_t conv_fwd_filter_floats(const ConvShape& s) { return use_wino(s) ? wino_fwd_filter_floats(s) : 0; }

void conv2d_fwd(const float* x, const float* w, const float* bias, float* y, const ConvShape& s,
                bool relu, hipStream_t st, float* scratch, float* dgrad_filters, bool pretransformed,
                const float* in_ss, bool in_relu) {
  MX_CHECK(!pretransformed || (scratch && use_wino(s)), "conv2d_fwd: pretransformed filters need the Winograd path");
  MX_CHECK(!in_ss || (scratch && use_wino(s)), "conv2d_fwd: a folded BN input needs the Winograd path");
  if (scratch && use_wino(s))
    return wino_fwd(x, w, bias, y, s, relu, scratch, st, dgrad_filters, pretransformed, in_ss, in_relu);
  if (g_gemm_precision == 0 && conv3x3_eligible(s)) return conv3x3_fwd(x, w, bias, y, s, relu, st);
  if (is_1x1_s1(s)) {
    Conv1x1FwdOp op{s.N * s.H * s.W, s.K, s.C, s.H * s.W, FastDiv(s.H * s.W), x, w, bias, y, relu};
    return run(op, 1, st);
  }
  ConvFwdOp op{s.N * s.P * s.Q, s.K, s.C * s.R * s.S, ConvG(s), x, w, bias, y, relu};
  if (run_partial(op, (int64_t)s.N * s.K * s.P * s.Q, y, bias, s.K, s.P * s.Q, relu, nullptr, false, st)) return;
  op.part = nullptr;
  run(op, 1, st);
}

void conv2d_dgrad(const float* dy, const float* w, float* dx, const ConvShape& s,
                  const float* relu_mask, bool accumulate, hipStream_t st, float* wt_scratch, bool pretransformed) {
  if (wt_scratch && use_wino(s))
    return wino_dgrad(dy, w, dx, s, relu_mask, accumulate, wt_scratch, st, pretransformed);
  if (wt_scratch && g_gemm_precision == 0 && conv3x3_eligible(s))
    return conv3x3_dgrad(dy, w, dx, s, relu_mask, accumulate, wt_scratch, st);
  if (wt_scratch && wino_s2_dgrad(s)) {
    const ConvShape t = s2_as_s1(s);
    float* u = wt_scratch + wino_scratch_floats(t);
    const int64_t total = (int64_t)s.N * s.K * s.H * s.W;
    MX_LAUNCH(zero_insert2_k, dim3((unsigned)std::min<int64_t>((total + 255) / 256, 4096)), dim3(256), 0, st, dy, u,
              (int64_t)s.N * s.K, s.P, s.Q);
    return wino_dgrad(u, w, dx, t, relu_mask, accumulate, wt_scratch, st);
  }
  if (wt_scratch && !relu_mask && !accumulate && dgrad_as_fwd(s)) {
    const int64_t total = (int64_t)s.K * s.C * s.R * s.S;
    MX_LAUNCH(flip_transpose_any_k, dim3((unsigned)std::min<int64_t>((total + 255) / 256, 2048)), dim3(256), 0, st, w,
              wt_scratch, s.K, s.C, s.R * s.S);
    const ConvShape t = ConvShape::make(s.N, s.K, s.P, s.Q, s.C, s.R, s.S, 1, 1, s.R - 1 - s.pad_h, s.S - 1 - s.pad_w);
    ConvFwdOp op{t.N * t.P * t.Q, t.K, t.C * t.R * t.S, ConvG(t), dy, wt_scratch, nullptr, dx, false};
    if (run_partial(op, (int64_t)t.N * t.K * t.P * t.Q, dx, nullptr, 1, 1, false, nullptr, false, st)) return;
    op.part = nullptr;
    return run(op, 1, st);
  }
  if (is_1x1_s1(s)) {
    Conv1x1DgradOp op{s.N * s.H * s.W, s.C, s.K, s.H * s.W, FastDiv(s.H * s.W), dy, w, dx, relu_mask,
                      accumulate ? kAccum : kStore};
    return run(op, 1, st);
  }
  ConvDgradOp op{s.N * s.H * s.W, s.C, s.K * s.R * s.S, ConvG(s), dy, w, dx, relu_mask,
                 accumulate ? kAccum : kStore};
  run(op, 1, st);
}

size_t conv_wgrad_scratch_floats(const ConvShape& s) { return use_wino(s) ? wino_wgrad_scratch_floats(s) : 0; }

bool conv2d_wgrad(const float* dy, const float* x, float* dw, const ConvShape& s, bool accumulate,
                  hipStream_t st, float* scratch, float* db, const float* in_ss, bool in_relu) {
  const bool wino = use_wino(s) && (scratch || wino_wgrad_scratch_floats(s) == 0);
  MX_CHECK(!in_ss || wino, "conv2d_wgrad: a folded BN input needs the Winograd path");
  if (wino) {
    wino_wgrad(dy, x, dw, s, accumulate, scratch, st, in_ss, in_relu);
    return false;
  }
  if (g_gemm_precision == 0 && conv3x3_wgrad_eligible(s)) {
    conv3x3_wgrad(dy, x, dw, s, accumulate, st);
    return false;
  }
  ConvWgradOp op{s.K, s.C * s.R * s.S, s.N * s.P * s.Q, ConvG(s), dy, x, dw, kAtomic};
  op.nw = op.N;
  if (db) {  // bias gradient as the extra column of ones
    op.db = db;
    op.N = op.nw + 1;
  }
  const int tiles = cdiv(op.M, 64) * cdiv(op.N, 64);
  const int splits = pick_splits(tiles, op.K, tiles < 64 ? 128 : 512, 768);
  if (splits == 1) {
    op.mode = accumulate ? kAccum : kStore;
  } else if (!accumulate) {
    zero_fill(dw, (int64_t)op.M * op.nw, st);
    if (db) zero_fill(db, op.M, st);
  }
  run(op, splits, st);
  return db != nullptr;
}

void linear_fwd(const float* x, const float* w, const float* b, float* y, int M, int N, int K,
                bool relu, hipStream_t st) {
  LinFwdOp op{M, N, K, x, w, b, y, relu, kStore};
  if (run_partial(op, (int64_t)M * N, y, b, N, 1, relu, nullptr, false, st)) return;
  op.part = nullptr;
  const int tiles = cdiv(M, 64) * cdiv(N, 64);
  int splits = relu ? 1 : pick_splits(tiles, K, 256, 256);
  if (splits > 1) {
    op.mode = kAtomic;
    zero_fill(y, (int64_t)M * N, st);
  }
  run(op, splits, st);
}

void linear_dgrad(const float* dy, const float* w, float* dx, int M, int N, int K,
                  const float* relu_mask, bool accumulate, hipStream_t st, const float* dy_mask) {
  // GEMM view: M x K(out=Kin) reduction over N(out features)
  LinDgradOp op{M, K, N, dy, w, dx, relu_mask, accumulate ? kAccum : kStore};
  op.amask = dy_mask;
  if (run_partial(op, (int64_t)M * K, dx, nullptr, 1, 1, false, relu_mask, accumulate, st)) return;
  op.part = nullptr;
  run(op, 1, st);
}

void linear_wgrad(const float* dy, const float* x, float* dw, int M, int N, int K, bool accumulate,
                  hipStream_t st, const float* dy_mask) {
  LinWgradOp op{N, K, M, dy, x, dw, kStore};
  op.amask = dy_mask;
  const int tiles = cdiv(N, 64) * cdiv(K, 64);
  const int splits = pick_splits(tiles, M, 256, 512);
  if (splits == 1) {
    op.mode = accumulate ? kAccum : kStore;
  } else {
    op.mode = kAtomic;
    if (!accumulate) zero_fill(dw, (int64_t)N * K, st);
  }
  run(op, splits, st);
}

void set_gemm_precision(int p) {
  MX_CHECK(p == 0 || p == 1, "gemm precision: 0 (fp32) or 1 (bf16)");
  g_gemm_precision = p;
}
int gemm_precision() { return g_gemm_precision; }

}  // namespace mx
