// Elementwise, pooling, loss and normalisation kernels (fp32, NCHW).
// Replace ATen/cuDNN kernels reached by the reference through nn.ReLU, nn.MaxPool2d /
// AvgPool2d (pytorch/model.py:11,76; tensorflow2/mnist_single.py:19,21), F.pad +
// residual add (pytorch/model.py:18,49), nn.BatchNorm2d (pytorch/model.py:27-33),
// and CrossEntropyLoss / log_softmax+NLL (pytorch/single_gpu.py:70).
#include "common.h"
#include "ops.h"

namespace mx {
namespace {

constexpr int kTB = 256;

inline int grid_for(int64_t n, int per_thread = 1) {
  int64_t g = (n + (int64_t)kTB * per_thread - 1) / ((int64_t)kTB * per_thread);
  if (g > 4096) g = 4096;  // grid-stride beyond ~16 blocks/CU
  return g < 1 ? 1 : (int)g;
}

__global__ void relu_fwd_k(const float* __restrict__ x, float* __restrict__ y, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = fmaxf(x[i], 0.f);
}
__global__ void relu_bwd_k(const float* __restrict__ dy, const float* __restrict__ y, float* __restrict__ dx,
                           int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dx[i] = y[i] > 0.f ? dy[i] : 0.f;
}
__global__ void add_k(float* __restrict__ y, const float* __restrict__ x, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] += x[i];
}
__global__ void scale_k(float* __restrict__ y, float a, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] *= a;
}
__global__ void fill_k(float* __restrict__ y, float v, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = v;
}

// Bias gradient db[c] = sum over (outer, inner) of dy[outer][C][inner], fixed summation order
// (deterministic).  inner > 1 (conv): one 1024-thread block per channel, the flattened
// (outer, inner) index split with a 32-bit magic division (a 64-bit divide per element made this
// 17 us per call for the Keras CNN's conv1), eight loads in flight per thread.  inner == 1
// (linear): a block covers 64 channels with its 4 waves taking every 4th row, partials combined
// through LDS in a fixed order.
constexpr int kBgTB = 1024, kBgU = 8;
__global__ __launch_bounds__(kBgTB) void bias_grad_k(const float* __restrict__ dy, float* __restrict__ db, int outer,
                                                     int C, int inner, FastDiv dv, int accumulate) {
  const int c = blockIdx.x;
  const int total = outer * inner;
  float s[kBgU];
#pragma unroll
  for (int k = 0; k < kBgU; ++k) s[k] = 0.f;
  int i = threadIdx.x;
  for (; i + (kBgU - 1) * kBgTB < total; i += kBgU * kBgTB) {
#pragma unroll
    for (int k = 0; k < kBgU; ++k) {
      const int j = i + k * kBgTB, o = (int)dv.div((uint32_t)j), in = j - o * inner;
      s[k] += dy[((size_t)o * C + c) * inner + in];
    }
  }
  for (; i < total; i += kBgTB) {
    const int o = (int)dv.div((uint32_t)i), in = i - o * inner;
    s[0] += dy[((size_t)o * C + c) * inner + in];
  }
  float t = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  t = wave_sum(t);
  __shared__ float red[kBgTB / 64];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    float u = 0.f;
#pragma unroll
    for (int w = 0; w < kBgTB / 64; ++w) u += red[w];
    db[c] = accumulate ? db[c] + u : u;
  }
}

__global__ __launch_bounds__(256) void bias_grad_rows_k(const float* __restrict__ dy, float* __restrict__ db, int rows,
                                                        int C, int accumulate, const float* __restrict__ mask) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, c = blockIdx.x * 64 + lane;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  // dy masked by (mask > 0) when given: the layer's fused ReLU, no separate relu_bwd pass
  auto ld = [&](size_t i) { return (mask && !(mask[i] > 0.f)) ? 0.f : dy[i]; };
  if (c < C) {
    int r = w;
    for (; r + 12 < rows; r += 16) {
#pragma unroll
      for (int k = 0; k < 4; ++k) s[k] += ld((size_t)(r + 4 * k) * C + c);
    }
    for (; r < rows; r += 4) s[0] += ld((size_t)r * C + c);
  }
  red[w][lane] = (s[0] + s[1]) + (s[2] + s[3]);
  __syncthreads();
  if (w == 0 && c < C) {
    const float u = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    db[c] = accumulate ? db[c] + u : u;
  }
}

__global__ void maxpool_fwd_k(const float* __restrict__ x, float* __restrict__ y, int32_t* __restrict__ idx,
                              int NC, int H, int W, int kh, int kw, int sh, int sw, int ph, int pw, int P,
                              int Q) {
  const int64_t total = (int64_t)NC * P * Q;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int q = i % Q, p = (i / Q) % P;
    const int64_t nc = i / ((int64_t)P * Q);
    const float* xp = x + nc * H * W;
    float best = -INFINITY;
    int bi = -1;
    const int h0 = p * sh - ph, w0 = q * sw - pw;
    for (int r = 0; r < kh; ++r) {
      const int h = h0 + r;
      if (h < 0 || h >= H) continue;
      for (int s = 0; s < kw; ++s) {
        const int w = w0 + s;
        if (w < 0 || w >= W) continue;
        const float v = xp[h * W + w];
        if (v > best || bi < 0 || isnan(v)) { best = v; bi = h * W + w; }
      }
    }
    y[i] = best;
    idx[i] = bi;
  }
}

// zero fill as a compute kernel: inside a captured hipGraph a memset becomes a separate memset
// node (a copy-engine operation on ROCm); kernels keep every node of a step on the compute queue
__global__ void zero_fill_k(float* __restrict__ p, int64_t n, int vec) {
  const int64_t n4 = vec ? n >> 2 : 0;
  float4* p4 = reinterpret_cast<float4*>(p);
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256)
    p4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t i = 4 * n4 + blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = 0.f;
}

// non-overlapping windows (kernel == stride, no padding): every input element has at most one
// window, so dx is a gather -- every element written once, no zero fill, no atomics
__global__ void maxpool_bwd_gather_k(const float* __restrict__ dy, const int32_t* __restrict__ idx,
                                     float* __restrict__ dx, int total, int H, int W, int P, int Q, FastDiv fW,
                                     FastDiv fH, FastDiv fsh, FastDiv fsw) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int r = (int)fW.div((uint32_t)i), w = i - r * W;
    const int nc = (int)fH.div((uint32_t)r), h = r - nc * H;
    const int p = (int)fsh.div((uint32_t)h), q = (int)fsw.div((uint32_t)w);
    float v = 0.f;
    if (p < P && q < Q) {
      const int o = (nc * P + p) * Q + q;
      if (idx[o] == h * W + w) v = dy[o];
    }
    dx[i] = v;
  }
}

__global__ void maxpool_bwd_k(const float* __restrict__ dy, const int32_t* __restrict__ idx, float* __restrict__ dx,
                              int NC, int H, int W, int P, int Q) {
  const int64_t total = (int64_t)NC * P * Q;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t nc = i / ((int64_t)P * Q);
    atomicAdd(dx + nc * H * W + idx[i], dy[i]);
  }
}

__device__ __forceinline__ void avg_window(int p, int q, int H, int W, int kh, int kw, int sh, int sw, int ph,
                                           int pw, int& hs, int& he, int& ws, int& we, float& inv) {
  hs = p * sh - ph;
  ws = q * sw - pw;
  he = min(hs + kh, H + ph);
  we = min(ws + kw, W + pw);
  const int cnt = (he - hs) * (we - ws);  // count_include_pad=True
  hs = max(hs, 0);
  ws = max(ws, 0);
  he = min(he, H);
  we = min(we, W);
  inv = 1.f / (float)cnt;
}

__global__ void avgpool_fwd_k(const float* __restrict__ x, float* __restrict__ y, int NC, int H, int W, int kh,
                              int kw, int sh, int sw, int ph, int pw, int P, int Q) {
  const int64_t total = (int64_t)NC * P * Q;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int q = i % Q, p = (i / Q) % P;
    const int64_t nc = i / ((int64_t)P * Q);
    int hs, he, ws, we;
    float inv;
    avg_window(p, q, H, W, kh, kw, sh, sw, ph, pw, hs, he, ws, we, inv);
    const float* xp = x + nc * H * W;
    float s = 0.f;
    for (int h = hs; h < he; ++h)
      for (int w = ws; w < we; ++w) s += xp[h * W + w];
    y[i] = s * inv;
  }
}

__global__ void avgpool_bwd_k(const float* __restrict__ dy, float* __restrict__ dx, int NC, int H, int W, int kh,
                              int kw, int sh, int sw, int ph, int pw, int P, int Q) {
  const int64_t total = (int64_t)NC * P * Q;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int q = i % Q, p = (i / Q) % P;
    const int64_t nc = i / ((int64_t)P * Q);
    int hs, he, ws, we;
    float inv;
    avg_window(p, q, H, W, kh, kw, sh, sw, ph, pw, hs, he, ws, we, inv);
    const float g = dy[i] * inv;
    float* dp = dx + nc * H * W;
    for (int h = hs; h < he; ++h)
      for (int w = ws; w < we; ++w) atomicAdd(dp + h * W + w, g);
  }
}

// One wave per row.
__global__ void xent_k(const float* __restrict__ logits, const int32_t* __restrict__ y, float* __restrict__ logp,
                       float* __restrict__ dlogits, float* __restrict__ loss_sum, float* __restrict__ correct,
                       int B, int C, float scale, float loss_scale) {
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= B) return;
  const float* lr = logits + (int64_t)row * C;
  float mx = -INFINITY;
  int am = 0;
  for (int c = lane; c < C; c += 64) {
    const float v = lr[c];
    if (v > mx) { mx = v; am = c; }
  }
  // argmax with first-index tie break (torch.max semantics)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(am, o, 64);
    if (om > mx || (om == mx && oa < am)) { mx = om; am = oa; }
  }
  float se = 0.f;
  for (int c = lane; c < C; c += 64) se += __expf(lr[c] - mx);
  se = wave_sum(se);
  const float lse = mx + __logf(se);
  const int label = y[row];
  if (logp)
    for (int c = lane; c < C; c += 64) logp[(int64_t)row * C + c] = lr[c] - lse;
  if (dlogits)
    for (int c = lane; c < C; c += 64) {
      const float pr = __expf(lr[c] - lse);
      dlogits[(int64_t)row * C + c] = (pr - (c == label ? 1.f : 0.f)) * scale;
    }
  if (lane == 0) {
    if (loss_sum) atomicAdd(loss_sum, (lse - lr[label]) * loss_scale);
    if (correct) atomicAdd(correct, am == label ? 1.f : 0.f);
  }
}

// -------------------------------------------------------------- BatchNorm (per-channel block)
template <int TB>
__device__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int w = 0; w < TB / 64; ++w) t += red[w];
  __syncthreads();
  return t;
}

__global__ void bn_fwd_eval_k(const float* __restrict__ x, const float* __restrict__ gamma,
                              const float* __restrict__ beta, float* __restrict__ y, const float* __restrict__ rm,
                              const float* __restrict__ rv, int N, int C, int HW, float eps, int relu) {
  const int64_t total = (int64_t)N * C * HW;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (i / HW) % C;
    float r = (x[i] - rm[c]) * rsqrtf(rv[c] + eps) * (gamma ? gamma[c] : 1.f) + (beta ? beta[c] : 0.f);
    y[i] = relu ? fmaxf(r, 0.f) : r;
  }
}

// ------------------------------------------------------------- PyramidNet shortcut
__global__ void shortcut_fwd_k(const float* __restrict__ x, float* __restrict__ y, int N, int Cin, int H, int W,
                               int Cout, int P, int Q, int stride) {
  const int64_t total = (int64_t)N * Cin * P * Q;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int q = i % Q, p = (i / Q) % P;
    const int64_t nc = i / ((int64_t)P * Q);
    const int c = nc % Cin, n = nc / Cin;
    const float* xp = x + nc * H * W;
    float v;
    if (stride == 1) {
      v = xp[p * W + q];
    } else {  // AvgPool2d(2,2,ceil_mode=True), count over in-bounds elements
      const int h0 = 2 * p, w0 = 2 * q, h1 = min(h0 + 2, H), w1 = min(w0 + 2, W);
      float s = 0.f;
      for (int h = h0; h < h1; ++h)
        for (int w = w0; w < w1; ++w) s += xp[h * W + w];
      v = s / (float)((h1 - h0) * (w1 - w0));
    }
    y[(((int64_t)n * Cout + c) * P + p) * Q + q] += v;
  }
}

__global__ void shortcut_bwd_k(const float* __restrict__ dy, float* __restrict__ dx, int N, int Cin, int H, int W,
                               int Cout, int P, int Q, int stride, int accumulate) {
  const int64_t total = (int64_t)N * Cin * H * W;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int w = i % W, h = (i / W) % H;
    const int64_t nc = i / ((int64_t)H * W);
    const int c = nc % Cin, n = nc / Cin;
    float g;
    if (stride == 1) {
      g = dy[(((int64_t)n * Cout + c) * P + h) * Q + w];
    } else {
      const int p = h / 2, q = w / 2;
      const int h1 = min(2 * p + 2, H), w1 = min(2 * q + 2, W);
      g = dy[(((int64_t)n * Cout + c) * P + p) * Q + q] / (float)((h1 - 2 * p) * (w1 - 2 * q));
    }
    dx[i] = accumulate ? dx[i] + g : g;
  }
}

}  // namespace

void relu_fwd(const float* x, float* y, int64_t n, hipStream_t st) {
  MX_LAUNCH(relu_fwd_k, dim3(grid_for(n)), dim3(kTB), 0, st, x, y, n);
}
void relu_bwd(const float* dy, const float* y, float* dx, int64_t n, hipStream_t st) {
  MX_LAUNCH(relu_bwd_k, dim3(grid_for(n)), dim3(kTB), 0, st, dy, y, dx, n);
}
void add_inplace(float* y, const float* x, int64_t n, hipStream_t st) {
  MX_LAUNCH(add_k, dim3(grid_for(n)), dim3(kTB), 0, st, y, x, n);
}
void scale_inplace(float* y, float a, int64_t n, hipStream_t st) {
  MX_LAUNCH(scale_k, dim3(grid_for(n)), dim3(kTB), 0, st, y, a, n);
}
void fill(float* y, float v, int64_t n, hipStream_t st) {
  MX_LAUNCH(fill_k, dim3(grid_for(n)), dim3(kTB), 0, st, y, v, n);
}
void bias_grad(const float* dy, float* db, int outer, int C, int inner, bool accumulate, hipStream_t st,
               const float* dy_mask) {
  MX_CHECK((int64_t)outer * inner < (1ll << 31), "bias_grad: reduction too large");
  if (inner == 1) {
    MX_LAUNCH(bias_grad_rows_k, dim3((C + 63) / 64), dim3(256), 0, st, dy, db, outer, C, accumulate ? 1 : 0, dy_mask);
    return;
  }
  MX_CHECK(!dy_mask, "bias_grad: a dy mask is supported for [rows][C] gradients only");
  MX_LAUNCH(bias_grad_k, dim3(C), dim3(kBgTB), 0, st, dy, db, outer, C, inner, FastDiv((uint32_t)inner),
            accumulate ? 1 : 0);
}
void zero_fill(float* p, int64_t n, hipStream_t st) {
  if (n <= 0) return;
  const int vec = (reinterpret_cast<uintptr_t>(p) & 15) == 0;  // float4 body only when aligned
  MX_LAUNCH(zero_fill_k, dim3((unsigned)std::min<int64_t>((n / 4 + 255) / 256 + 1, 2048)), dim3(256), 0, st, p, n,
            vec);
}
void maxpool2d_fwd(const float* x, float* y, int32_t* idx, int N, int C, int H, int W, int kh, int kw, int sh,
                   int sw, int ph, int pw, int P, int Q, hipStream_t st) {
  MX_LAUNCH(maxpool_fwd_k, dim3(grid_for((int64_t)N * C * P * Q)), dim3(kTB), 0, st, x, y, idx, N * C, H,
                     W, kh, kw, sh, sw, ph, pw, P, Q);
}
void maxpool2d_bwd(const float* dy, const int32_t* idx, float* dx, int N, int C, int H, int W, int P, int Q,
                   hipStream_t st, int sh, int sw) {
  if (sh > 0 && sw > 0 && (int64_t)N * C * H * W < (1ll << 31)) {
    const int total = N * C * H * W;
    MX_LAUNCH(maxpool_bwd_gather_k, dim3(grid_for(total)), dim3(kTB), 0, st, dy, idx, dx, total, H, W, P, Q,
              FastDiv(W), FastDiv(H), FastDiv(sh), FastDiv(sw));
    return;
  }
  zero_fill(dx, (int64_t)N * C * H * W, st);
  MX_LAUNCH(maxpool_bwd_k, dim3(grid_for((int64_t)N * C * P * Q)), dim3(kTB), 0, st, dy, idx, dx, N * C,
                     H, W, P, Q);
}
void avgpool2d_fwd(const float* x, float* y, int N, int C, int H, int W, int kh, int kw, int sh, int sw, int ph,
                   int pw, int P, int Q, hipStream_t st) {
  MX_LAUNCH(avgpool_fwd_k, dim3(grid_for((int64_t)N * C * P * Q)), dim3(kTB), 0, st, x, y, N * C, H, W,
                     kh, kw, sh, sw, ph, pw, P, Q);
}
void avgpool2d_bwd(const float* dy, float* dx, int N, int C, int H, int W, int kh, int kw, int sh, int sw, int ph,
                   int pw, int P, int Q, hipStream_t st) {
  zero_fill(dx, (int64_t)N * C * H * W, st);
  MX_LAUNCH(avgpool_bwd_k, dim3(grid_for((int64_t)N * C * P * Q)), dim3(kTB), 0, st, dy, dx, N * C, H, W,
                     kh, kw, sh, sw, ph, pw, P, Q);
}
void xent_fwd_bwd(const float* logits, const int32_t* y, float* logp, float* dlogits, float* loss_sum,
                  float* correct, int B, int C, float grad_scale, hipStream_t st, float loss_scale) {
  const int rows_per_block = 4;
  MX_LAUNCH(xent_k, dim3(cdiv(B, rows_per_block)), dim3(64 * rows_per_block), 0, st, logits, y, logp,
                     dlogits, loss_sum, correct, B, C, grad_scale, loss_scale);
}
void bn_fwd_eval(const float* x, const float* gamma, const float* beta, float* y, const float* rm, const float* rv,
                 int N, int C, int HW, float eps, bool relu, hipStream_t st) {
  MX_LAUNCH(bn_fwd_eval_k, dim3(grid_for((int64_t)N * C * HW)), dim3(kTB), 0, st, x, gamma, beta, y, rm,
                     rv, N, C, HW, eps, relu ? 1 : 0);
}
void shortcut_pad_add(const float* x, float* y, int N, int Cin, int H, int W, int Cout, int P, int Q, int stride,
                      hipStream_t st) {
  MX_LAUNCH(shortcut_fwd_k, dim3(grid_for((int64_t)N * Cin * P * Q)), dim3(kTB), 0, st, x, y, N, Cin, H,
                     W, Cout, P, Q, stride);
}
void shortcut_pad_add_bwd(const float* dy, float* dx, int N, int Cin, int H, int W, int Cout, int P, int Q,
                          int stride, bool accumulate, hipStream_t st) {
  MX_LAUNCH(shortcut_bwd_k, dim3(grid_for((int64_t)N * Cin * H * W)), dim3(kTB), 0, st, dy, dx, N, Cin, H,
                     W, Cout, P, Q, stride, accumulate ? 1 : 0);
}

}  // namespace mx
