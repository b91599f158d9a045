// Host-callable launchers for every mxddp HIP kernel (fp32 unless noted).
// All pointers are device pointers; all launches are asynchronous on `st` and
// graph-capturable (no allocation, no synchronisation inside).
#pragma once
#include <vector>
#include <hip/hip_runtime.h>

#include <cstdint>

namespace mx {

struct ConvShape {
  int N, C, H, W;        // input
  int K, R, S;           // filters
  int P, Q;              // output spatial
  int str_h, str_w, pad_h, pad_w, dil_h, dil_w;
  static ConvShape make(int N, int C, int H, int W, int K, int R, int S, int sh, int sw, int ph,
                        int pw, int dh = 1, int dw = 1) {
    ConvShape c{N, C, H, W, K, R, S, 0, 0, sh, sw, ph, pw, dh, dw};
    c.P = (H + 2 * ph - dh * (R - 1) - 1) / sh + 1;
    c.Q = (W + 2 * pw - dw * (S - 1) - 1) / sw + 1;
    return c;
  }
};

// ---- GEMM-shaped (ops_gemm.hip) ----
// dgrad_filters (optional, conv_dgrad_filter_floats(s) floats; 0 = not applicable): the forward
// also prepares the filters the Winograd data gradient will use (pass them to conv2d_dgrad with
// pretransformed = true)
// in_ss (optional, [C][2]): the input is a folded BN's output, relu?(x * scale[c] + shift[c]),
// formed while the input tile is staged (Winograd path only; padding stays zero)
void conv2d_fwd(const float* x, const float* w, const float* bias, float* y, const ConvShape& s,
                bool relu, hipStream_t st, float* scratch = nullptr, float* dgrad_filters = nullptr,
                bool pretransformed = false, const float* in_ss = nullptr, bool in_relu = false);
size_t conv_dgrad_filter_floats(const ConvShape& s);
// forward Winograd filter floats (0 = this conv does not run the Winograd path)
size_t conv_fwd_filter_floats(const ConvShape& s);
// dx = conv_transpose(dy, w) [* (mask > 0)], stored (=) or accumulated (+=).  `wt_scratch`
// (conv_scratch_floats(s) floats, optional) enables the Winograd / direct 3x3 paths.
void conv2d_dgrad(const float* dy, const float* w, float* dx, const ConvShape& s,
                  const float* relu_mask, bool accumulate, hipStream_t st, float* wt_scratch = nullptr,
                  bool pretransformed = false);
// Direct-LDS 3x3 stride-1 pad-1 convolution (conv3x3.hip), fp32 MFMA; W <= 64.
bool conv3x3_eligible(const ConvShape& s);
void conv3x3_fwd(const float* x, const float* w, const float* bias, float* y, const ConvShape& s, bool relu,
                 hipStream_t st);
void conv3x3_dgrad(const float* dy, const float* w, float* dx, const ConvShape& s, const float* relu_mask,
                   bool accumulate, float* wt_scratch, hipStream_t st);
bool conv3x3_wgrad_eligible(const ConvShape& s);  // + W % 4 == 0
void conv3x3_wgrad(const float* dy, const float* x, float* dw, const ConvShape& s, bool accumulate, hipStream_t st);
// Fused Winograd F(2x2,3x3) on fp32 MFMA (winograd.hip): 3x3 s1 p1, square 8/16/32 images.
// `scratch` holds the transformed filters: wino_scratch_floats(s) floats.
bool wino_eligible(const ConvShape& s);
size_t wino_scratch_floats(const ConvShape& s);
// U_dgrad_out (optional, wino_dgrad_filter_floats(s)): also write the data-gradient filters
// pretransformed: `scratch` already holds the forward filters (WinoFilterBank / an earlier call)
void wino_fwd(const float* x, const float* w, const float* bias, float* y, const ConvShape& s, bool relu,
              float* scratch, hipStream_t st, float* U_dgrad_out = nullptr, bool pretransformed = false,
              const float* in_ss = nullptr, bool in_relu = false);
size_t wino_dgrad_filter_floats(const ConvShape& s);
size_t wino_fwd_filter_floats(const ConvShape& s);
// Persistent Winograd filters of many 3x3 convs, re-transformed by ONE launch per <= 64 convs
// after each optimizer step (the layer path's per-conv forward transform launches disappear).
class WinoFilterBank {
 public:
  void add(const float* w, float* U_fwd, float* U_dgrad, int K, int C);  // U_dgrad may be null
  void clear() { jobs_.clear(); }
  size_t size() const { return jobs_.size(); }
  void refresh(hipStream_t st) const;

 private:
  struct Job {
    const float* w;
    float* Uf;
    float* Ud;
    int K, C;
  };
  std::vector<Job> jobs_;
};
// pretransformed: `scratch` already holds the filters written by wino_fwd(..., U_dgrad_out)
void wino_dgrad(const float* dy, const float* w, float* dx, const ConvShape& s, const float* relu_mask,
                bool accumulate, float* scratch, hipStream_t st, bool pretransformed = false);
// partial-sum scratch: wino_wgrad_scratch_floats(s) floats (0 = none needed)
size_t wino_wgrad_scratch_floats(const ConvShape& s);
void wino_wgrad_set_slots(int per_cu);  // weight-gradient blocks aimed at per CU (3)
void wino_wgrad(const float* dy, const float* x, float* dw, const ConvShape& s, bool accumulate, float* scratch,
                hipStream_t st, const float* in_ss = nullptr, bool in_relu = false);
// 3x3 s1 algorithm: 0 = auto (Winograd where eligible, else direct-LDS), 1 = direct-LDS only.
void set_conv_algo(int a);
int conv_algo();
// floats of scratch conv2d_fwd / conv2d_dgrad can use for this shape (0 = none needed)
size_t conv_scratch_floats(const ConvShape& s);
// dw (+)= sum_{n,p,q} dy * im2col(x)
// db (optional): the bias gradient sum_{n,p,q} dy is produced by the same GEMM (an extra column of
// ones) where the generic path runs; returns whether it did (else the caller runs bias_grad)
// in_ss: as conv2d_fwd's (the input recomputed from the folded BN's input; Winograd path only)
bool conv2d_wgrad(const float* dy, const float* x, float* dw, const ConvShape& s, bool accumulate,
                  hipStream_t st, float* scratch = nullptr, float* db = nullptr, const float* in_ss = nullptr,
                  bool in_relu = false);
size_t conv_wgrad_scratch_floats(const ConvShape& s);
// y[M,N] = x[M,K] @ w[N,K]^T + b  (optional ReLU)
void linear_fwd(const float* x, const float* w, const float* b, float* y, int M, int N, int K,
                bool relu, hipStream_t st);
// dx[M,K] (+)= dy[M,N] @ w[N,K]  [* (mask > 0)]
// dy_mask (optional, [M,N]): dy is used as dy * (dy_mask > 0) -- the layer's own fused ReLU,
// applied on load instead of a separate relu_bwd pass (also for linear_wgrad / bias_grad)
void linear_dgrad(const float* dy, const float* w, float* dx, int M, int N, int K,
                  const float* relu_mask, bool accumulate, hipStream_t st, const float* dy_mask = nullptr);
// dw[N,K] (+)= dy[M,N]^T @ x[M,K]
void linear_wgrad(const float* dy, const float* x, float* dw, int M, int N, int K, bool accumulate,
                  hipStream_t st, const float* dy_mask = nullptr);

// GEMM operand precision for every op above: 0 = fp32 MFMA (exact fp32, default),
// 1 = bf16 operands with fp32 accumulation (mixed precision; fp32 tensors in memory).
void set_gemm_precision(int p);
int gemm_precision();

// ---- elementwise / reductions (ops_elementwise.hip) ----
// fp32 <-> bf16 (round to nearest even) for bf16 gradient communication (grad_cast.hip)
void cast_f32_bf16(const float* x, uint16_t* y, int64_t n, hipStream_t st);
void cast_bf16_f32(const uint16_t* x, float* y, int64_t n, hipStream_t st);
void relu_fwd(const float* x, float* y, int64_t n, hipStream_t st);
void relu_bwd(const float* dy, const float* y, float* dx, int64_t n, hipStream_t st);
// db[c] (+)= sum over (outer, inner) of dy[outer][c][inner]
void bias_grad(const float* dy, float* db, int outer, int C, int inner, bool accumulate,
               hipStream_t st, const float* dy_mask = nullptr);
void add_inplace(float* y, const float* x, int64_t n, hipStream_t st);
// p[0..n) = 0 by a kernel (not a memset node inside captured graphs)
void zero_fill(float* p, int64_t n, hipStream_t st);
void scale_inplace(float* y, float a, int64_t n, hipStream_t st);
void fill(float* y, float v, int64_t n, hipStream_t st);

// maxpool 2D (NCHW); idx stores the flat argmax offset inside the input plane.
void maxpool2d_fwd(const float* x, float* y, int32_t* idx, int N, int C, int H, int W, int kh, int kw,
                   int sh, int sw, int ph, int pw, int P, int Q, hipStream_t st);
// sh, sw > 0: the windows do not overlap (kernel == stride, no padding) -> gather, no zero fill
void maxpool2d_bwd(const float* dy, const int32_t* idx, float* dx, int N, int C, int H, int W, int P,
                   int Q, hipStream_t st, int sh = 0, int sw = 0);
// avgpool 2D (count_include_pad=True semantics of nn.AvgPool2d, ceil_mode clipping)
void avgpool2d_fwd(const float* x, float* y, int N, int C, int H, int W, int kh, int kw, int sh, int sw,
                   int ph, int pw, int P, int Q, hipStream_t st);
void avgpool2d_bwd(const float* dy, float* dx, int N, int C, int H, int W, int kh, int kw, int sh,
                   int sw, int ph, int pw, int P, int Q, hipStream_t st);

// Fused log_softmax + NLL (mean) forward + backward in one pass.
//  logits [B,C] -> loss_sum (atomic += sum of -logp[y]), correct (atomic += #argmax==y),
//  dlogits = (softmax - onehot) * grad_scale  (if dlogits != nullptr), logp (optional).
// `probs_input`=true treats logits as already-softmaxed probabilities (Keras softmax head).
// loss_scale multiplies each row's loss before the sum (1 / B: loss_sum is the mean).
void xent_fwd_bwd(const float* logits, const int32_t* y, float* logp, float* dlogits,
                  float* loss_sum, float* correct, int B, int C, float grad_scale, hipStream_t st,
                  float loss_scale = 1.f);

// BatchNorm2d (training): batch stats, running-stat update, normalise (+ optional ReLU).
// Split reduction (ops_bn.hip): S x C workgroups write partial sums to `part`
// (bn_partial_floats(N, C, HW) floats, fully rewritten by every call), the elementwise pass sums
// its channel's partials in a fixed order (deterministic, no atomics).
int bn_splits(int N, int C, int HW);
size_t bn_partial_floats(int N, int C, int HW);
void bn_fwd_train(const float* x, const float* gamma, const float* beta, float* y, float* mean,
                  float* invstd, float* run_mean, float* run_var, int N, int C, int HW,
                  float momentum, float eps, bool relu, float* part, hipStream_t st,
                  int64_t* num_batches = nullptr,  // num_batches: += 1 on device
                  const float* residual = nullptr, int residual_C = 0,  // y[:, :Cr] += residual
                  // y == nullptr: no apply pass -- the statistics and the per-channel (scale, shift)
                  // pairs [C][2] go to ss_out for a convolution that applies them to its input
                  float* ss_out = nullptr);
void bn_fwd_eval(const float* x, const float* gamma, const float* beta, float* y,
                 const float* run_mean, const float* run_var, int N, int C, int HW, float eps,
                 bool relu, hipStream_t st);
void bn_bwd(const float* dy, const float* x, const float* y_relu, const float* gamma,
            const float* mean, const float* invstd, float* dx, float* dgamma, float* dbeta, int N,
            int C, int HW, bool accumulate_params, float* part, hipStream_t st,
            const float* extra = nullptr, int extra_C = 0,  // dx += extra[:, :C] ([N][extra_C][HW])
            // the fused ReLU's mask recomputed from x and the forward's (scale, shift) pairs
            // (y_relu == nullptr: the output was never stored)
            const float* ss_mask = nullptr);

// PyramidNet shortcut: y[n,c,:,:] += (c < Cin ? pool(x)[n,c] : 0); pool = 2x2 avg, ceil.
void shortcut_pad_add(const float* x, float* y, int N, int Cin, int H, int W, int Cout, int P, int Q,
                      int stride, hipStream_t st);
void shortcut_pad_add_bwd(const float* dy, float* dx, int N, int Cin, int H, int W, int Cout, int P,
                          int Q, int stride, bool accumulate, hipStream_t st);

// ---- channels-last bf16 path (nhwc_bf16.hip): activations bf16 [N][H][W][C], C % 8 == 0 ----
void nhwc_from_nchw(const float* x, uint16_t* y, int N, int C, int H, int W, int Cp, hipStream_t st);
// wt (or null): fwd layout bf16 [K][R][S][Cp] (channel-padded); wtd (or null): dgrad layout bf16 [C][R][S][K]
void nhwc_repack_weight(const float* w, uint16_t* wt, uint16_t* wtd, int K, int C, int R, int S, int Cp,
                        hipStream_t st);
// all convolutions of a model in one launch: desc = device int64 [n][8] rows {w, wt, wtd (or 0), K,
// C, R*S, Cp, first block}, first blocks = prefix sums of nhwc_repack_blocks(...)
int nhwc_repack_blocks(int K, int C, int R, int S, int Cp, bool fwd, bool dgrad);
// rows of BN partial sums a forward conv's epilogue may write (size of nhwc_conv_fwd's bnpart / 2K)
int nhwc_conv_bn_rows(int N, int H, int W, int Cp, int K, int R, int S, int sh, int sw, int ph, int pw, int P, int Q);
void nhwc_repack_many(const int64_t* desc, int n, int total_blocks, hipStream_t st);
// scratch (or null = no split-K): nhwc_conv_scratch_floats(M = output pixels, Ng = output
// channels, Kg = R*S*input channels) floats of fp32 split-K partials
size_t nhwc_conv_scratch_floats(int M, int Ng, int Kg);
// bnpart (optional, [nhwc_conv_bn_rows][2K] floats): the output feeds a training BatchNorm; the
// epilogue (LDS-DMA / band / stem kernels, unsplit) or the split-K reduce writes the BN partial
// sums of (y - bnshift[c]) there and the call returns the number of rows written (pass them to
// nhwc_bn_fwd), else 0
int nhwc_conv_fwd(const uint16_t* x, const uint16_t* wt, uint16_t* y, int N, int H, int W, int Cp, int K, int R,
                  int S, int sh, int sw, int ph, int pw, int P, int Q, float* scratch, hipStream_t st,
                  float* bnpart = nullptr, const float* bnshift = nullptr);
// large-layer LDS-DMA conv kernel: 0 = off, 1 = large layers (default), 2 = always
void nhwc_conv_set_glds(int mode);
// the 256 x 256-tile LDS-DMA kernel: 0 = off, 1 = layers with >= 256 tiles and >= 4 k-tiles (default), 2 = wherever Ng % 256 == 0
void nhwc_conv_set_glds256(int mode);
void nhwc_wgrad_set_waves8(int on);  // 8-wave 128-row weight-gradient tiles (A/B)
void nhwc_conv_set_glds_deep(int mode);
void nhwc_conv_set_glds_par(int on);  // stride-2 data gradients on the two-stage LDS-DMA tiles  // 128 x 128 LDS-DMA tiles for deep reductions on few tiles
void nhwc_conv_set_gk2(int mode);  // two-stage 128 x 128 tiles: 0 = 8 waves of 64 x 32, 1 = gk2 (64 x 64 wave tiles, k-groups) 16x16x32, 2 = gk2 32x32x16
void nhwc_conv_set_glds_short(int mode);  // two-stage 128-pixel LDS-DMA variant for short reductions
void nhwc_conv_set_split_blocks(int n);  // generic conv kernel: split-K below this many blocks (256)
void nhwc_wgrad_set_target(int n);  // weight gradient: blocks aimed at when splitting the pixels (512)
void nhwc_wgrad_set_small_npix(int n);  // layers of <= n pixels with >= 32 planes aim at half of it (25,088)
void nhwc_wgrad_set_tile256(int on);  // weight gradient: 256 x 256 tiles where K and R*S*C reach 256 (1)
void nhwc_bn_set_grid_cap(int cap);
void nhwc_bn_set_wt(int on);
void nhwc_conv_set_wt(int on);  // conv epilogue outputs stored write-through (A/B)  // BN apply passes: outputs stored write-through (A/B)  // most blocks of the NHWC BN apply kernels (A/B; 2048 = round-3 grids)
// split-K scratch of nhwc_conv_dgrad (floats; 0 = none needed)
size_t nhwc_conv_dgrad_scratch_floats(int N, int H, int W, int C, int K, int R, int S, int sh, int sw, int ph, int pw,
                                      int P, int Q);
// addend (optional, bf16 [N][H][W][C]): dx = conv_transpose(dy) + addend, summed in the epilogue.
// bnpart / bx / bmean (optional): dx is the output gradient of a training BatchNorm with input bx
// and batch mean bmean (ReLU mask from bfcoef or bmask when brelu): the epilogue writes that BN's
// backward partial sums to bnpart (at most nhwc_conv_dgrad_bn_rows rows of 2 C floats).  Returns
// the rows written (0: the kernel chosen for this shape cannot, the BN runs its own pass).
// amask: the addend is masked by these ReLU bits (bit e of byte i / 8 for element i) before the add.
// addend_sub: the addend is [N][H / 2][W / 2][C] and is added at even (h, w) only (1x1 layers).
int nhwc_conv_dgrad(const uint16_t* dy, const uint16_t* wt_d, uint16_t* dx, int N, int H, int W, int C, int K, int R,
                    int S, int sh, int sw, int ph, int pw, int P, int Q, float* scratch, hipStream_t st,
                    const uint16_t* addend = nullptr, float* bnpart = nullptr, const uint16_t* bx = nullptr,
                    const float* bmean = nullptr, const float* bfcoef = nullptr, const uint8_t* bmask = nullptr,
                    bool brelu = false, const uint8_t* amask = nullptr, bool addend_sub = false);
int nhwc_conv_dgrad_bn_rows(int N, int H, int W, int C, int K, int R, int S, int sh, int sw, int ph, int pw, int P,
                            int Q);
// dw fp32 [K][Cin][R][S] (+)= ...; x has Cp >= Cin channels (padding ignored);
// scratch: nhwc_wgrad_scratch_floats(...) floats of per-split partial sums
size_t nhwc_wgrad_scratch_floats(int N, int Cp, int K, int R, int S, int P, int Q);
void nhwc_conv_wgrad(const uint16_t* dy, const uint16_t* x, float* dw, int N, int H, int W, int Cin, int Cp, int K,
                     int R, int S, int sh, int sw, int ph, int pw, int P, int Q, bool accumulate, float* scratch,
                     hipStream_t st);
// y = relu?(bn(x) + res); scratch: nhwc_bn_scratch_floats(Npix, C) floats (partial sums +
// per-channel coefficients, fully rewritten by every call)
size_t nhwc_bn_scratch_floats(int Npix, int C);
void nhwc_bn_fwd(const uint16_t* x, const uint16_t* res, uint16_t* y, const float* gamma, const float* beta,
                 float* mean, float* invstd, float* run_mean, float* run_var, int64_t* num_batches, int Npix, int C,
                 float momentum, float eps, bool relu, float* scratch, hipStream_t st,
                 float* coef_out = nullptr,  // coef_out: [C][2] (scale, shift) kept for nhwc_bn_bwd
                 uint8_t* mask_out = nullptr,  // ReLU mask bits [Npix * C / 8] for nhwc_bn_bwd
                 // partial sums already written by the producing conv (nhwc_conv_fwd's bnpart)
                 const float* pre_part = nullptr, int pre_gx = 0, const float* kshift = nullptr);
void nhwc_bn_bwd(const uint16_t* dy, const uint16_t* x, const uint16_t* y, const float* gamma, const float* mean,
                 const float* invstd, uint16_t* dx, uint16_t* dres, float* dgamma, float* dbeta, int Npix, int C,
                 bool relu, bool accumulate_params, float* scratch, hipStream_t st,
                 const float* fcoef = nullptr, const uint8_t* mask = nullptr,
                 // backward partial sums already written by the consuming conv's data-gradient
                 // epilogue (nhwc_conv_dgrad's bnpart): the statistics pass over dy and x is skipped
                 const float* pre_part = nullptr, int pre_gx = 0);  // fcoef: the forward's coef_out (ReLU, no residual,
                                                 // C <= 512): mask from x, y not read
void nhwc_maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* arg, int N, int H, int W, int C, int P, int Q, int k,
                      int s, int p, hipStream_t st);
void nhwc_maxpool_bwd(const uint16_t* dy, const uint8_t* arg, uint16_t* dx, int N, int H, int W, int C, int P, int Q,
                      int k, int s, int p, hipStream_t st);
void nhwc_gap_fwd(const uint16_t* x, float* y, int N, int HW, int C, hipStream_t st);
void nhwc_gap_bwd(const float* dy, uint16_t* dx, int N, int HW, int C, hipStream_t st);

// split-K partial planes of a stream, allocated ahead of a graph capture on it (ops_gemm.hip)
void reserve_splitk_planes(hipStream_t st);

// ---- optimizers (ops_optim.hip): flat multi-tensor, fp32 master ----
// SGD (PyTorch semantics): g' = g*gscale + wd*p; buf = mom*buf + g' (buf=g' at first step); p -= lr*buf
// `lr` is read from device memory so a captured graph follows LR schedules.
void sgd_step(float* p, const float* g, float* buf, const float* lr, float gscale, float momentum,
              float wd, int64_t n, bool first_step, hipStream_t st);
// Adam (PyTorch semantics, or Keras / Chainer eps_hat), bias-corrected.  `state` = int32[2]
// device words {completed steps, arrival ticket (0 between launches)}: the kernel advances the
// step count itself, so a captured graph needs no host value per step.
void adam_step(float* p, const float* g, float* m, float* v, const float* lr, int32_t* state,
               float gscale, float b1, float b2, float eps, float wd, bool eps_hat, int64_t n, hipStream_t st);

// ---- data (ops_data.hip) ----
// Class-conditional synthetic images: x = 0.5*template[y] + 0.5*noise, y ~ U{0..C-1}.
// Deterministic in (seed, counter[0]); counter is incremented on device after each batch.
void synth_batch(float* x, int32_t* y, const float* templates, int B, int D, int C, uint64_t seed,
                 int32_t* counter, hipStream_t st, bool bump = true);
void synth_templates(float* templates, int C, int D, uint64_t seed, hipStream_t st);
// On-device CIFAR-style augmentation: random crop (pad 4) + h-flip + normalize (NCHW).
void augment_crop_flip_norm(const float* x, float* y, int N, int C, int H, int W, int pad,
                            const float* mean, const float* std, uint64_t seed, int32_t* counter,
                            hipStream_t st);
// argmax(logits)==y counts (metrics)
void count_correct(const float* logits, const int32_t* y, float* correct, int B, int C, hipStream_t st);

}  // namespace mx
