// Fused gfx950 kernels for the training step of the reference's Chainer MLP
// (chainer/train_mnist.py:13-26,69: 784 -> 1000 -> 1000 -> 10, ReLU, softmax cross entropy,
// Chainer Adam = epsilon-hat Adam).  See mlp_kernels.hip for the step map.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace mx {

constexpr int kMlpMaxBatch = 512;  // per device; batches need not be multiples of the 16-row tile

// Flat parameter layout = MLP state_dict order (models/mlp.py: l1, l2, l3 weight / bias).
struct MlpLayout {
  static constexpr int kIn = 784, kH = 1000, kHP = 1024, kNC = 10;
  static constexpr size_t w1 = 0, b1 = 784000, w2 = 785000, b2 = 1785000, w3 = 1786000, b3 = 1796000,
                          total = 1796010;
};

struct MlpFused {
  int B;             // batch (rows that count: loss, accuracy, 1/B)
  int Bp;            // B rounded up to the 16-row MFMA tile: every [B]-shaped buffer below has Bp
                     // rows; rows B.. carry zero loss gradient, so they add nothing to any sum
  float* x;          // [B][784]
  int32_t* y;        // [B]
  float* p;          // flat params (MlpLayout)
  float* g;          // flat grads (written when the gradient is all-reduced before Adam)
  float* h1;         // [B][1024] l1 output (post-ReLU); columns 1000.. are zero
  float* h2;         // [B][1024] l2 output (post-ReLU); columns 1000.. are zero
  float* dl;         // [B][16] dlogits (10 used)
  float* dh2;        // [B][1024] grad wrt the l2 pre-activation; columns 1000.. are zero
  float* dh1p;       // [4][B][1024] l2 data-gradient partials of the 4 row slices of W2 (unmasked)
  float* lsum;       // [B/16][2] per-row-tile loss / correct sums (K3)
  float* metrics;    // [0] loss sum, [1] correct count (accumulated on the device)
  int32_t* counter;  // synthetic-data batch counter
  const float* tmpl; // class templates [10][784]
  uint64_t seed;     // per-rank generator seed
  int synth;         // 1: K1 generates the batch; 0: x / y provided by the caller
  // 1: Adam fused into the gradient kernels (no gradient collectives); 0: gradients go to g
  // (all-reduced next) and the flat Adam kernel updates afterwards
  int fused_adam;
  float* m;
  float* v;
  const float* lr;
  int32_t* adam_state;  // {completed steps, step being applied}: see ops_optim.hip adam_k
  float b1, b2, eps, wd;
  int eps_hat;
  // 1: the dW2 tile + its update run as extra resident blocks of K5 (not in K4), shortening the
  // dgrad chain K4 -> K5; set by the engine when the l2 gradient need not be ready after K4
  int w2_defer;
};

void mlp_fused_forward(const MlpFused& f, hipStream_t st);    // K1, K2, K3
void mlp_fused_backward2(const MlpFused& f, hipStream_t st);  // K4: l2 / l3 gradients (+ Adam) -> bucket 0
void mlp_fused_backward1(const MlpFused& f, hipStream_t st);  // K5: l1 gradients (+ Adam)      -> bucket 1
// process-wide switch of MlpFused::w2_defer (default off; the engine applies it with fused Adam
// or a single merged gradient bucket)
void mlp_set_w2_defer(int on);
int mlp_w2_defer();

}  // namespace mx
