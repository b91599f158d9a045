// Fused gfx950 kernels for the training step of the reference's TF2 Keras CNN
// (tensorflow2/mnist_single.py:16-26; MirroredStrategy parity, BASELINE config 4):
//   Conv2D(32,3)+ReLU -> MaxPool2 -> Conv2D(64,3)+ReLU -> MaxPool2 -> Conv2D(64,3)+ReLU ->
//   Flatten -> Dense(64)+ReLU -> Dense(10) -> softmax + sparse CE, Adam (Keras epsilon-hat).
// See keras_kernels.hip for the step map.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "peer.h"

namespace mx {

// Flat parameter layout = KerasCNN state_dict order (models/keras_cnn.py).
struct KerasLayout {
  static constexpr size_t w1 = 0, b1 = 288, w2 = 320, b2 = 18752, w3 = 18816, b3 = 55680, fw1 = 55744,
                          fb1 = 92608, fw2 = 92672, fb2 = 93312, total = 93322;
  static size_t workspace_bytes(int B);
};

struct KerasFused {
  int B;
  float* x;          // [B][784]
  int32_t* y;        // [B]
  float* p;          // flat params (KerasLayout)
  float* g;          // flat grads (written by the finalize in DDP mode)
  float* p1;         // [B][32][169] pooled conv1 output (post-ReLU)
  uint8_t* q1;       // [B][32][169] argmax code (2*dy + dx) inside each 2x2 window
  float* p2;         // [B][64][25] pooled conv2 output (post-ReLU)
  uint8_t* q2;       // [B][64][25]
  float* x3;         // [B][576] conv3 output (post-ReLU) = fc1 input
  float* h1;         // [B][64] fc1 output (post-ReLU)
  float* dl;         // [B][16] dlogits (10 used)
  float* dh1;        // [B][64] grad wrt fc1 pre-activation
  float* dx3;        // [B][576] grad wrt conv3 pre-activation
  float* dp2;        // [B][64][25] grad wrt the pooled conv2 output, ReLU-masked
  float* sv;         // [B][256] per-image bias grads: conv2 @0, conv3 @64, fc1 @128, fc2 @192
  float* pl1;        // [4B][320] conv1 weight+bias grad partial planes
  float* pl2;        // [B][18432] conv2 weight grad planes (one per image)
  float* pl3;        // [B/8][36864] conv3 weight grad planes (one per 8-image group)
  float* pf1;        // [B/8][36864] fc1 weight grad planes
  float* gf2;        // [640] fc2 weight grad
  float* w2f;        // conv2 weights as forward MFMA B fragments [4 co-group][72 k-step][64 lane]
  float* w2d;        // conv2 weights as data-gradient B fragments [2 ci-half][4 wave][36 k-step][64 lane]
  float* metrics;    // [0] loss sum, [1] correct count
  int32_t* counter;  // synthetic-data batch counter
  const float* tmpl; // class templates [10][784]
  uint64_t seed;
  int synth;         // 1: KF1 generates the batch; 0: x / y provided
  // Adam (Keras / Chainer epsilon-hat form when eps_hat): m, v flat; state = {steps, ticket}
  float* m;
  float* v;
  const float* lr;
  int32_t* adam_state;
  float b1, b2, eps, wd;
  int eps_hat;
};

// mode 0: finalize grads + Adam + weight packing (no gradient collectives);
// 1: finalize into g only (DDP: g is all-reduced next); 2: Adam from g (scaled by gscale) +
// packing; 3: packing only (after an external weight load)
void keras_fused_forward(const KerasFused& f, hipStream_t st);   // KF1 + KF2
void keras_fused_backward(const KerasFused& f, hipStream_t st);  // KB1
void keras_fused_update(const KerasFused& f, int mode, float gscale, hipStream_t st);  // KO
// KX (DDP over the peer transport): the one-shot gradient exchange co-scheduled with Adam --
// replaces the bucket all-reduce and mode 2 (a: PeerComm::oneshot_args of g)
void keras_fused_exchange_adam(const KerasFused& f, const PeerArgs& a, hipStream_t st);
int keras_exchange_blocks();

}  // namespace mx
