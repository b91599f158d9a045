// Fused CDNA4 kernels for the MNIST CNN training step (see mnist_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "peer.h"

namespace mx {

struct MnistFused {
  int B;                 // rows of every [B] buffer: the batch rounded up to the 16-row MFMA tile
  int nB;                // the real batch (loss / accuracy / 1/B); rows nB.. get zero loss gradient
  float* x;              // [B,1,28,28]
  int32_t* y;            // [B]
  float* p;              // flat params (MnistLayout offsets)
  float* g;              // flat grads
  float* a1;             // [B,32,26,26] post-ReLU conv1
  float* pool;           // [B,64,12,12] post-ReLU pooled conv2
  int32_t* idx;          // used as uint8 [B,64,12,12]: argmax 0..3 inside the 2x2 window, 4 = dead
  // [B,128] fc1 pre-activation as int64 fixed point (kHScale): F3's split-K partials are added
  // with 64-bit integer atomics, so the sum is exact and independent of their order
  long long* h;
  float* dh;             // [B,128] grad wrt fc1 pre-activation
  float* dp;             // [B,9216] grad wrt pooled activation (0 on dead windows)
  float* scratch;        // packed weights + accumulators
  float* metrics;        // [0] loss sum, [1] correct count (accumulated on device)
  int32_t* counter;      // synthetic-data batch counter
  const float* tmpl;     // class templates [10][784] for the on-device generator
  uint64_t seed;         // per-rank generator seed
  uint32_t* trace;       // optional per-phase timestamps (s_memrealtime, 100 MHz) for profiling, or null
  int synth;             // 1: F2 generates the batch on device; 0: x/y provided by the caller
  // fc1-weight SGD folded into F5 (no gradient collectives in the step): each F5 block updates
  // the weight columns whose gradient it just produced (the gradient is not written to g), and
  // the SGD launch skips them
  int fc1_sgd;
  // with fc1_sgd: F5 only computes dp (+ the head) and publishes dh; the fc1 weight gradient and
  // its SGD update run in extra blocks at the end of the conv-backward launch (F67), which take
  // the CU slots its data-gradient blocks free first (the next step's F3 is the first reader of
  // the updated weights)
  int fc1_defer;
  // conv-backward launch (F67) block order: 1 = the XCD-aware placement of f67_role (set by the
  // launcher for the batch-64 three-blocks-per-CU grid), 0 = the plain [F6W | F7W | fc1] order
  int f67_order;
  float* mom;            // flat momentum buffer
  const float* lr;       // device learning rate
  float sgd_mom, sgd_wd;
  // co-scheduled fc-bucket exchange: blocks [0, co_blocks) of the conv-backward launch run the
  // two-shot peer all-reduce of the fc gradients (ready since F5), the rest the conv work
  int co_blocks;
  PeerArgs co_args;
  PeerPartition co_part;
  // bulk outputs written with agent-scope (sc1: not kept dirty in the XCD's L2) stores, per
  // kernel: 1 = F5 (fc1 weights / momentum / dp), 2 = F2 (a1, pool), 4 = F6W (weight slabs)
  int wt;
};
size_t mnist_fused_scratch_floats(int B);
void mnist_set_wt_stores(int mask);  // process-wide default of MnistFused::wt
// process-wide default of MnistFused::fc1_defer (world size 1): 0 off, 1 fc1 blocks after F7W's
// in the two-block-per-CU F67, 2 the three-block-per-CU F67 (single V buffer) with them resident
void mnist_set_fc1_defer(int mode);
int mnist_fc1_defer();
// F67 block placement (MnistFused::f67_order) where the launcher can apply it: 1 on, 0 off
void mnist_set_f67_order(int on);
int mnist_f67_order();
int mnist_wt_stores();

// Pack conv2 weights into the F2 Winograd fragment order and zero the cross-step accumulators;
// needed once and after any change of the parameters outside the fused SGD.
void mnist_fused_init(const MnistFused& f, hipStream_t st);
void mnist_fused_forward(const MnistFused& f, hipStream_t st);  // F2 + F3
void mnist_fused_fc1_bwd(const MnistFused& f, hipStream_t st);  // F5 (head + fc1 backward)
// F6 + F7 (+ F8 unless `finalize_in_sgd`: then mnist_fused_sgd(..., finalize = true) does F8's work)
void mnist_fused_conv_bwd(const MnistFused& f, hipStream_t st, bool finalize_in_sgd = false);
void mnist_fused_sgd(const MnistFused& f, float* mom_buf, const float* lr, float gscale, float momentum, float wd,
                     hipStream_t st, bool finalize = false);

}  // namespace mx
