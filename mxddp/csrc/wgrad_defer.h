// Deferred weight-gradient reductions (the launch floor of the layer-path steps).
//
// The split-K weight-gradient kernels (Winograd wgrad: winograd.hip; channels-last bf16 wgrad:
// nhwc_bf16.hip) write fp32 partial planes that a second, tiny launch sums into dW -- one reduce
// launch per convolution per step (PyramidNet-110: ~100, ResNet-50: 53), each a few us plus a
// kernel boundary.  When the destination is a flat gradient buffer that the optimizer reads
// only at its step, the reduction can wait: the wgrad call records a job instead of launching,
// and the optimizer flushes every pending job of its device in a few batched launches (job table
// by value in the kernel arguments, graph-capturable), before the update.  The per-element
// arithmetic is the single-job kernels', so the gradients are bitwise identical.
//
// The Python layer opts a call in (thread-local flag around one wgrad call whose partial-plane
// scratch it keeps alive until the flush); nothing defers unless asked.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace mx {

struct RedJob {
  const float* part;
  float* dw;
  int64_t plane, pstride;  // kind 0: plane floats / plane stride; kind 1: plane = float4 quads
  int nplanes, G, acc, kind;
  int Kout, Ng, Ca, Cin, RS;  // kind 1: [K][(r, s, c)] -> [K][C][R][S] scatter
  int blocks, blk0;
};
constexpr int kRedMaxJobs = 40;
struct RedBatch {
  RedJob j[kRedMaxJobs];
  int n;
};

void wgrad_defer_set(bool on);  // this thread's next wgrad calls may defer (until reset)
bool wgrad_defer_active();
bool wgrad_defer_took();        // the last wgrad call on this thread recorded a job
void wgrad_defer_push(const RedJob& j);  // under the current HIP device
int wgrad_defer_flush(hipStream_t st);   // the current device's jobs, in order; returns how many
int wgrad_defer_pending();               // jobs pending on the current device

void wino_reduce_batch_launch(const RedBatch& b, int blocks, hipStream_t st);  // winograd.hip
void nhwc_reduce_batch_launch(const RedBatch& b, int blocks, hipStream_t st);  // nhwc_bf16.hip

}  // namespace mx
