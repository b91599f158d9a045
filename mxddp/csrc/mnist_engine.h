// Native data-parallel training step for the north-star MNIST CNN
//   conv(1->32,3)+ReLU -> conv(32->64,3)+ReLU -> maxpool2 -> fc(9216->128)+ReLU -> fc(128->10)
//   -> log_softmax + NLL (mean), SGD(momentum, weight decay)
// (north star op list in BASELINE.json).
//
// The whole step -- on-device synthetic batch, forward, backward, bucketed RCCL gradient
// all-reduce on a side stream overlapped with the conv backward, and the fused flat SGD
// update -- is issued from C++ into one HIP stream pair and captured ONCE into a hipGraph;
// every training step is then a single graph launch (no Python, no host sync).
//
// Parameters / grads / momentum are three flat fp32 buffers in PyTorch state_dict order
// (conv1.weight, conv1.bias, conv2.weight, conv2.bias, fc1.weight, fc1.bias, fc2.weight,
// fc2.bias) owned by the Python side, so checkpoints keep the reference layout
// (pytorch/distributed_data_parallel.py:103-115).
#pragma once
#include <hip/hip_runtime.h>

#include <functional>
#include <memory>
#include <utility>
#include <vector>

#include "comm.h"
#include "mnist_kernels.h"
#include "reducer.h"

namespace mx {

struct MnistLayout {
  static constexpr int kC1 = 32, kC2 = 64, kH = 28, kH1 = 26, kH2 = 24, kHP = 12, kF1 = 128, kNC = 10;
  static constexpr size_t w1 = 0, b1 = 288, w2 = 320, b2 = 18752, fw1 = 18816, fb1 = 1198464, fw2 = 1198592,
                          fb2 = 1199872, total = 1199882;
  static size_t workspace_bytes(int B);
  static int padded(int B) { return (B + 15) / 16 * 16; }  // rows of the fused kernels' buffers
};

class MnistEngine {
 public:
  MnistEngine(int batch, uintptr_t params, uintptr_t grads, uintptr_t mom, uintptr_t workspace,
              size_t workspace_bytes, Comm* comm, uint64_t seed, float momentum, float weight_decay,
              uintptr_t lr_dev, uintptr_t metrics_dev, int kernel_variant);
  ~MnistEngine();

  void step();               // one training step, eager launches on stream()
  // Record the step into hipGraph(s) (call after a warm-up step).  mode 1: one graph for the
  // whole step, RCCL collectives captured inside; mode 2: three compute graphs with the two
  // bucket all-reduces issued eagerly between them; -1: 1 when world_size == 1, else 2.
  // steps_per_graph > 1 (mode 1 only) unrolls that many consecutive steps into one graph, so
  // the per-launch graph overhead is paid once per group (batches, LR and metrics all live in
  // device memory, so every unrolled step is a distinct, correct training step).
  void capture(int mode = -1, int steps_per_graph = 1);
  void replay(int n);        // n steps via the captured graph(s) (eager if not captured)
  // launch every captured graph once (real training steps; returns how many): untimed warm-up
  // of graph execs that a replay would otherwise run for the first time
  int warm_graphs();
  // replay order of a step count that needs several graphs: full groups first, then the
  // remainder graphs largest first (default), or the remainder smallest first (measured: no gain)
  void set_small_first(bool on) { small_first_ = on; }
  int graph_mode() const { return graph_mode_; }
  // captured graphs bake in whether collectives run (and whether F8 folds into the SGD launch):
  // changing it drops them (eager until capture() is called again)
  void set_force_collectives(bool on) {
    if (on != reducer_->forced()) uncapture();
    reducer_->set_force_collectives(on);
    merged_reducer_->set_force_collectives(on);
    co_reducer_->set_force_collectives(on);
  }
  void set_overlap(bool on) { reducer_->set_overlap(on); }  // see Reducer::set_overlap
  // gradient transport: nullptr = RCCL, else the direct xGMI peer all-reduce (peer.h); drops
  // captured graphs (they bake in the collective kernels)
  void set_peer(PeerComm* p) {
    if (p != reducer_->peer()) uncapture();
    reducer_->set_peer(p);
    merged_reducer_->set_peer(p);
    co_reducer_->set_peer(p);
    if (coscheduled_) set_coscheduled(true);  // re-derive the exchange arguments (or drop it)
  }
  // RCCL communicator (same rank / world size; one of the configured variants of
  // parallel/comm.py); drops captured graphs
  void set_comm(Comm* c);
  // pad the all-reduce of a bucket that ends at the end of the gradient buffer up to a multiple
  // of `multiple` elements, into zeroed slack (capacity = elements the grads buffer really has)
  void set_bucket_padding(size_t capacity, size_t multiple) {
    reducer_->set_padding(MnistLayout::total, capacity, multiple);
    merged_reducer_->set_padding(MnistLayout::total, capacity, multiple);
  }
  // merged = true: ONE all-reduce over the whole gradient after the conv backward instead of
  // the fc bucket (overlappable) + the conv bucket: one collective latency per step instead of
  // two, no overlap.  Drops captured graphs.
  void set_merged(bool on) {
    if (on != merged_) uncapture();
    merged_ = on;
  }
  bool merged() const { return merged_; }
  // co-scheduled = true (peer transport only): the fc bucket's two-shot exchange runs in the
  // first blocks of the conv-backward launch itself (overlapping it without a second stream);
  // the conv bucket follows after F8.  Drops captured graphs.  False if the transport cannot.
  bool set_coscheduled(bool on);
  bool coscheduled() const { return co_active(); }
  bool peer_active() const { return reducer_->peer() != nullptr; }
  // data-parallel degree: the RCCL communicator's, else the peer transport's (a peer-only job,
  // e.g. several ranks sharing one GPU in tests)
  int world_size() const {
    return comm_ ? comm_->world_size() : (reducer_->peer() ? reducer_->peer()->world_size() : 1);
  }
  bool overlap() const { return !merged_ && reducer_->overlap(); }
  bool reducer_active() const { return reducer_->active(); }
  void uncapture();  // drop captured graphs (back to eager; capture() may be called again)
  void forward_only(uintptr_t x, uintptr_t logits, int B);  // eval helper (no grads)
  void sync();
  // Re-derive the fused path's packed weights / accumulators after the parameters were changed
  // outside the engine (checkpoint load, broadcast).
  void repack();
  uintptr_t stream() const { return reinterpret_cast<uintptr_t>(s_); }
  uintptr_t x_ptr() const { return reinterpret_cast<uintptr_t>(x_); }
  uintptr_t y_ptr() const { return reinterpret_cast<uintptr_t>(y_); }
  // synthetic-data stream position (4 x int32 Philox counter): saved in the resume state
  uintptr_t counter_ptr() const { return reinterpret_cast<uintptr_t>(counter_); }
  void set_external_batch(bool on) { external_batch_ = on; }
  // in-kernel phase timestamps (MnistFused::trace); 0 = off.  Eager steps only: a captured
  // graph keeps the arguments it was captured with.
  void set_trace(uintptr_t buf) { trace_ = reinterpret_cast<uint32_t*>(buf); }
  float last_comm_ms() { return reducer_ ? red().last_comm_ms() : 0.f; }
  bool captured() const { return exec_ != nullptr || seg_exec_[0] != nullptr; }

 private:
  Reducer& red() const { return merged_ ? *merged_reducer_ : *reducer_; }
  void launch_step();
  void segment(int k);
  MnistFused fused_args() const;
  hipGraphExec_t capture_fn(const std::function<void()>& fn, hipGraph_t* g);
  hipGraph_t seg_graph_[3] = {nullptr, nullptr, nullptr};
  hipGraphExec_t seg_exec_[3] = {nullptr, nullptr, nullptr};
  int graph_mode_ = 0;
  uint32_t* trace_ = nullptr;
  int steps_per_graph_ = 1;
  bool small_first_ = false;
  void fwd(const float* x, float* logits_out, int B);
  int B_;   // batch
  int Bp_;  // rows of the workspace buffers (fused variant: B_ rounded up to 16)
  float *p_, *g_, *m_;
  float *x_, *a1_, *c2_, *pool_, *h_, *logits_, *dlogits_, *dh_, *dp_, *dc2_, *da1_, *tmpl_, *scratch_;
  int32_t *y_, *idx_, *counter_;
  float *lr_, *metrics_;
  bool co_active() const {
    return coscheduled_ && variant_ == 1 && reducer_->peer() != nullptr && reducer_->active();
  }
  bool coscheduled_ = false;
  PeerArgs co_args_{};
  PeerPartition co_part_{};
  std::unique_ptr<Reducer> co_reducer_;  // the conv bucket alone (the fc bucket rides F67)
  Comm* comm_;
  std::unique_ptr<Reducer> reducer_;         // buckets [fc1.w .. fc2.b], [conv1.w .. conv2.b]
  std::unique_ptr<Reducer> merged_reducer_;  // one bucket: the whole flat gradient
  bool merged_ = false;
  uint64_t seed_;
  float momentum_, wd_;
  int variant_;
  bool external_batch_ = false;
  hipStream_t s_ = nullptr;
  hipGraph_t graph_ = nullptr;
  hipGraphExec_t exec_ = nullptr;
  // mode 1, steps_per_graph > 1: graphs of 2^k < steps_per_graph steps for the remainder of a
  // replay(n) (largest first), so a step count that is not a multiple of the group size still
  // runs entirely from graphs
  std::vector<std::pair<int, hipGraphExec_t>> rem_exec_;
  std::vector<hipGraph_t> rem_graph_;
};

}  // namespace mx
