// Native data-parallel training step for the reference's Chainer MLP (chainer/train_mnist.py:
// 13-26,69; ParallelUpdater parity at chainer/train_mnist_gpu.py:87-93): on-device batch, the 5
// fused launches of mlp_kernels.hip with Chainer Adam folded into the gradient kernels at
// world size 1, or -- with gradient collectives -- the gradients in two buckets ([l2, l3] ready
// after K4, overlappable with K5; [l1] after K5) all-reduced over RCCL or the xGMI peer
// transport, then the flat Adam.  Issued from C++ on one stream and captured into hipGraphs.
// Parameters, gradients and Adam moments are flat fp32 buffers in MLP state_dict order owned by
// the Python side (mxddp/mlp_engine.py).
#pragma once
#include <hip/hip_runtime.h>

#include <memory>

#include "comm.h"
#include "graph_runner.h"
#include "mlp_kernels.h"
#include "reducer.h"

namespace mx {

class MlpEngine {
 public:
  MlpEngine(int batch, uintptr_t params, uintptr_t grads, uintptr_t m, uintptr_t v, uintptr_t adam_state,
            uintptr_t workspace, size_t workspace_bytes, Comm* comm, uint64_t seed, uintptr_t lr_dev,
            uintptr_t metrics_dev, float b1, float b2, float eps, float weight_decay, bool eps_hat);
  ~MlpEngine();
  MlpEngine(const MlpEngine&) = delete;
  MlpEngine& operator=(const MlpEngine&) = delete;

  static size_t workspace_bytes(int B);
  void step();                                   // one eager step on stream()
  // mode 1: whole step(s), collectives included, in one graph per steps_per_graph steps;
  // mode 0: eager launches
  void capture(int mode, int steps_per_graph);
  void replay(int n);
  void uncapture();
  int warm_graphs() { return graphs_.warm(); }
  void sync();
  int graph_mode() const { return graphs_.captured() ? 1 : 0; }
  bool captured() const { return graphs_.captured(); }

  // DDP launch strategy (world size > 1); each drops captured graphs
  void set_peer(PeerComm* p);
  void set_comm(Comm* c);
  void set_force_collectives(bool on);
  void set_merged(bool on);   // one all-reduce of the whole gradient after K5
  void set_overlap(bool on);  // bucket 0 on the side stream, overlapping K5
  void set_bucket_padding(size_t capacity, size_t multiple);
  bool merged() const { return merged_; }
  bool overlap() const { return !merged_ && reducer_->overlap(); }
  int world_size() const;
  bool reducer_active() const { return reducer_->active(); }
  bool peer_active() const { return reducer_->peer() != nullptr; }

  void set_external_batch(bool on) { external_ = on; }
  uintptr_t stream() const { return reinterpret_cast<uintptr_t>(s_); }
  uintptr_t x_ptr() const { return reinterpret_cast<uintptr_t>(f_.x); }
  uintptr_t y_ptr() const { return reinterpret_cast<uintptr_t>(f_.y); }
  uintptr_t counter_ptr() const { return reinterpret_cast<uintptr_t>(f_.counter); }

 private:
  void launch_step();
  MlpFused args() const;
  Reducer& red() const { return merged_ ? *merged_reducer_ : *reducer_; }
  int B_;
  MlpFused f_{};
  Comm* comm_;
  uint64_t seed_;
  bool external_ = false, merged_ = false;
  hipStream_t s_ = nullptr;
  std::unique_ptr<Reducer> reducer_;         // [l2.w .. l3.b] then [l1.w, l1.b]
  std::unique_ptr<Reducer> merged_reducer_;  // the whole gradient
  GraphRunner graphs_;
};

}  // namespace mx
