// Native data-parallel training step for the reference's TF2 Keras CNN (BASELINE config 4,
// tensorflow2/mnist_mirror_strategy.py:12,68-79): the whole step -- on-device batch, fused
// forward / backward (keras_kernels.hip), the gradient all-reduce when replicas or ranks exist
// (RCCL or the xGMI peer transport, one 373 KB bucket), Adam with its step count on the device
// -- issued from C++ on one stream and captured into hipGraphs, so a training step is one graph
// launch.  Parameters / Adam moments are flat fp32 buffers in KerasCNN state_dict order owned by
// the Python side (mxddp/keras_engine.py).
#pragma once
#include <hip/hip_runtime.h>

#include <memory>
#include <utility>
#include <vector>

#include "comm.h"
#include "keras_kernels.h"
#include "reducer.h"

namespace mx {

class KerasEngine {
 public:
  KerasEngine(int batch, uintptr_t params, uintptr_t grads, uintptr_t m, uintptr_t v, uintptr_t adam_state,
              uintptr_t workspace, size_t workspace_bytes, Comm* comm, uint64_t seed, uintptr_t lr_dev,
              uintptr_t metrics_dev, float b1, float b2, float eps, float weight_decay, bool eps_hat);
  ~KerasEngine();
  KerasEngine(const KerasEngine&) = delete;
  KerasEngine& operator=(const KerasEngine&) = delete;

  static size_t workspace_bytes(int B);
  void step();                           // one eager step on stream()
  void capture(int steps_per_graph);     // whole step(s), collectives included, in one graph
  void replay(int n);                    // n steps (graphs once captured)
  void uncapture();
  int warm_graphs();
  void repack();                         // after parameters changed outside the engine
  void sync();
  // gradient transport at world size > 1: RCCL (default) or the peer transport; drops graphs
  void set_peer(PeerComm* p);
  void set_force_collectives(bool on);
  void set_external_batch(bool on) { external_ = on; }
  int world_size() const;
  bool reducer_active() const { return reducer_->active(); }
  bool peer_active() const { return reducer_->peer() != nullptr; }
  bool captured() const { return exec_ != nullptr; }
  uintptr_t stream() const { return reinterpret_cast<uintptr_t>(s_); }
  uintptr_t x_ptr() const { return reinterpret_cast<uintptr_t>(f_.x); }
  uintptr_t y_ptr() const { return reinterpret_cast<uintptr_t>(f_.y); }
  uintptr_t counter_ptr() const { return reinterpret_cast<uintptr_t>(f_.counter); }

 private:
  void launch_step();
  KerasFused args() const;
  hipGraphExec_t capture_fn(int steps, hipGraph_t* g);
  int B_;
  KerasFused f_{};
  Comm* comm_;
  uint64_t seed_;
  bool external_ = false;
  hipStream_t s_ = nullptr;
  std::unique_ptr<Reducer> reducer_;
  int steps_per_graph_ = 1;
  hipGraph_t graph_ = nullptr;
  hipGraphExec_t exec_ = nullptr;
  std::vector<std::pair<int, hipGraphExec_t>> rem_exec_;
  std::vector<hipGraph_t> rem_graph_;
};

}  // namespace mx
