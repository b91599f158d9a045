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
#include "graph_runner.h"
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
  // mode 1: whole step(s), collectives included, in one graph per steps_per_graph steps;
  // mode 0: eager launches
  void capture(int mode, int steps_per_graph);
  void replay(int n);                    // n steps (graphs once captured)
  void uncapture();
  int warm_graphs() { return graphs_.warm(); }
  void repack();                         // after parameters changed outside the engine
  void sync();
  // gradient transport at world size > 1: RCCL (default) or the peer transport; drops graphs
  void set_peer(PeerComm* p);
  void set_comm(Comm* c);  // another RCCL communicator over the same ranks (comm.py variants)
  void set_force_collectives(bool on);
  // the step all-reduces its 373 KB gradient as ONE bucket between the finalize and Adam: the
  // bucket strategies of the other engines ("one" is the only one) and the all-reduce padding
  void set_merged(bool) {}
  void set_overlap(bool) {}
  bool merged() const { return true; }
  bool overlap() const { return false; }
  void set_bucket_padding(size_t capacity, size_t multiple) {
    reducer_->set_padding(KerasLayout::total, capacity, multiple);
  }
  // peer transport: the exchange co-scheduled with Adam in one launch (keras_fused_exchange_adam)
  // instead of a separate all-reduce; false (and off) when no opened peer transport can take it.
  // The PeerComm's other exchanges may run before / after only across a synchronisation of every
  // rank (see kx_kernel).
  bool set_coscheduled(bool on);
  bool coscheduled() const { return coscheduled_; }
  void set_external_batch(bool on) { external_ = on; }
  int world_size() const;
  bool reducer_active() const { return reducer_->active(); }
  bool peer_active() const { return reducer_->peer() != nullptr; }
  bool captured() const { return graphs_.captured(); }
  int graph_mode() const { return graphs_.captured() ? 1 : 0; }
  uintptr_t stream() const { return reinterpret_cast<uintptr_t>(s_); }
  uintptr_t x_ptr() const { return reinterpret_cast<uintptr_t>(f_.x); }
  uintptr_t y_ptr() const { return reinterpret_cast<uintptr_t>(f_.y); }
  uintptr_t counter_ptr() const { return reinterpret_cast<uintptr_t>(f_.counter); }

 private:
  void launch_step();
  KerasFused args() const;
  int B_;
  KerasFused f_{};
  Comm* comm_;
  uint64_t seed_;
  bool external_ = false;
  bool coscheduled_ = false;
  PeerArgs co_args_{};
  hipStream_t s_ = nullptr;
  std::unique_ptr<Reducer> reducer_;
  GraphRunner graphs_;
};

}  // namespace mx
