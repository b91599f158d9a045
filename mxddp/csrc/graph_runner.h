// Whole-step hipGraph capture / replay shared by the fused engines (MLP, Keras CNN).
//
// capture(step, k) records k consecutive training steps into one graph (batches, learning rate,
// optimizer step counts and metrics all live in device memory, so every unrolled step is a
// distinct, correct step), plus 2^j-step graphs for the remainder of a replay(n) whose n is not
// a multiple of k: a replay then runs entirely from graphs.  warm() launches every graph once
// (real steps; the first launch of a graph exec pays one-time costs).
#pragma once
#include <hip/hip_runtime.h>

#include <functional>
#include <utility>
#include <vector>

#include "common.h"

namespace mx {

class GraphRunner {
 public:
  explicit GraphRunner(hipStream_t s = nullptr) : s_(s) {}
  ~GraphRunner() { clear(); }
  GraphRunner(const GraphRunner&) = delete;
  GraphRunner& operator=(const GraphRunner&) = delete;
  void set_stream(hipStream_t s) { s_ = s; }

  bool captured() const { return exec_ != nullptr; }
  int steps_per_graph() const { return spg_; }

  void capture(const std::function<void()>& step, int steps_per_graph) {
    if (exec_) return;
    MX_HIP_CHECK(hipStreamSynchronize(s_));
    spg_ = steps_per_graph < 1 ? 1 : steps_per_graph;
    exec_ = record(step, spg_, &graph_);
    int k = 1;
    while (2 * k < spg_) k *= 2;
    for (; k >= 1 && spg_ > 1; k /= 2) {  // remainder graphs, largest first
      hipGraph_t g = nullptr;
      rem_exec_.emplace_back(k, record(step, k, &g));
      rem_graph_.push_back(g);
    }
  }

  // n steps: full groups, then the remainder graphs, then (never, once captured) eager steps
  void replay(int n, const std::function<void()>& step) {
    if (!exec_) {
      for (int i = 0; i < n; ++i) step();
      return;
    }
    const int full = n / spg_;
    n -= full * spg_;
    for (int i = 0; i < full; ++i) MX_HIP_CHECK(hipGraphLaunch(exec_, s_));
    for (const auto& e : rem_exec_)
      if (n >= e.first) {
        MX_HIP_CHECK(hipGraphLaunch(e.second, s_));
        n -= e.first;
      }
    for (; n > 0; --n) step();
  }

  int warm() {
    if (!exec_) return 0;
    int steps = spg_;
    MX_HIP_CHECK(hipGraphLaunch(exec_, s_));
    for (const auto& e : rem_exec_) {
      MX_HIP_CHECK(hipGraphLaunch(e.second, s_));
      steps += e.first;
    }
    MX_HIP_CHECK(hipStreamSynchronize(s_));
    return steps;
  }

  void clear() {
    if (s_ && (exec_ || !rem_exec_.empty())) hipStreamSynchronize(s_);
    if (exec_) hipGraphExecDestroy(exec_);
    if (graph_) hipGraphDestroy(graph_);
    exec_ = nullptr;
    graph_ = nullptr;
    for (auto& e : rem_exec_) hipGraphExecDestroy(e.second);
    for (auto g : rem_graph_) hipGraphDestroy(g);
    rem_exec_.clear();
    rem_graph_.clear();
  }

 private:
  hipGraphExec_t record(const std::function<void()>& step, int steps, hipGraph_t* g) {
    MX_HIP_CHECK(hipStreamBeginCapture(s_, hipStreamCaptureModeThreadLocal));
    try {
      for (int i = 0; i < steps; ++i) step();
    } catch (...) {
      hipGraph_t tmp = nullptr;
      hipStreamEndCapture(s_, &tmp);
      if (tmp) hipGraphDestroy(tmp);
      throw;
    }
    MX_HIP_CHECK(hipStreamEndCapture(s_, g));
    hipGraphExec_t exec = nullptr;
    MX_HIP_CHECK(hipGraphInstantiate(&exec, *g, nullptr, nullptr, 0));
    MX_HIP_CHECK(hipGraphUpload(exec, s_));
    return exec;
  }
  hipStream_t s_;
  int spg_ = 1;
  hipGraph_t graph_ = nullptr;
  hipGraphExec_t exec_ = nullptr;
  std::vector<std::pair<int, hipGraphExec_t>> rem_exec_;
  std::vector<hipGraph_t> rem_graph_;
};

}  // namespace mx
