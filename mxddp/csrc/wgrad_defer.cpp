#include "wgrad_defer.h"

#include <map>
#include <mutex>
#include <vector>

#include "common.h"

namespace mx {

namespace {
thread_local bool t_active = false;
thread_local bool t_took = false;
std::mutex g_mu;
std::map<int, std::vector<RedJob>> g_jobs;  // HIP device -> pending jobs, in issue order

int cur_device() {
  int d = 0;
  MX_HIP_CHECK(hipGetDevice(&d));
  return d;
}
}  // namespace

void wgrad_defer_set(bool on) {
  t_active = on;
  t_took = false;
}
bool wgrad_defer_active() { return t_active; }
bool wgrad_defer_took() { return t_took; }

void wgrad_defer_push(const RedJob& j) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_jobs[cur_device()].push_back(j);
  t_took = true;
}

int wgrad_defer_pending() {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_jobs.find(cur_device());
  return it == g_jobs.end() ? 0 : (int)it->second.size();
}

int wgrad_defer_flush(hipStream_t st) {
  std::vector<RedJob> jobs;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_jobs.find(cur_device());
    if (it == g_jobs.end()) return 0;
    jobs.swap(it->second);
  }
  // consecutive jobs of one kind per launch; a launch never holds two jobs writing the same dW
  // (a later one may accumulate onto an earlier one: gradient accumulation), so they stay ordered
  size_t i = 0;
  while (i < jobs.size()) {
    RedBatch b{};
    int blocks = 0;
    const int kind = jobs[i].kind;
    while (i < jobs.size() && b.n < kRedMaxJobs && jobs[i].kind == kind) {
      bool dup = false;
      for (int q = 0; q < b.n; ++q) dup = dup || b.j[q].dw == jobs[i].dw;
      if (dup) break;
      RedJob j = jobs[i++];
      j.blk0 = blocks;
      blocks += j.blocks;
      b.j[b.n++] = j;
    }
    if (kind == 0) wino_reduce_batch_launch(b, blocks, st);
    else nhwc_reduce_batch_launch(b, blocks, st);
  }
  return (int)jobs.size();
}

}  // namespace mx
