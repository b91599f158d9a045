#include "reducer.h"

#include "common.h"

namespace mx {

Reducer::Reducer(Comm* comm, uintptr_t flat_grad, DType dtype, const std::vector<BucketSpec>& buckets,
                 const std::vector<int>& param_bucket, RedOp op, bool timing)
    : comm_(comm), flat_(reinterpret_cast<char*>(flat_grad)), dtype_(dtype), op_(op),
      param_bucket_(param_bucket), timing_(timing) {
  for (const auto& b : buckets) buckets_.push_back(Bucket{b.offset, b.numel, 0, 0, false, nullptr});
  for (int pb : param_bucket_) {
    MX_CHECK(pb >= 0 && pb < (int)buckets_.size(), "param assigned to unknown bucket");
    buckets_[pb].total++;
  }
  for (auto& b : buckets_) MX_HIP_CHECK(hipEventCreateWithFlags(&b.ev, hipEventDisableTiming));
  MX_HIP_CHECK(hipStreamCreateWithFlags(&comm_stream_, hipStreamNonBlocking));
  MX_HIP_CHECK(hipEventCreateWithFlags(&done_, hipEventDisableTiming));
  if (timing_) {
    MX_HIP_CHECK(hipEventCreate(&t0_));
    MX_HIP_CHECK(hipEventCreate(&t1_));
  }
  marked_.assign(param_bucket_.size(), 0);
  prepare();
}

Reducer::~Reducer() {
  for (auto& b : buckets_)
    if (b.ev) hipEventDestroy(b.ev);
  if (done_) hipEventDestroy(done_);
  if (t0_) hipEventDestroy(t0_);
  if (t1_) hipEventDestroy(t1_);
  if (comm_stream_) hipStreamDestroy(comm_stream_);
}

void Reducer::prepare() {
  for (auto& b : buckets_) {
    b.pending = b.total;
    b.ready = false;
  }
  std::fill(marked_.begin(), marked_.end(), 0);
  next_ = 0;
}

void Reducer::mark_ready(int p, hipStream_t compute) {
  MX_CHECK(p >= 0 && p < (int)param_bucket_.size(), "mark_ready: bad parameter index");
  MX_CHECK(!marked_[p], "parameter marked ready twice in one backward pass (reentrant backward or "
                        "shared parameter); reducer state would race");
  marked_[p] = 1;
  Bucket& b = buckets_[param_bucket_[p]];
  if (--b.pending == 0) {
    b.ready = true;
    launch_ready(compute);
  }
}

void Reducer::mark_bucket_ready(int bi, hipStream_t compute) {
  MX_CHECK(bi >= 0 && bi < (int)buckets_.size(), "mark_bucket_ready: bad bucket");
  Bucket& b = buckets_[bi];
  b.pending = 0;
  b.ready = true;
  launch_ready(compute);
}

bool Reducer::active() const { return comm_ && (comm_->world_size() > 1 || force_); }

void Reducer::launch_ready(hipStream_t compute) {
  const bool act = active();
  while (next_ < (int)buckets_.size() && buckets_[next_].ready) {
    Bucket& b = buckets_[next_];
    MX_CHECK(b.pending == 0, "bucket launched before all its gradients were ready");
    if (act) {  // no collectives -> no fences either (a fence alone costs a few us of GPU idle)
      hipStream_t st = compute;
      if (overlap_) {
        MX_HIP_CHECK(hipEventRecord(b.ev, compute));
        MX_HIP_CHECK(hipStreamWaitEvent(comm_stream_, b.ev, 0));
        st = comm_stream_;
        side_used_ = true;
      }
      if (timing_ && next_ == 0) MX_HIP_CHECK(hipEventRecord(t0_, st));
      char* p = flat_ + b.offset * dtype_size(dtype_);
      comm_->all_reduce(p, p, b.numel, dtype_, op_, st);
    }
    ++next_;
  }
}

void Reducer::finalize(hipStream_t compute) {
  for (auto& b : buckets_) {
    if (!b.ready) {  // unused parameters: reduce whatever the bucket holds (zeros on this rank)
      b.pending = 0;
      b.ready = true;
    }
  }
  launch_ready(compute);
  if (!active()) return;
  if (timing_) {
    MX_HIP_CHECK(hipEventRecord(t1_, side_used_ ? comm_stream_ : compute));
    timed_ = true;
  }
  if (side_used_) {
    MX_HIP_CHECK(hipEventRecord(done_, comm_stream_));
    MX_HIP_CHECK(hipStreamWaitEvent(compute, done_, 0));
    side_used_ = false;
  }
}

float Reducer::last_comm_ms() {
  if (!timing_ || !timed_) return 0.f;
  MX_HIP_CHECK(hipEventSynchronize(t1_));
  float ms = 0.f;
  MX_HIP_CHECK(hipEventElapsedTime(&ms, t0_, t1_));
  return ms;
}

}  // namespace mx
