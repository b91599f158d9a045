#include "reducer.h"

#include "common.h"
#include "ops.h"

namespace mx {

static bool g_dry = false;
void reducer_set_dry(bool on) { g_dry = on; }
bool reducer_dry() { return g_dry; }

Reducer::Reducer(Comm* comm, uintptr_t flat_grad, DType dtype, const std::vector<BucketSpec>& buckets,
                 const std::vector<int>& param_bucket, RedOp op, bool timing)
    : comm_(comm), flat_(reinterpret_cast<char*>(flat_grad)), dtype_(dtype), op_(op), timing_(timing) {
  std::vector<std::pair<size_t, size_t>> spans;
  for (const auto& b : buckets) spans.emplace_back(b.offset, b.numel);
  sched_ = BucketSchedule(spans, param_bucket);
  ev_.assign(buckets.size(), nullptr);
  for (auto& e : ev_) MX_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  // the side stream is created on first use (side()): reducers that never overlap -- a merged
  // bucket, the co-scheduled engines' -- then hold no stream, i.e. no extra hardware queue
  MX_HIP_CHECK(hipGetDevice(&dev_));
  MX_HIP_CHECK(hipEventCreateWithFlags(&done_, hipEventDisableTiming));
  if (timing_) {
    MX_HIP_CHECK(hipEventCreate(&t0_));
    MX_HIP_CHECK(hipEventCreate(&t1_));
  }
}

Reducer::~Reducer() {
  for (auto e : ev_)
    if (e) hipEventDestroy(e);
  if (done_) hipEventDestroy(done_);
  if (t0_) hipEventDestroy(t0_);
  if (t1_) hipEventDestroy(t1_);
  if (comm_stream_) hipStreamDestroy(comm_stream_);
}

void Reducer::prepare() {
  MX_CHECK(!side_used_, "reducer: a new backward started while the previous one's side-stream all-reduces were "
                        "never joined (finalize() not called): the optimizer would race the comm stream");
  sched_.prepare();
  in_step_ = true;
  step_compute_ = nullptr;
}

void Reducer::set_comm_dtype(DType t, uintptr_t shadow) {
  MX_CHECK(t == dtype_ || (t == DType::kBF16 && dtype_ == DType::kF32 && shadow),
           "reducer: bf16 communication of an fp32 gradient needs a bf16 shadow buffer");
  MX_CHECK(!in_step_, "reducer: communication dtype changed inside a backward");
  shadow_ = t == dtype_ ? nullptr : reinterpret_cast<uint16_t*>(shadow);
}

void Reducer::abort() {
  // a backward that raised after some buckets were launched: wait for what the side stream
  // already runs (nothing may still write the gradient), then forget the step
  if (side_used_) MX_HIP_CHECK(hipStreamSynchronize(comm_stream_));
  side_used_ = false;
  in_step_ = false;
  step_compute_ = nullptr;
  sched_.prepare();
}

void Reducer::set_timing(bool on) {
  if (on && !t0_) {
    MX_HIP_CHECK(hipEventCreate(&t0_));
    MX_HIP_CHECK(hipEventCreate(&t1_));
  }
  timing_ = on;
}

void Reducer::mark_ready(int p, hipStream_t compute) {
  if (sched_.mark(p)) launch_ready(compute);
}

void Reducer::mark_bucket_ready(int bi, hipStream_t compute) {
  sched_.mark_bucket(bi);
  launch_ready(compute);
}

bool Reducer::active() const {
  return (comm_ && (comm_->world_size() > 1 || force_)) || (peer_ && peer_->world_size() > 1);
}

hipStream_t Reducer::side() {
  if (!comm_stream_) {
    int cur = 0;
    MX_HIP_CHECK(hipGetDevice(&cur));
    if (cur != dev_) MX_HIP_CHECK(hipSetDevice(dev_));
    MX_HIP_CHECK(hipStreamCreateWithFlags(&comm_stream_, hipStreamNonBlocking));
    if (cur != dev_) MX_HIP_CHECK(hipSetDevice(cur));
  }
  return comm_stream_;
}

void Reducer::launch_ready(hipStream_t compute) {
  const bool act = active();
  if (in_step_) {
    if (!step_compute_) step_compute_ = compute;
    MX_CHECK(step_compute_ == compute, "reducer: buckets of one backward marked ready from two different compute "
                                       "streams (each bucket's fence must follow the stream that wrote it)");
  }
  for (int bi = sched_.pop_ready(); bi >= 0; bi = sched_.pop_ready()) {
    const BucketSchedule::Bucket& b = sched_.bucket(bi);
    if (act) {  // no collectives -> no fences either (a fence alone costs a few us of GPU idle)
      hipStream_t st = compute;
      if (overlap_) {
        MX_HIP_CHECK(hipEventRecord(ev_[bi], compute));
        st = side();
        MX_HIP_CHECK(hipStreamWaitEvent(st, ev_[bi], 0));
        side_used_ = true;
      }
      if (timing_ && bi == 0) MX_HIP_CHECK(hipEventRecord(t0_, st));
      char* p = flat_ + b.offset * dtype_size(dtype_);
      const bool via_peer = peer_ && (op_ == RedOp::kSum || op_ == RedOp::kAvg) && peer_->world_size() > 1;
      const size_t n = via_peer ? b.numel : padded_count(b.offset, b.numel);
      void* buf = p;
      DType t = dtype_;
      if (shadow_) {  // bf16 on the wire: cast in, all-reduce, cast back (same stream)
        buf = shadow_ + b.offset;
        t = DType::kBF16;
        cast_f32_bf16(reinterpret_cast<const float*>(p), shadow_ + b.offset, (int64_t)n, st);
      }
      if (g_dry) {
        // compute-only pass: no exchange (the casts above / below still run)
      } else if (via_peer) {
        peer_->all_reduce(buf, n, t, st, op_);
      } else {
        MX_CHECK(comm_ != nullptr, "reducer: no RCCL communicator for this collective");
        comm_->all_reduce(buf, buf, n, t, op_, st);
      }
      if (shadow_) cast_bf16_f32(shadow_ + b.offset, reinterpret_cast<float*>(p), (int64_t)b.numel, st);
    }
  }
}

void Reducer::finalize(hipStream_t compute) {
  sched_.release_all();  // unused parameters: reduce whatever the bucket holds (zeros on this rank)
  launch_ready(compute);
  in_step_ = false;
  step_compute_ = nullptr;
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

size_t Reducer::padded_count(size_t offset, size_t numel) const {
  if (pad_mult_ <= 1 || offset + numel != pad_total_) return numel;
  const size_t n = (numel + pad_mult_ - 1) / pad_mult_ * pad_mult_;
  return offset + n <= pad_cap_ ? n : numel;
}

float Reducer::last_comm_ms() {
  if (!timing_ || !timed_) return 0.f;
  MX_HIP_CHECK(hipEventSynchronize(t1_));
  float ms = 0.f;
  MX_HIP_CHECK(hipEventElapsedTime(&ms, t0_, t1_));
  return ms;
}

}  // namespace mx
