// Gradient-bucket reducer: the MI355X-native replacement for torch DDP's C++ Reducer
// (reached via DistributedDataParallel at pytorch/distributed_data_parallel.py:74).
//
//  * gradients live in ONE flat buffer; every parameter's .grad is a view into it, so a
//    bucket is a contiguous [offset, offset+numel) slice: no copy-in / copy-out;
//  * buckets are assigned in reverse registration order (the order backward produces
//    grads) by the Python layer; each bucket counts down as its params become ready;
//  * a ready bucket is launched strictly in bucket order (all ranks must issue RCCL
//    collectives in the same order): event recorded on the compute stream, the comm
//    stream waits on it, then an in-place RCCL all-reduce runs on the comm stream and
//    overlaps the remaining backward;
//  * finalize() makes the compute stream wait on the comm stream before the optimizer.
//  * debug checks: a parameter marked twice in one backward, or a bucket launched
//    before all of its parameters were marked, raises (race detection);
//    so do buckets of one backward marked from two different compute streams (the event
//    fence would order the all-reduce after the wrong stream's work) and a new backward
//    started while the previous one's side-stream all-reduces were never joined.
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "bucket_schedule.h"
#include "comm.h"
#include "peer.h"

namespace mx {

// Process-wide: every Reducer keeps its fences and stream joins but issues no collective (the
// bench's compute-only pass after the timed region: exposed comm time = the step with the
// gradient exchange minus the same captured step without it; replicas diverge, so never train
// this way).  Graphs captured before a switch keep what they captured.
void reducer_set_dry(bool on);
bool reducer_dry();

class Reducer {
 public:
  struct BucketSpec {
    size_t offset, numel;
  };
  Reducer(Comm* comm, uintptr_t flat_grad, DType dtype, const std::vector<BucketSpec>& buckets,
          const std::vector<int>& param_bucket, RedOp op, bool timing);
  ~Reducer();

  void prepare();
  // drop a step whose backward failed between prepare() and finalize() (joins the side stream)
  void abort();
  // start of a backward pass
  void mark_ready(int param_idx, hipStream_t compute);
  void mark_bucket_ready(int bucket, hipStream_t compute);  // fused engines: whole bucket at once
  void finalize(hipStream_t compute);               // launch stragglers; compute waits on comm
  hipStream_t comm_stream() { return side(); }
  int num_buckets() const { return sched_.size(); }
  int launched() const { return sched_.launched(); }
  // milliseconds between first bucket launch and comm completion of the last step
  // (requires timing=true; synchronises on the comm stream's end event).
  float last_comm_ms();
  // time the next steps' comm window (eager steps only: a graph captured while timing would
  // bake the event records in)
  void set_timing(bool on);
  bool timing() const { return timing_; }
  void set_comm(Comm* c) { comm_ = c; }
  // A bucket that ends where the gradients end ([offset, total)) is all-reduced over
  // roundup(numel, multiple) elements when the buffer has that much zeroed slack (capacity):
  // every rank's share of every channel then starts 16-byte aligned (xGMI sizing).
  // Interior buckets are never padded (their tail is the next bucket's data).
  void set_padding(size_t total, size_t capacity, size_t multiple) {
    pad_total_ = total;
    pad_cap_ = capacity;
    pad_mult_ = multiple;
  }
  size_t padded_count(size_t offset, size_t numel) const;
  // issue the collectives even at world_size 1 (exercises the RCCL + graph-capture path on
  // a single GPU; an all-reduce over one rank is the identity)
  void set_force_collectives(bool on) { force_ = on; }
  bool forced() const { return force_; }
  // overlap = true: each bucket's all-reduce runs on the side comm stream as soon as it is ready
  // (event fence compute -> comm, and compute waits on comm at finalize).  overlap = false: the
  // all-reduces are issued in order on the compute stream itself -- no cross-stream fences,
  // which on ROCm cost several us each, but no overlap with the rest of the backward.
  void set_overlap(bool on) { overlap_ = on; }
  bool overlap() const { return overlap_; }
  // true when collectives are actually issued (world size > 1, or forced for testing)
  bool active() const;
  // transport for sum all-reduces: RCCL (nullptr, default) or the direct xGMI peer transport
  // (peer.h).  Every rank must make the same choice.
  void set_peer(PeerComm* p) { peer_ = p; }
  PeerComm* peer() const { return peer_; }
  // opt-in reduced-precision communication of an fp32 gradient: each bucket is cast to bf16 into
  // `shadow` (a bf16 buffer as long as the gradient buffer's capacity), all-reduced in bf16 and
  // cast back into the fp32 bucket (half the bytes over the links).  kF32 = off.
  void set_comm_dtype(DType t, uintptr_t shadow);
  DType comm_dtype() const { return shadow_ ? DType::kBF16 : dtype_; }

 private:
  void launch_ready(hipStream_t compute);
  Comm* comm_;
  PeerComm* peer_ = nullptr;
  char* flat_;
  DType dtype_;
  RedOp op_;
  BucketSchedule sched_;          // host state machine (bucket_schedule.h)
  std::vector<hipEvent_t> ev_;    // per-bucket compute -> comm fence
  hipStream_t comm_stream_ = nullptr;  // side stream, created on first use (side())
  int dev_ = 0;
  hipStream_t side();
  hipEvent_t done_ = nullptr, t0_ = nullptr, t1_ = nullptr;
  bool timing_ = false, timed_ = false, force_ = false, overlap_ = true, side_used_ = false;
  // stream discipline: every bucket of one backward is fenced against ONE compute
  // stream, and a backward's side-stream work must be joined (finalize) before the next begins
  hipStream_t step_compute_ = nullptr;
  size_t pad_total_ = 0, pad_cap_ = 0, pad_mult_ = 1;
  uint16_t* shadow_ = nullptr;  // bf16 communication buffer (set_comm_dtype), or null
  bool in_step_ = false;
};

}  // namespace mx
