#include "keras_engine.h"

#include "common.h"
#include "ops.h"

namespace mx {

namespace {
constexpr size_t kAlign = 64;  // floats (256 B)
inline size_t al(size_t n) { return (n + kAlign - 1) / kAlign * kAlign; }

struct Carve {
  char* base;
  size_t off, cap;  // floats
  template <class T>
  T* take(size_t n) {
    T* p = reinterpret_cast<T*>(base + off * 4);
    off += al((n * sizeof(T) + 3) / 4);
    MX_CHECK(!base || off * 4 <= cap, "keras engine workspace too small");
    return p;
  }
};

// one carve for sizing (base = null) and for the real buffers
void carve_all(Carve& c, KerasFused& f, int B) {
  f.x = c.take<float>((size_t)B * 784);
  f.y = c.take<int32_t>(B);
  f.p1 = c.take<float>((size_t)B * 5408);
  f.q1 = c.take<uint8_t>((size_t)B * 5408);
  f.p2 = c.take<float>((size_t)B * 1600);
  f.q2 = c.take<uint8_t>((size_t)B * 1600);
  f.x3 = c.take<float>((size_t)B * 576);
  f.h1 = c.take<float>((size_t)B * 64);
  f.dl = c.take<float>((size_t)B * 16);
  f.dh1 = c.take<float>((size_t)B * 64);
  f.dx3 = c.take<float>((size_t)B * 576);
  f.dp2 = c.take<float>((size_t)B * 1600);
  f.sv = c.take<float>((size_t)B * 256);
  f.pl1 = c.take<float>((size_t)4 * B * 320);
  f.pl2 = c.take<float>((size_t)B * 18432);
  f.pl3 = c.take<float>((size_t)(B / 8) * 36864);
  f.pf1 = c.take<float>((size_t)(B / 8) * 36864);
  f.gf2 = c.take<float>(640);
  f.w2f = c.take<float>(18432);
  f.w2d = c.take<float>(18432);
  f.counter = c.take<int32_t>(4);
  f.tmpl = c.take<float>(10 * 784);
}
}  // namespace

size_t KerasEngine::workspace_bytes(int B) {
  KerasFused f{};
  Carve c{nullptr, 0, 0};
  carve_all(c, f, B);
  return c.off * 4;
}

KerasEngine::KerasEngine(int batch, uintptr_t params, uintptr_t grads, uintptr_t m, uintptr_t v,
                         uintptr_t adam_state, uintptr_t workspace, size_t workspace_bytes, Comm* comm, uint64_t seed,
                         uintptr_t lr_dev, uintptr_t metrics_dev, float b1, float b2, float eps, float weight_decay,
                         bool eps_hat)
    : B_(batch), comm_(comm), seed_(seed) {
  MX_CHECK(B_ > 0 && B_ % 8 == 0 && B_ <= 1024, "keras engine: batch must be a multiple of 8 (<= 1024)");
  Carve c{reinterpret_cast<char*>(workspace), 0, workspace_bytes};
  carve_all(c, f_, B_);
  f_.B = B_;
  f_.p = reinterpret_cast<float*>(params);
  f_.g = reinterpret_cast<float*>(grads);
  f_.m = reinterpret_cast<float*>(m);
  f_.v = reinterpret_cast<float*>(v);
  f_.adam_state = reinterpret_cast<int32_t*>(adam_state);
  f_.lr = reinterpret_cast<const float*>(lr_dev);
  f_.metrics = reinterpret_cast<float*>(metrics_dev);
  f_.b1 = b1;
  f_.b2 = b2;
  f_.eps = eps;
  f_.wd = weight_decay;
  f_.eps_hat = eps_hat ? 1 : 0;
  MX_HIP_CHECK(hipStreamCreateWithFlags(&s_, hipStreamNonBlocking));
  graphs_.set_stream(s_);
  MX_HIP_CHECK(hipMemsetAsync(f_.counter, 0, 16, s_));
  synth_templates(const_cast<float*>(f_.tmpl), 10, 784, seed_ ^ 0x5eedull, s_);  // identical on every rank
  // one bucket: the whole 373 KB gradient, all-reduced in order on the compute stream
  std::vector<Reducer::BucketSpec> buckets = {{0, KerasLayout::total}};
  reducer_ = std::make_unique<Reducer>(comm_, grads, DType::kF32, buckets, std::vector<int>(10, 0), RedOp::kSum,
                                       false);
  reducer_->set_overlap(false);
  repack();
  MX_HIP_CHECK(hipStreamSynchronize(s_));
}

KerasEngine::~KerasEngine() {
  uncapture();
  reducer_.reset();
  if (s_) hipStreamDestroy(s_);
}

int KerasEngine::world_size() const {
  return comm_ ? comm_->world_size() : (reducer_->peer() ? reducer_->peer()->world_size() : 1);
}

KerasFused KerasEngine::args() const {
  KerasFused f = f_;
  const int rank = comm_ ? comm_->rank() : (reducer_->peer() ? reducer_->peer()->rank() : 0);
  f.seed = seed_ + rank * 7919ull;  // per-rank data shard
  f.synth = external_ ? 0 : 1;
  return f;
}

void KerasEngine::repack() { keras_fused_update(args(), 3, 1.f, s_); }

void KerasEngine::launch_step() {
  const KerasFused f = args();
  keras_fused_forward(f, s_);
  keras_fused_backward(f, s_);
  if (!reducer_->active()) {
    keras_fused_update(f, 0, 1.f, s_);
    return;
  }
  keras_fused_update(f, 1, 1.f, s_);  // finalize into g
  if (coscheduled_) {
    keras_fused_exchange_adam(f, co_args_, s_);  // exchange + average + Adam in one launch
    return;
  }
  reducer_->prepare();
  reducer_->mark_bucket_ready(0, s_);  // sum all-reduce of g
  reducer_->finalize(s_);
  keras_fused_update(f, 2, 1.f / (float)world_size(), s_);  // Adam on the averaged gradient
}

void KerasEngine::step() { launch_step(); }

void KerasEngine::capture(int mode, int steps_per_graph) {
  if (mode == 0 || graphs_.captured()) return;
  graphs_.capture([this] { launch_step(); }, steps_per_graph);
}

void KerasEngine::replay(int n) { graphs_.replay(n, [this] { launch_step(); }); }

void KerasEngine::uncapture() {
  if (s_) MX_HIP_CHECK(hipStreamSynchronize(s_));
  graphs_.clear();
}

void KerasEngine::set_comm(Comm* c) {
  if (c == comm_) return;
  MX_CHECK(!c || !comm_ || (c->rank() == comm_->rank() && c->world_size() == comm_->world_size()),
           "set_comm: the communicator must have this engine's rank and world size");
  uncapture();
  comm_ = c;
  reducer_->set_comm(c);
}

void KerasEngine::set_peer(PeerComm* p) {
  if (p != reducer_->peer()) uncapture();
  reducer_->set_peer(p);
  if (coscheduled_) set_coscheduled(true);  // re-derive the arguments, or drop the mode
}

bool KerasEngine::set_coscheduled(bool on) {
  if (on) {
    PeerComm* pc = reducer_->peer();
    on = pc && reducer_->active() && keras_exchange_blocks() <= kPeerMaxBlocks &&
         pc->oneshot_args(f_.g, KerasLayout::total, RedOp::kAvg, &co_args_);
  }
  if (on != coscheduled_) uncapture();
  coscheduled_ = on;
  return on;
}

void KerasEngine::set_force_collectives(bool on) {
  if (on != reducer_->forced()) uncapture();
  reducer_->set_force_collectives(on);
}

void KerasEngine::sync() { MX_HIP_CHECK(hipStreamSynchronize(s_)); }

}  // namespace mx
