#include "mlp_engine.h"

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
    MX_CHECK(!base || off * 4 <= cap, "mlp engine workspace too small");
    return p;
  }
};

// one carve for sizing (base = null) and for the real buffers
void carve_all(Carve& c, MlpFused& f, int B) {
  using L = MlpLayout;
  f.x = c.take<float>((size_t)B * L::kIn);
  f.y = c.take<int32_t>(B);
  f.h1 = c.take<float>((size_t)B * L::kHP);
  f.h2 = c.take<float>((size_t)B * L::kHP);
  f.dl = c.take<float>((size_t)B * 16);
  f.dh2 = c.take<float>((size_t)B * L::kHP);
  f.dh1p = c.take<float>((size_t)4 * B * L::kHP);
  f.lsum = c.take<float>((size_t)B / 16 * 2);
  f.counter = c.take<int32_t>(4);
  f.tmpl = c.take<float>(10 * L::kIn);
}
}  // namespace

size_t MlpEngine::workspace_bytes(int B) {
  MlpFused f{};
  Carve c{nullptr, 0, 0};
  carve_all(c, f, (B + 15) / 16 * 16);  // every [B] buffer has the padded tile count of rows
  return c.off * 4;
}

MlpEngine::MlpEngine(int batch, uintptr_t params, uintptr_t grads, uintptr_t m, uintptr_t v, uintptr_t adam_state,
                     uintptr_t workspace, size_t workspace_bytes, Comm* comm, uint64_t seed, uintptr_t lr_dev,
                     uintptr_t metrics_dev, float b1, float b2, float eps, float weight_decay, bool eps_hat)
    : B_(batch), comm_(comm), seed_(seed) {
  using L = MlpLayout;
  MX_CHECK(B_ >= 1 && B_ <= kMlpMaxBatch, "mlp engine: batch must be in [1, 512]");
  const int Bp = (B_ + 15) / 16 * 16;  // MFMA row tiles; rows B.. are masked out of every sum
  Carve c{reinterpret_cast<char*>(workspace), 0, workspace_bytes};
  carve_all(c, f_, Bp);
  f_.B = B_;
  f_.Bp = Bp;
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
  // h1 / h2 / dh2 pad columns must read as zero before the first step writes them
  MX_HIP_CHECK(hipMemsetAsync(f_.h1, 0, sizeof(float) * Bp * L::kHP, s_));
  MX_HIP_CHECK(hipMemsetAsync(f_.h2, 0, sizeof(float) * Bp * L::kHP, s_));
  // a caller's batch fills rows 0..B-1 only: the tail rows of the last tile stay finite zeros
  MX_HIP_CHECK(hipMemsetAsync(f_.x, 0, sizeof(float) * Bp * L::kIn, s_));
  MX_HIP_CHECK(hipMemsetAsync(f_.y, 0, sizeof(int32_t) * Bp, s_));
  synth_templates(const_cast<float*>(f_.tmpl), 10, L::kIn, seed_ ^ 0x5eedull, s_);  // identical on every rank
  // bucket 0: [l2.w .. l3.b] (complete after K4, overlappable with K5); bucket 1: [l1.w, l1.b]
  std::vector<Reducer::BucketSpec> buckets = {{L::w2, L::total - L::w2}, {0, L::w2}};
  reducer_ = std::make_unique<Reducer>(comm_, grads, DType::kF32, buckets, std::vector<int>{1, 1, 0, 0, 0, 0},
                                       RedOp::kSum, false);
  merged_reducer_ = std::make_unique<Reducer>(comm_, grads, DType::kF32,
                                              std::vector<Reducer::BucketSpec>{{0, L::total}},
                                              std::vector<int>(6, 0), RedOp::kSum, false);
  merged_reducer_->set_overlap(false);
  MX_HIP_CHECK(hipStreamSynchronize(s_));
}

MlpEngine::~MlpEngine() {
  uncapture();
  reducer_.reset();
  merged_reducer_.reset();
  if (s_) hipStreamDestroy(s_);
}

int MlpEngine::world_size() const {
  return comm_ ? comm_->world_size() : (reducer_->peer() ? reducer_->peer()->world_size() : 1);
}

MlpFused MlpEngine::args() const {
  MlpFused f = f_;
  const int rank = comm_ ? comm_->rank() : (reducer_->peer() ? reducer_->peer()->rank() : 0);
  f.seed = seed_ + rank * 7919ull;  // per-rank data shard
  f.synth = external_ ? 0 : 1;
  f.fused_adam = reducer_->active() ? 0 : 1;
  f.w2_defer = mlp_w2_defer() && (f.fused_adam || merged_) ? 1 : 0;  // bucket 0 is not ready after K4 otherwise
  return f;
}

void MlpEngine::launch_step() {
  const MlpFused f = args();
  mlp_fused_forward(f, s_);
  if (f.fused_adam) {
    mlp_fused_backward2(f, s_);
    mlp_fused_backward1(f, s_);
    return;
  }
  Reducer& r = red();
  r.prepare();
  mlp_fused_backward2(f, s_);
  if (!merged_) r.mark_bucket_ready(0, s_);  // [l2, l3] all-reduce (side stream when overlapping) ...
  mlp_fused_backward1(f, s_);                // ... while K5 computes the l1 gradient
  r.mark_bucket_ready(merged_ ? 0 : 1, s_);
  r.finalize(s_);
  adam_step(f_.p, f_.g, f_.m, f_.v, f_.lr, f_.adam_state, 1.f / (float)world_size(), f_.b1, f_.b2, f_.eps, f_.wd,
            f_.eps_hat != 0, (int64_t)MlpLayout::total, s_);
}

void MlpEngine::step() { launch_step(); }

void MlpEngine::capture(int mode, int steps_per_graph) {
  if (mode == 0 || graphs_.captured()) return;
  graphs_.capture([this] { launch_step(); }, steps_per_graph);
}

void MlpEngine::replay(int n) { graphs_.replay(n, [this] { launch_step(); }); }

void MlpEngine::uncapture() {
  if (s_) MX_HIP_CHECK(hipStreamSynchronize(s_));
  graphs_.clear();
}

void MlpEngine::sync() { MX_HIP_CHECK(hipStreamSynchronize(s_)); }

void MlpEngine::set_peer(PeerComm* p) {
  if (p != reducer_->peer()) uncapture();
  reducer_->set_peer(p);
  merged_reducer_->set_peer(p);
}

void MlpEngine::set_comm(Comm* c) {
  if (c == comm_) return;
  MX_CHECK(!c || !comm_ || (c->rank() == comm_->rank() && c->world_size() == comm_->world_size()),
           "set_comm: the communicator must have this engine's rank and world size");
  uncapture();
  comm_ = c;
  reducer_->set_comm(c);
  merged_reducer_->set_comm(c);
}

void MlpEngine::set_force_collectives(bool on) {
  if (on != reducer_->forced()) uncapture();
  reducer_->set_force_collectives(on);
  merged_reducer_->set_force_collectives(on);
}

void MlpEngine::set_merged(bool on) {
  if (on != merged_) uncapture();
  merged_ = on;
}

void MlpEngine::set_overlap(bool on) {
  if (on != reducer_->overlap()) uncapture();
  reducer_->set_overlap(on);
}

void MlpEngine::set_bucket_padding(size_t capacity, size_t multiple) {
  reducer_->set_padding(MlpLayout::total, capacity, multiple);
  merged_reducer_->set_padding(MlpLayout::total, capacity, multiple);
}

}  // namespace mx
