#include "mnist_engine.h"

#include "common.h"
#include "ops.h"
#include "mnist_kernels.h"

namespace mx {

namespace {
constexpr size_t kAlign = 64;  // floats (256 B)
inline size_t al(size_t n) { return (n + kAlign - 1) / kAlign * kAlign; }
struct Carve {
  char* base;
  size_t off = 0, cap;
  template <class T>
  T* take(size_t n) {
    T* p = reinterpret_cast<T*>(base + off * 4);
    off += al(n * sizeof(T) / 4 + 1);
    MX_CHECK(off * 4 <= cap, "mnist engine workspace too small");
    return p;
  }
};
size_t ws_floats(int B) {
  size_t t = 0;
  auto add = [&](size_t n) { t += al(n + 1); };
  add(B * 784);            // x
  add(B);                  // y
  add((size_t)B * 21632);  // a1
  add((size_t)B * 36864);  // c2
  add((size_t)B * 9216);   // pool
  add((size_t)B * 9216);   // idx
  add(B * 256);            // h (int64 fixed point)
  add(B * 10);             // logits
  add(B * 10);             // dlogits
  add(B * 128);            // dh
  add((size_t)B * 9216);   // dp
  add((size_t)B * 36864);  // dc2
  add((size_t)B * 21632);  // da1
  add(10 * 784);           // templates
  add(4);                  // counter
  add(mnist_fused_scratch_floats(B));
  return t;
}
}  // namespace

// every [B] buffer has the padded row count of the fused kernels (16-row MFMA tiles)
size_t MnistLayout::workspace_bytes(int B) { return ws_floats(MnistLayout::padded(B)) * 4; }

MnistEngine::MnistEngine(int batch, uintptr_t params, uintptr_t grads, uintptr_t mom, uintptr_t workspace,
                         size_t workspace_bytes, Comm* comm, uint64_t seed, float momentum, float weight_decay,
                         uintptr_t lr_dev, uintptr_t metrics_dev, int kernel_variant)
    : B_(batch), p_(reinterpret_cast<float*>(params)), g_(reinterpret_cast<float*>(grads)),
      m_(reinterpret_cast<float*>(mom)), lr_(reinterpret_cast<float*>(lr_dev)),
      metrics_(reinterpret_cast<float*>(metrics_dev)), comm_(comm), seed_(seed), momentum_(momentum),
      wd_(weight_decay), variant_(kernel_variant) {
  MX_CHECK(B_ > 0, "batch must be positive");
  // the fused kernels run whole 16-row tiles: a partial last tile is padded with rows that carry
  // no loss (F5 masks them); the generic variant runs the exact batch
  Bp_ = variant_ == 1 ? MnistLayout::padded(B_) : B_;
  Carve c{reinterpret_cast<char*>(workspace), 0, workspace_bytes};
  x_ = c.take<float>(Bp_ * 784);
  y_ = c.take<int32_t>(Bp_);
  a1_ = c.take<float>((size_t)Bp_ * 21632);
  c2_ = c.take<float>((size_t)Bp_ * 36864);
  pool_ = c.take<float>((size_t)Bp_ * 9216);
  idx_ = c.take<int32_t>((size_t)Bp_ * 9216);
  h_ = c.take<float>(Bp_ * 256);  // int64 [B][128] on the fused path, float [B][128] on the generic one
  logits_ = c.take<float>(Bp_ * 10);
  dlogits_ = c.take<float>(Bp_ * 10);
  dh_ = c.take<float>(Bp_ * 128);
  dp_ = c.take<float>((size_t)Bp_ * 9216);
  dc2_ = c.take<float>((size_t)Bp_ * 36864);
  da1_ = c.take<float>((size_t)Bp_ * 21632);
  tmpl_ = c.take<float>(10 * 784);
  counter_ = c.take<int32_t>(4);
  scratch_ = c.take<float>(mnist_fused_scratch_floats(Bp_));
  MX_HIP_CHECK(hipStreamCreateWithFlags(&s_, hipStreamNonBlocking));
  MX_HIP_CHECK(hipMemsetAsync(counter_, 0, 16, s_));
  // a caller's batch fills rows 0..B-1 only: the pad rows stay finite zeros (0 * NaN would not)
  MX_HIP_CHECK(hipMemsetAsync(x_, 0, sizeof(float) * Bp_ * 784, s_));
  MX_HIP_CHECK(hipMemsetAsync(y_, 0, sizeof(int32_t) * Bp_, s_));
  synth_templates(tmpl_, 10, 784, seed_ ^ 0x5eedull, s_);  // identical on every rank
  // Two buckets in backward order: [fc1.w .. fc2.b] (4.72 MB, ready right after the fc
  // backward) and [conv1.w .. conv2.b] (75 KB, ready at the end).  The big bucket's
  // all-reduce overlaps the whole conv backward.
  std::vector<Reducer::BucketSpec> buckets = {
      {MnistLayout::fw1, MnistLayout::total - MnistLayout::fw1},
      {0, MnistLayout::fw1},
  };
  reducer_ = std::make_unique<Reducer>(comm_, reinterpret_cast<uintptr_t>(g_), DType::kF32, buckets,
                                       std::vector<int>{1, 1, 1, 1, 0, 0, 0, 0}, RedOp::kSum, false);
  merged_reducer_ = std::make_unique<Reducer>(
      comm_, reinterpret_cast<uintptr_t>(g_), DType::kF32, std::vector<Reducer::BucketSpec>{{0, MnistLayout::total}},
      std::vector<int>(8, 0), RedOp::kSum, false);
  merged_reducer_->set_overlap(false);  // issued at the end of the backward: nothing to overlap
  co_reducer_ = std::make_unique<Reducer>(
      comm_, reinterpret_cast<uintptr_t>(g_), DType::kF32, std::vector<Reducer::BucketSpec>{{0, MnistLayout::fw1}},
      std::vector<int>(8, 0), RedOp::kSum, false);
  co_reducer_->set_overlap(false);
  repack();
  MX_HIP_CHECK(hipStreamSynchronize(s_));
}

void MnistEngine::set_comm(Comm* c) {
  if (c == comm_) return;
  MX_CHECK(!c || !comm_ || (c->rank() == comm_->rank() && c->world_size() == comm_->world_size()),
           "set_comm: the communicator must have this engine's rank and world size");
  uncapture();
  comm_ = c;
  reducer_->set_comm(c);
  merged_reducer_->set_comm(c);
  co_reducer_->set_comm(c);
}

bool MnistEngine::set_coscheduled(bool on) {
  if (on) {
    PeerComm* pc = reducer_->peer();
    if (!pc || variant_ != 1 ||
        !pc->coschedule_args(g_ + MnistLayout::fw1, MnistLayout::total - MnistLayout::fw1, RedOp::kSum, &co_args_,
                             &co_part_) ||
        pc->blocks() % 8 != 0)
      on = false;
  }
  if (on != coscheduled_) uncapture();
  coscheduled_ = on;
  return on;
}

void MnistEngine::repack() {
  if (variant_ == 1) mnist_fused_init(fused_args(), s_);
}

void MnistEngine::uncapture() {
  if (s_) MX_HIP_CHECK(hipStreamSynchronize(s_));
  if (exec_) hipGraphExecDestroy(exec_);
  if (graph_) hipGraphDestroy(graph_);
  exec_ = nullptr;
  graph_ = nullptr;
  for (auto& e : rem_exec_) hipGraphExecDestroy(e.second);
  for (auto g : rem_graph_) hipGraphDestroy(g);
  rem_exec_.clear();
  rem_graph_.clear();
  for (int k = 0; k < 3; ++k) {
    if (seg_exec_[k]) hipGraphExecDestroy(seg_exec_[k]);
    if (seg_graph_[k]) hipGraphDestroy(seg_graph_[k]);
    seg_exec_[k] = nullptr;
    seg_graph_[k] = nullptr;
  }
  graph_mode_ = 0;
}

MnistEngine::~MnistEngine() {
  uncapture();
  reducer_.reset();
  merged_reducer_.reset();
  co_reducer_.reset();
  if (s_) hipStreamDestroy(s_);
}

void MnistEngine::fwd(const float* x, float* logits_out, int B) {
  using L = MnistLayout;
  const ConvShape s1 = ConvShape::make(B, 1, 28, 28, 32, 3, 3, 1, 1, 0, 0);
  const ConvShape s2 = ConvShape::make(B, 32, 26, 26, 64, 3, 3, 1, 1, 0, 0);
  conv2d_fwd(x, p_ + L::w1, p_ + L::b1, a1_, s1, true, s_);
  conv2d_fwd(a1_, p_ + L::w2, p_ + L::b2, c2_, s2, true, s_);
  maxpool2d_fwd(c2_, pool_, idx_, B, 64, 24, 24, 2, 2, 2, 2, 0, 0, 12, 12, s_);
  linear_fwd(pool_, p_ + L::fw1, p_ + L::fb1, h_, B, 128, 9216, false, s_);
  relu_fwd(h_, h_, (int64_t)B * 128, s_);
  linear_fwd(h_, p_ + L::fw2, p_ + L::fb2, logits_out, B, 10, 128, false, s_);
}

MnistFused MnistEngine::fused_args() const {
  const int rank = comm_ ? comm_->rank() : (reducer_ && reducer_->peer() ? reducer_->peer()->rank() : 0);
  const uint64_t data_seed = seed_ + rank * 7919ull;  // per-rank data shard
  MnistFused f{};
  f.B = Bp_;
  f.nB = B_;
  f.x = x_;
  f.y = y_;
  f.p = p_;
  f.g = g_;
  f.a1 = a1_;
  f.pool = pool_;
  f.idx = idx_;
  f.h = reinterpret_cast<long long*>(h_);
  f.dh = dh_;
  f.dp = dp_;
  f.scratch = scratch_;
  f.metrics = metrics_;
  f.counter = counter_;
  f.tmpl = tmpl_;
  f.seed = data_seed;
  f.trace = trace_;
  f.synth = external_batch_ ? 0 : 1;
  // without gradient collectives F5 applies the fc1 weight update itself (no all-reduce has to
  // come between the gradient and the update)
  f.fc1_sgd = (variant_ == 1 && !reducer_->active()) ? 1 : 0;
  // the deferred update's blocks stage dh + a pool slice in F67's LDS: batch <= 96
  // mode 2 runs F67 at three blocks per CU with the fc1 blocks' dh + pool slice in LDS: batch
  // <= 64; mode 1 (two per CU): batch <= 96; otherwise F5 keeps the update
  // With gradient collectives the fc1 weight gradient may move into F67 too (written to g, the
  // update stays in the SGD launch) -- but only when nothing exchanges the fc bucket before F67
  // ends: one merged all-reduce after the conv backward, no co-scheduled exchange.
  const int dm = mnist_fc1_defer();
  const bool can = variant_ == 1 && (f.fc1_sgd || (merged_ && !co_active()));
  f.fc1_defer = (can && ((dm == 2 && Bp_ <= 64) || (dm == 1 && Bp_ <= 96))) ? dm : 0;
  f.mom = m_;
  f.lr = lr_;
  f.sgd_mom = momentum_;
  f.sgd_wd = wd_;
  f.wt = mnist_wt_stores();
  if (co_active()) {
    f.co_blocks = reducer_->peer()->blocks();
    f.co_args = co_args_;
    f.co_part = co_part_;
  }
  return f;
}

// Segment 0: batch + forward + head + fc backward  -> bucket 0 (fc grads, 4.72 MB) is complete.
void MnistEngine::segment(int k) {
  using L = MnistLayout;
  const int B = B_;
  const ConvShape s1 = ConvShape::make(B, 1, 28, 28, 32, 3, 3, 1, 1, 0, 0);
  const ConvShape s2 = ConvShape::make(B, 32, 26, 26, 64, 3, 3, 1, 1, 0, 0);
  if (k == 0) {
    if (variant_ == 0) {  // reference path: generic implicit-GEMM kernels, one op per launch
      if (!external_batch_) synth_batch(x_, y_, tmpl_, B, 784, 10, fused_args().seed, counter_, s_, true);
      fwd(x_, logits_, B);
      xent_fwd_bwd(logits_, y_, nullptr, dlogits_, metrics_, metrics_ + 1, B, 10, 1.f / B, s_);
      linear_wgrad(dlogits_, h_, g_ + L::fw2, B, 10, 128, false, s_);
      bias_grad(dlogits_, g_ + L::fb2, B, 10, 1, false, s_);
      linear_dgrad(dlogits_, p_ + L::fw2, dh_, B, 10, 128, h_, false, s_);
      linear_wgrad(dh_, pool_, g_ + L::fw1, B, 128, 9216, false, s_);
      bias_grad(dh_, g_ + L::fb1, B, 128, 1, false, s_);
      linear_dgrad(dh_, p_ + L::fw1, dp_, B, 128, 9216, nullptr, false, s_);
    } else {  // fused path (mnist_kernels.hip): the batch is generated inside F1
      const MnistFused f = fused_args();
      mnist_fused_forward(f, s_);
      mnist_fused_fc1_bwd(f, s_);
    }
  } else if (k == 1) {  // conv backward -> bucket 1 (conv grads, 75 KB) complete
    if (variant_ == 0) {
      maxpool2d_bwd(dp_, idx_, dc2_, B, 64, 24, 24, 12, 12, s_);
      relu_bwd(dc2_, c2_, dc2_, (int64_t)B * 36864, s_);
      conv2d_wgrad(dc2_, a1_, g_ + L::w2, s2, false, s_);
      bias_grad(dc2_, g_ + L::b2, B, 64, 576, false, s_);
      conv2d_dgrad(dc2_, p_ + L::w2, da1_, s2, a1_, false, s_);
      conv2d_wgrad(da1_, x_, g_ + L::w1, s1, false, s_);
      bias_grad(da1_, g_ + L::b1, B, 32, 676, false, s_);
    } else {
      // no gradient collectives this step: F8's finalize folds into the SGD launch
      mnist_fused_conv_bwd(fused_args(), s_, !reducer_->active());
    }
  } else {  // optimizer: flat SGD, DDP's 1/world_size average folded into the update
    const int ws = world_size();
    if (variant_ == 0)
      sgd_step(p_, g_, m_, lr_, 1.f / ws, momentum_, wd_, (int64_t)L::total, false, s_);
    else  // + conv2 weight repack for the next step's F2/F7 + conv2 bias-grad reset
      mnist_fused_sgd(fused_args(), m_, lr_, 1.f / ws, momentum_, wd_, s_, !reducer_->active());
  }
}

void MnistEngine::launch_step() {
  if (co_active()) {
    Reducer& rc = *co_reducer_;
    rc.prepare();
    segment(0);                   // ... F5: the fc bucket is complete
    segment(1);                   // F67 (its first blocks all-reduce the fc bucket) + F8
    rc.mark_bucket_ready(0, s_);  // the 75 KB conv bucket
    rc.finalize(s_);
    segment(2);
    return;
  }
  Reducer& r = red();
  r.prepare();
  segment(0);
  if (!merged_) r.mark_bucket_ready(0, s_);  // fc grads all-reduce on the side stream ...
  segment(1);                                // ... overlapped with the whole conv backward
  r.mark_bucket_ready(merged_ ? 0 : 1, s_);
  r.finalize(s_);                            // compute stream waits for the comm stream
  segment(2);
}

void MnistEngine::step() { launch_step(); }

hipGraphExec_t MnistEngine::capture_fn(const std::function<void()>& fn, hipGraph_t* g) {
  MX_HIP_CHECK(hipStreamBeginCapture(s_, hipStreamCaptureModeThreadLocal));
  try {
    fn();
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

void MnistEngine::capture(int mode, int steps_per_graph) {
  if (exec_ || seg_exec_[0]) return;
  const bool multi = world_size() > 1;
  // default: one graph at world size 1; eager launches (mode 0) when real collectives run --
  // the caller (FusedMnistTrainer.autotune) may pick a graph mode after timing the options.
  if (mode < 0) mode = multi ? 0 : 1;
  if (mode == 2 && co_active()) mode = 1;  // the fc exchange lives inside segment 1's launch
  MX_HIP_CHECK(hipStreamSynchronize(s_));
  graph_mode_ = mode;
  if (mode == 1) {  // whole step(s), RCCL collectives included (one launch per group of steps)
    steps_per_graph_ = steps_per_graph < 1 ? 1 : steps_per_graph;
    exec_ = capture_fn([this] {
      for (int i = 0; i < steps_per_graph_; ++i) launch_step();
    }, &graph_);
    int k = 1;
    while (2 * k < steps_per_graph_) k *= 2;
    for (; k >= 1 && steps_per_graph_ > 1; k /= 2) {
      hipGraph_t g = nullptr;
      hipGraphExec_t e = capture_fn([this, k] {
        for (int i = 0; i < k; ++i) launch_step();
      }, &g);
      rem_graph_.push_back(g);
      rem_exec_.emplace_back(k, e);
    }
  } else if (mode == 2) {  // three compute graphs; the two collectives are issued eagerly between them
    for (int k = 0; k < 3; ++k) seg_exec_[k] = capture_fn([this, k] { segment(k); }, &seg_graph_[k]);
  }
}

void MnistEngine::replay(int n) {
  if (graph_mode_ == 1 && exec_ && steps_per_graph_ > 1) {
    // remainder from the 2^k-step graphs.  small_first_: launched smallest first, ahead of the
    // full groups, so the device starts on a short graph while the host submits the long ones
    // (driver-length run 824-826k vs 827-833k img/s full groups first: off by default)
    const int full = n / steps_per_graph_;
    n -= full * steps_per_graph_;
    std::vector<hipGraphExec_t> rem;
    for (const auto& e : rem_exec_)  // rem_exec_ is largest first
      if (n >= e.first) {
        rem.push_back(e.second);
        n -= e.first;
      }
    if (!small_first_) {
      for (int i = 0; i < full; ++i) MX_HIP_CHECK(hipGraphLaunch(exec_, s_));
      for (auto e : rem) MX_HIP_CHECK(hipGraphLaunch(e, s_));
    } else {
      for (auto it = rem.rbegin(); it != rem.rend(); ++it) MX_HIP_CHECK(hipGraphLaunch(*it, s_));
      for (int i = 0; i < full; ++i) MX_HIP_CHECK(hipGraphLaunch(exec_, s_));
    }
    for (; n > 0; --n) launch_step();
    return;
  }
  for (int i = 0; i < n; ++i) {
    if (graph_mode_ == 1 && exec_) {
      MX_HIP_CHECK(hipGraphLaunch(exec_, s_));
    } else if (graph_mode_ == 2 && seg_exec_[0]) {
      Reducer& r = red();
      r.prepare();
      MX_HIP_CHECK(hipGraphLaunch(seg_exec_[0], s_));
      if (!merged_) r.mark_bucket_ready(0, s_);
      MX_HIP_CHECK(hipGraphLaunch(seg_exec_[1], s_));
      r.mark_bucket_ready(merged_ ? 0 : 1, s_);
      r.finalize(s_);
      MX_HIP_CHECK(hipGraphLaunch(seg_exec_[2], s_));
    } else {
      launch_step();
    }
  }
}

int MnistEngine::warm_graphs() {
  // one launch of every captured multi-step graph (each is a real training step group): the
  // first launch of a graph exec pays one-time costs the later launches do not
  if (graph_mode_ != 1 || !exec_) return 0;
  int steps = steps_per_graph_;
  MX_HIP_CHECK(hipGraphLaunch(exec_, s_));
  for (const auto& e : rem_exec_) {
    MX_HIP_CHECK(hipGraphLaunch(e.second, s_));
    steps += e.first;
  }
  MX_HIP_CHECK(hipStreamSynchronize(s_));
  return steps;
}

void MnistEngine::forward_only(uintptr_t x, uintptr_t logits, int B) {
  MX_CHECK(B <= B_, "eval batch larger than engine batch");
  fwd(reinterpret_cast<const float*>(x), reinterpret_cast<float*>(logits), B);
  // the generic forward stores into h_, which the fused F3 uses as a zeroed split-K accumulator
  if (variant_ == 1) MX_HIP_CHECK(hipMemsetAsync(h_, 0, sizeof(long long) * Bp_ * 128, s_));
}

void MnistEngine::sync() { MX_HIP_CHECK(hipStreamSynchronize(s_)); }

}  // namespace mx
