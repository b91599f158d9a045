#include "comm.h"

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>

#include "common.h"

namespace mx {

#define MX_NCCL_CHECK(expr)                                                                     \
  do {                                                                                           \
    ncclResult_t r_ = (expr);                                                                    \
    if (r_ != ncclSuccess)                                                                       \
      throw std::runtime_error(std::string("RCCL error '") + ncclGetErrorString(r_) + "' at " + \
                               __FILE__ ":" + std::to_string(__LINE__) + ": " #expr);           \
  } while (0)

ncclDataType_t to_nccl(DType t) {
  switch (t) {
    case DType::kF32: return ncclFloat32;
    case DType::kBF16: return ncclBfloat16;
    case DType::kF16: return ncclFloat16;
    case DType::kI32: return ncclInt32;
    case DType::kI64: return ncclInt64;
    case DType::kU8: return ncclUint8;
  }
  throw std::runtime_error("bad dtype");
}

ncclRedOp_t to_nccl(RedOp o) {
  switch (o) {
    case RedOp::kSum: return ncclSum;
    case RedOp::kAvg: return ncclAvg;
    case RedOp::kMax: return ncclMax;
    case RedOp::kMin: return ncclMin;
    case RedOp::kProd: return ncclProd;
  }
  throw std::runtime_error("bad op");
}

size_t dtype_size(DType t) {
  switch (t) {
    case DType::kF32: case DType::kI32: return 4;
    case DType::kBF16: case DType::kF16: return 2;
    case DType::kI64: return 8;
    case DType::kU8: return 1;
  }
  return 0;
}

std::string Comm::new_unique_id() {
  ncclUniqueId id;
  MX_NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

std::string CommConfig::name() const {
  if (ctas <= 0 && algo.empty() && proto.empty()) return "default";
  std::string n = algo.empty() ? "auto" : algo;
  if (!proto.empty()) n += "/" + proto;
  if (ctas > 0) n += ":c" + std::to_string(ctas);
  return n;
}

namespace {
// The communicator-config prefix that every RCCL >= 2.18 understands.  The headers here are
// newer (2.27) than the RCCL inside the PyTorch wheel this module links (2.26): RCCL copies
// `size` bytes of the caller's struct over its defaults, so handing it the 2.27 struct would
// write past its own.  The fields after splitShare keep RCCL's defaults.
struct CommConfigV218 {
  size_t size;
  unsigned int magic, version;
  int blocking, cgaClusterSize, minCTAs, maxCTAs;
  const char* netName;
  int splitShare;
};

// Watchdog of one blocking communicator init: if the init has not returned `seconds` after the
// guard was made, a helper thread names what was being initialised and ends the process with
// Comm::kInitTimeoutExit (the driver / launcher sees a non-zero exit instead of a hang).
class InitDeadline {
 public:
  InitDeadline(double seconds, std::string what) {
    if (seconds <= 0) return;
    th_ = std::thread([this, seconds, what = std::move(what)] {
      std::unique_lock<std::mutex> lk(mu_);
      if (cv_.wait_for(lk, std::chrono::duration<double>(seconds), [this] { return done_; })) return;
      std::fprintf(stderr,
                   "mxddp: RCCL communicator init did not complete within %.0f s: %s -- a rank never joined the "
                   "rendezvous or RCCL's bootstrap is wedged; exiting with code %d (MXDDP_RCCL_INIT_TIMEOUT_S sets the "
                   "deadline)\n",
                   seconds, what.c_str(), Comm::kInitTimeoutExit);
      std::fflush(stderr);
      std::_Exit(Comm::kInitTimeoutExit);
    });
  }
  ~InitDeadline() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      done_ = true;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
  }
  InitDeadline(const InitDeadline&) = delete;
  InitDeadline& operator=(const InitDeadline&) = delete;

 private:
  std::thread th_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool done_ = false;
};

double g_init_timeout_s = -1.0;  // < 0: not read from the environment yet

// NCCL_ALGO / NCCL_PROTO for the duration of one communicator init
class ScopedEnv {
 public:
  ScopedEnv(const char* key, const std::string& val) : key_(key) {
    if (val.empty()) return;
    const char* old = std::getenv(key);
    had_ = old != nullptr;
    if (had_) old_ = old;
    setenv(key, val.c_str(), 1);
    set_ = true;
  }
  ~ScopedEnv() {
    if (!set_) return;
    if (had_) setenv(key_, old_.c_str(), 1);
    else unsetenv(key_);
  }

 private:
  const char* key_;
  std::string old_;
  bool had_ = false, set_ = false;
};
}  // namespace

int Comm::version() {
  int v = 0;
  MX_NCCL_CHECK(ncclGetVersion(&v));
  return v;
}

void Comm::set_init_timeout(double seconds) { g_init_timeout_s = seconds <= 0 ? 0.0 : seconds; }

double Comm::init_timeout() {
  if (g_init_timeout_s < 0) {
    const char* e = std::getenv("MXDDP_RCCL_INIT_TIMEOUT_S");
    g_init_timeout_s = e ? std::max(0.0, std::atof(e)) : 120.0;
  }
  return g_init_timeout_s;
}

int Comm::nranks() const {
  int n = 0;
  MX_NCCL_CHECK(ncclCommCount(comm_, &n));
  return n;
}

int Comm::hip_device() const {
  int d = -1;
  MX_NCCL_CHECK(ncclCommCuDevice(comm_, &d));
  return d;
}

Comm::Comm(const std::string& uid, int rank, int world_size, int device, const CommConfig& cfg)
    : rank_(rank), ws_(world_size), device_(device), cfg_(cfg) {
  MX_CHECK(uid.size() == sizeof(ncclUniqueId), "unique id has wrong size");
  ncclUniqueId id;
  std::memcpy(&id, uid.data(), sizeof(id));
  MX_HIP_CHECK(hipSetDevice(device));
  InitDeadline deadline(init_timeout(), "rank " + std::to_string(rank) + " of " + std::to_string(world_size) +
                                            ", device " + std::to_string(device) + ", variant '" + cfg.name() + "'");
  ScopedEnv algo("NCCL_ALGO", cfg.algo), proto("NCCL_PROTO", cfg.proto);
  if (cfg.ctas > 0) {
    // the prefix struct is only valid for a linked RCCL that reads the >= 2.18 config layout (it
    // copies `size` bytes and checks magic / version): refuse anything older with a clear error
    // instead of handing it a struct it would misread
    int v = 0;
    MX_NCCL_CHECK(ncclGetVersion(&v));
    MX_CHECK(v >= NCCL_VERSION(2, 18, 0),
             "RCCL " + std::to_string(v) + " is older than 2.18: pinned-CTA communicator variants ('" + cfg.name() +
                 "') need ncclCommInitRankConfig's 2.18 config layout; use the default variant");
    CommConfigV218 c{sizeof(CommConfigV218), 0xcafebeef, NCCL_VERSION(2, 18, 0), 1,
                     NCCL_CONFIG_UNDEF_INT, cfg.ctas, cfg.ctas, nullptr, NCCL_CONFIG_UNDEF_INT};
    MX_NCCL_CHECK(ncclCommInitRankConfig(&comm_, world_size, id, rank, reinterpret_cast<ncclConfig_t*>(&c)));
  } else {
    MX_NCCL_CHECK(ncclCommInitRank(&comm_, world_size, id, rank));
  }
}

Comm::Comm(ncclComm_t c, int rank, int world_size, int device)
    : comm_(c), rank_(rank), ws_(world_size), device_(device) {}

Comm::~Comm() {
  if (comm_ && !aborted_) ncclCommDestroy(comm_);
}

std::vector<Comm*> Comm::init_all(const std::vector<int>& devices) {
  std::vector<ncclComm_t> comms(devices.size());
  {
    InitDeadline deadline(init_timeout(), "ncclCommInitAll over " + std::to_string(devices.size()) + " devices");
    MX_NCCL_CHECK(ncclCommInitAll(comms.data(), (int)devices.size(), devices.data()));
  }
  std::vector<Comm*> out;
  for (size_t i = 0; i < devices.size(); ++i) out.push_back(new Comm(comms[i], (int)i, (int)devices.size(), devices[i]));
  return out;
}

void Comm::all_reduce(const void* send, void* recv, size_t count, DType t, RedOp op, hipStream_t st) {
  MX_NCCL_CHECK(ncclAllReduce(send, recv, count, to_nccl(t), to_nccl(op), comm_, st));
}
void Comm::broadcast(const void* send, void* recv, size_t count, DType t, int root, hipStream_t st) {
  MX_NCCL_CHECK(ncclBroadcast(send, recv, count, to_nccl(t), root, comm_, st));
}
void Comm::reduce_scatter(const void* send, void* recv, size_t recv_count, DType t, RedOp op, hipStream_t st) {
  MX_NCCL_CHECK(ncclReduceScatter(send, recv, recv_count, to_nccl(t), to_nccl(op), comm_, st));
}
void Comm::all_gather(const void* send, void* recv, size_t send_count, DType t, hipStream_t st) {
  MX_NCCL_CHECK(ncclAllGather(send, recv, send_count, to_nccl(t), comm_, st));
}
void Comm::all_to_all(const void* send, void* recv, size_t count, DType t, hipStream_t st) {
  const size_t esz = dtype_size(t);
  MX_NCCL_CHECK(ncclGroupStart());
  for (int p = 0; p < ws_; ++p) {
    MX_NCCL_CHECK(ncclSend(static_cast<const char*>(send) + p * count * esz, count, to_nccl(t), p, comm_, st));
    MX_NCCL_CHECK(ncclRecv(static_cast<char*>(recv) + p * count * esz, count, to_nccl(t), p, comm_, st));
  }
  MX_NCCL_CHECK(ncclGroupEnd());
}
void Comm::send(const void* buf, size_t count, DType t, int peer, hipStream_t st) {
  MX_NCCL_CHECK(ncclSend(buf, count, to_nccl(t), peer, comm_, st));
}
void Comm::recv(void* buf, size_t count, DType t, int peer, hipStream_t st) {
  MX_NCCL_CHECK(ncclRecv(buf, count, to_nccl(t), peer, comm_, st));
}
void Comm::check_async_error() const {
  ncclResult_t r = ncclSuccess;
  MX_NCCL_CHECK(ncclCommGetAsyncError(comm_, &r));
  if (r != ncclSuccess && r != ncclInProgress)
    throw std::runtime_error(std::string("RCCL async error: ") + ncclGetErrorString(r));
}
void Comm::abort() {
  if (comm_ && !aborted_) {
    ncclCommAbort(comm_);
    aborted_ = true;
  }
}
void Comm::group_start() { MX_NCCL_CHECK(ncclGroupStart()); }
void Comm::group_end() { MX_NCCL_CHECK(ncclGroupEnd()); }

}  // namespace mx
