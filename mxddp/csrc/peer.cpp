#include "peer.h"

#include <cstdlib>

#include "common.h"

namespace mx {

namespace {
constexpr size_t kSigBytes = 2ull * kPeerMaxBlocks * kPeerMaxRanks * sizeof(uint32_t);

// Uncached device memory that can be exported through HIP IPC; falls back to fine-grained
// (then the kernel also runs the acquire fences) and finally to ordinary device memory.
char* alloc_shared(size_t bytes, std::string* kind) {
  void* p = nullptr;
  if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) == hipSuccess) {
    hipIpcMemHandle_t h;
    if (hipIpcGetMemHandle(&h, p) == hipSuccess) {
      *kind = "uncached";
      return static_cast<char*>(p);
    }
    hipFree(p);
  }
  (void)hipGetLastError();
  if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained) == hipSuccess) {
    hipIpcMemHandle_t h;
    if (hipIpcGetMemHandle(&h, p) == hipSuccess) {
      *kind = "finegrained";
      return static_cast<char*>(p);
    }
    hipFree(p);
  }
  (void)hipGetLastError();
  MX_HIP_CHECK(hipMalloc(&p, bytes));
  *kind = "coarse";
  return static_cast<char*>(p);
}
}  // namespace

PeerComm::PeerComm(int rank, int world_size, int device, size_t cap_bytes, int blocks)
    : rank_(rank), ws_(world_size), dev_(device), blocks_(blocks) {
  MX_CHECK(world_size >= 1 && world_size <= kPeerMaxRanks, "peer transport: 1..8 ranks");
  MX_CHECK(rank >= 0 && rank < world_size, "peer transport: bad rank");
  MX_CHECK(blocks >= 1 && blocks <= kPeerMaxBlocks, "peer transport: 1..256 blocks");
  MX_HIP_CHECK(hipSetDevice(device));
  cap_ = (cap_bytes + 15) / 16 * 16;
  // one slot holds one rank's chunk (rounded to the 16-byte vector): ceil(cap / ws) + 16
  slot_bytes_ = ((cap_ + ws_ - 1) / ws_ + 16 + 255) / 256 * 256;
  xbytes_ = 4ull * ws_ * slot_bytes_;  // (scatter + gather region) x 2 call parities
  sbytes_ = kSigBytes;
  std::string k1, k2;
  xbuf_ = alloc_shared(xbytes_, &k1);
  sig_ = reinterpret_cast<uint32_t*>(alloc_shared(sbytes_, &k2));
  mem_kind_ = k1 == k2 ? k1 : k1 + "+" + k2;
  // uncached exchange memory: remote stores bypass the producer's L2 and every load of
  // exchanged bytes is `nt` from uncached memory (bypasses L1 and L2), so the consumer needs no
  // acquire; the release before each flag store is kept (it orders the flag behind the payload's
  // write acknowledgements on every path).  Cached fallbacks run both fences.
  fence_ = mem_kind_ == "uncached" ? 1 : 3;
  MX_HIP_CHECK(hipMemset(sig_, 0, sbytes_));
  MX_HIP_CHECK(hipMalloc(&epoch_, kPeerMaxBlocks * sizeof(uint32_t)));
  MX_HIP_CHECK(hipMemset(epoch_, 0, kPeerMaxBlocks * sizeof(uint32_t)));
  MX_HIP_CHECK(hipHostMalloc(&err_host_, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
  *err_host_ = 0;
  MX_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&err_dev_), err_host_, 0));
  if (const char* t = std::getenv("MXDDP_PEER_TIMEOUT_MS")) set_timeout_ms(std::atof(t));
  else timeout_ = 3000000000ll;  // 30 s: a slow rank (checkpoint, evaluation) is not an error
  MX_HIP_CHECK(hipDeviceSynchronize());
  peer_x_[rank_] = xbuf_;
  peer_sig_[rank_] = sig_;
}

PeerComm::~PeerComm() {
  hipSetDevice(dev_);
  hipDeviceSynchronize();
  for (int p = 0; p < ws_; ++p) {
    if (p == rank_ || !opened_ || local_) continue;
    if (peer_x_[p]) hipIpcCloseMemHandle(peer_x_[p]);
    if (peer_sig_[p]) hipIpcCloseMemHandle(peer_sig_[p]);
  }
  if (xbuf_) hipFree(xbuf_);
  if (sig_) hipFree(sig_);
  if (epoch_) hipFree(epoch_);
  if (err_host_) hipHostFree(err_host_);
}

std::string PeerComm::handles() const {
  hipIpcMemHandle_t h[2];
  MX_HIP_CHECK(hipIpcGetMemHandle(&h[0], xbuf_));
  MX_HIP_CHECK(hipIpcGetMemHandle(&h[1], sig_));
  return std::string(reinterpret_cast<const char*>(h), sizeof(h));
}

void PeerComm::open(const std::vector<std::string>& all) {
  MX_CHECK(!opened_, "peer transport already opened");
  MX_CHECK(static_cast<int>(all.size()) == ws_, "peer transport: need one handle blob per rank");
  MX_HIP_CHECK(hipSetDevice(dev_));
  for (int p = 0; p < ws_; ++p) {
    if (p == rank_) continue;
    MX_CHECK(all[p].size() == 2 * sizeof(hipIpcMemHandle_t), "peer transport: bad handle blob");
    hipIpcMemHandle_t h[2];
    std::memcpy(h, all[p].data(), sizeof(h));
    void* x = nullptr;
    void* s = nullptr;
    MX_HIP_CHECK(hipIpcOpenMemHandle(&x, h[0], hipIpcMemLazyEnablePeerAccess));
    MX_HIP_CHECK(hipIpcOpenMemHandle(&s, h[1], hipIpcMemLazyEnablePeerAccess));
    peer_x_[p] = static_cast<char*>(x);
    peer_sig_[p] = static_cast<uint32_t*>(s);
  }
  opened_ = true;
}

void PeerComm::open_local(const std::vector<PeerComm*>& all) {
  MX_CHECK(!opened_, "peer transport already opened");
  MX_CHECK(static_cast<int>(all.size()) == ws_, "peer transport: need one PeerComm per rank");
  MX_HIP_CHECK(hipSetDevice(dev_));
  for (int p = 0; p < ws_; ++p) {
    MX_CHECK(all[p] && all[p]->ws_ == ws_ && all[p]->rank_ == p, "peer transport: replicas out of rank order");
    MX_CHECK(all[p]->blocks_ == blocks_ && all[p]->slot_bytes_ == slot_bytes_, "peer transport: replica shapes differ");
    if (p == rank_) continue;
    const int d = all[p]->dev_;
    if (d != dev_) {
      int can = 0;
      MX_HIP_CHECK(hipDeviceCanAccessPeer(&can, dev_, d));
      MX_CHECK(can, "peer transport: no peer access between the replicas' devices");
      const hipError_t e = hipDeviceEnablePeerAccess(d, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) MX_HIP_CHECK(e);
      (void)hipGetLastError();
    }
    peer_x_[p] = all[p]->xbuf_;
    peer_sig_[p] = all[p]->sig_;
  }
  opened_ = local_ = true;
}

void PeerComm::set_blocks(int b) {
  MX_CHECK(b >= 1 && b <= kPeerMaxBlocks, "peer transport: 1..256 blocks");
  blocks_ = b;  // every rank must use the same value (flag sets are per block)
}

void PeerComm::reset_state() {
  MX_HIP_CHECK(hipSetDevice(dev_));
  MX_HIP_CHECK(hipDeviceSynchronize());
  MX_HIP_CHECK(hipMemset(sig_, 0, sbytes_));
  MX_HIP_CHECK(hipMemset(epoch_, 0, kPeerMaxBlocks * sizeof(uint32_t)));
  MX_HIP_CHECK(hipDeviceSynchronize());
  reset_error();
}

int PeerComm::error() const { return __atomic_load_n(err_host_, __ATOMIC_ACQUIRE); }
void PeerComm::reset_error() { __atomic_store_n(err_host_, 0, __ATOMIC_RELEASE); }

bool PeerComm::coschedule_args(void* data, size_t count, RedOp op, PeerArgs* a, PeerPartition* part) const {
  if (ws_ == 1 || count == 0 || !opened_ || count * 4 > cap_) return false;
  if (reinterpret_cast<uintptr_t>(data) % 16) return false;
  *a = PeerArgs{};
  for (int p = 0; p < ws_; ++p) {
    a->xbuf[p] = peer_x_[p];
    a->sig[p] = peer_sig_[p];
  }
  a->epoch = epoch_;
  a->err = err_dev_;
  a->slot_bytes = static_cast<long long>(slot_bytes_);
  a->timeout = timeout_;
  a->rank = rank_;
  a->ws = ws_;
  a->fence = fence_ | ((withhold_ & 2) ? 4 : 0);
  a->scale = op == RedOp::kAvg ? 1.f / static_cast<float>(ws_) : 1.f;
  a->data = data;
  a->count = static_cast<long long>(count);
  *part = PeerPartition::make(a->count, ws_, blocks_, 4);
  return part->chunk * 4 <= a->slot_bytes;
}

bool PeerComm::oneshot_args(void* data, size_t count, RedOp op, PeerArgs* a) const {
  PeerPartition part{};
  if (!coschedule_args(data, count, op, a, &part)) return false;
  return static_cast<long long>(count) * 4 <= a->slot_bytes;
}

void PeerComm::all_reduce(void* data, size_t count, DType t, hipStream_t st, RedOp op) {
  if (ws_ == 1 || count == 0) return;
  MX_CHECK(op == RedOp::kSum || op == RedOp::kAvg, "peer transport: sum or average only");
  MX_CHECK(opened_, "peer transport: open() the peer handles first");
  const size_t esz = dtype_size(t);
  const size_t per = cap_ / esz;  // elements per launch
  PeerArgs a{};
  for (int p = 0; p < ws_; ++p) {
    a.xbuf[p] = peer_x_[p];
    a.sig[p] = peer_sig_[p];
  }
  a.epoch = epoch_;
  a.err = err_dev_;
  a.slot_bytes = static_cast<long long>(slot_bytes_);
  a.timeout = timeout_;
  a.rank = rank_;
  a.ws = ws_;
  a.fence = fence_ | ((withhold_ & 1) ? 4 : 0);
  a.scale = op == RedOp::kAvg ? 1.f / static_cast<float>(ws_) : 1.f;
  for (size_t off = 0; off < count; off += per) {
    a.data = static_cast<char*>(data) + off * esz;
    a.count = static_cast<long long>(count - off < per ? count - off : per);
    peer_all_reduce_launch(a, t, blocks_, st, oneshot_bytes_);
  }
}

}  // namespace mx
