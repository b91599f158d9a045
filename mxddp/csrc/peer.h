// Direct peer-to-peer all-reduce over xGMI ("peer transport").
//
// An 8x MI355X node is a FULLY CONNECTED xGMI mesh: every GPU has one point-to-point link to
// each of its 7 peers.  A ring all-reduce (RCCL's default) moves each byte through 2(W-1)
// link hops one after another, and at the message sizes of this framework's gradient
// buckets (4.7 MB for the MNIST CNN) it is latency bound.  The peer transport is a two-shot
// all-reduce that drives ALL 7 links at once, in ONE kernel per bucket:
//
//   1. scatter  : rank r stores chunk p of its bucket into rank p's exchange buffer (slot r),
//                 for every peer p at the same time (one link each);
//   2. reduce   : rank r sums chunk r over all W slots in a FIXED rank order (so every rank
//                 ends with bit-identical values), writes it back, and stores the sum into
//                 every peer's gather slot r;
//   3. gather   : rank r copies the other W-1 reduced chunks from its gather slots.
//
// Each link carries 2 * S / W bytes per bucket (S = bucket bytes).  Buckets up to 256 KB take a
// one-shot kernel instead (every rank pushes its whole bucket to every peer, one flag round, each
// rank sums all W copies in rank order): S bytes per link, but one synchronisation round
// fewer, which is what a small all-reduce costs.  Synchronisation is per
// workgroup: block b of rank r only waits for block b of the peers (flags, no grid barrier).
// The exchange buffers and flags live in UNCACHED device memory (hipDeviceMallocUncached)
// shared between the processes through HIP IPC handles: remote stores land in the owner's
// HBM, and local reads of them are `nt` loads of uncached memory (bypass L1 and L2), so no
// cache holds a stale copy.  Every wait is bounded: a peer that never arrives sets an error word in
// host-mapped memory and the kernel exits (PeerComm::error()), so a broken peer can never
// leave waves spinning on the GPU.
//
// Where the reference's DDP rides NCCL's ring (pytorch/distributed_data_parallel.py:74,132),
// this is selected per machine: FusedMnistTrainer.autotune / the DDP reducer time it against
// RCCL (and validate the result against RCCL's) before using it.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "comm.h"

namespace mx {

constexpr int kPeerMaxRanks = 8;
constexpr int kPeerMaxBlocks = 256;

struct PeerArgs {
  char* xbuf[kPeerMaxRanks];      // every rank's exchange buffer (mapped into this process)
  uint32_t* sig[kPeerMaxRanks];   // every rank's flag array
  uint32_t* epoch;                // per-block call counter (local)
  int* err;                       // host-mapped error word
  void* data;                     // bucket (in place)
  long long count;                // elements
  long long slot_bytes;           // bytes of one slot (region = W slots; 2 regions x 2 parities)
  long long timeout;              // s_memrealtime ticks (100 MHz)
  float scale;                    // applied to the sum (1 = sum, 1/ws = average)
  int rank, ws;
  int fence;                      // bit 0: system release before flag stores; bit 1: acquire after waits;
                                  // bit 2: withhold this rank's flags (PeerComm::set_withhold, tests)
};

// host-side partition shared by the kernel and the tests: chunk (elements) per rank and
// slice (elements) per block, both multiples of the 16-byte vector width `vec`
struct PeerPartition {
  long long chunk, slice;
  static PeerPartition make(long long count, int ws, int blocks, int vec);
};

class PeerComm {
 public:
  // cap_bytes: largest bucket one launch handles (bigger ones are split); blocks: workgroups
  // per launch (and flag sets)
  PeerComm(int rank, int world_size, int device, size_t cap_bytes, int blocks);
  ~PeerComm();
  PeerComm(const PeerComm&) = delete;
  PeerComm& operator=(const PeerComm&) = delete;

  std::string handles() const;                       // this rank's IPC handles (opaque bytes)
  void open(const std::vector<std::string>& all);    // every rank's handles, rank order
  // in-process replicas (one PeerComm per device, one process): map the other ranks' buffers
  // directly (device peer access instead of IPC); `all` in rank order
  void open_local(const std::vector<PeerComm*>& all);
  // in-place all-reduce of `count` elements (f32 or bf16) on `st`: sum, or average
  // (RedOp::kAvg, the sum times 1/world_size); graph-capturable
  void all_reduce(void* data, size_t count, DType t, hipStream_t st, RedOp op = RedOp::kSum);
  // kernel arguments of ONE two-shot f32 exchange of `count` elements run by blocks() blocks of
  // another kernel (peer_device.h: peer_two_shot_f32_block); false if it does not fit one
  // launch (bucket above the exchange capacity) or world size 1
  bool coschedule_args(void* data, size_t count, RedOp op, PeerArgs* a, PeerPartition* part) const;
  // kernel arguments of ONE one-shot f32 exchange of `count` elements (every rank's whole bucket
  // in each peer's slot) run by another kernel's blocks; false if it does not fit one slot
  bool oneshot_args(void* data, size_t count, RedOp op, PeerArgs* a) const;
  int error() const;                                 // 0 = ok; else 1 + (peer that timed out)
  void reset_error();
  void set_blocks(int b);
  void set_fence(int f) { fence_ = f & 3; }
  // tests only: this rank stops publishing its flags (a peer that never arrives), so the
  // fail-fast / autotune-drop paths can be exercised on one box.  mask bit 0: the standalone
  // all-reduce kernels; bit 1: exchanges co-scheduled inside another kernel (coschedule_args /
  // oneshot_args, taken when that kernel's launch or graph is built)
  void set_withhold(int mask) { withhold_ = mask; }
  // every rank, device idle and host-synchronised with its peers (parallel/peer.py: resync):
  // zero this rank's flags, per-block epochs and error word, so the next exchange starts a
  // fresh epoch sequence on every rank -- after a timed-out exchange left the ranks' epochs
  // apart, or before another kernel family with its own block partition takes the buffers
  void reset_state();
  void set_timeout_ms(double ms) { timeout_ = static_cast<long long>(ms * 1e5); }
  // buckets up to this size take the one-shot kernel (every rank must use the same value)
  void set_oneshot_bytes(long long b) { oneshot_bytes_ = b; }
  long long oneshot_bytes() const { return oneshot_bytes_; }
  int blocks() const { return blocks_; }
  int fence() const { return fence_; }
  int rank() const { return rank_; }
  int world_size() const { return ws_; }
  bool opened() const { return opened_; }
  const std::string& mem_kind() const { return mem_kind_; }
  size_t cap_bytes() const { return cap_; }

 private:
  int rank_, ws_, dev_, blocks_;
  size_t cap_, slot_bytes_, xbytes_, sbytes_;
  char* xbuf_ = nullptr;
  uint32_t* sig_ = nullptr;
  uint32_t* epoch_ = nullptr;
  int* err_host_ = nullptr;
  int* err_dev_ = nullptr;
  char* peer_x_[kPeerMaxRanks] = {};
  uint32_t* peer_sig_[kPeerMaxRanks] = {};
  bool opened_ = false, local_ = false;
  int fence_ = 1;
  int withhold_ = 0;
  long long timeout_ = 3000000000ll;  // 30 s
  long long oneshot_bytes_ = 256 << 10;
  std::string mem_kind_;
};

// buckets of at most `oneshot_bytes` use the one-shot kernel (one flag round), larger ones the
// two-shot kernel
void peer_all_reduce_launch(const PeerArgs& a, DType t, int blocks, hipStream_t st, long long oneshot_bytes);

}  // namespace mx
