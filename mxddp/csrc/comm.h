// RCCL communicator owned by mxddp (one per process and device; or one per device
// for the in-process replica engine).  The ncclUniqueId is exchanged through the
// torch.distributed TCPStore by the Python layer (mxddp/parallel/comm.py), mirroring
// the reference's `dist.init_process_group(nccl, tcp://...)` rendezvous
// (pytorch/distributed_data_parallel.py:61-62) but giving us our own communicator
// and HIP streams, so collectives can be issued from C++ and captured in hipGraphs.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <string>
#include <vector>

namespace mx {

enum class DType : int { kF32 = 0, kBF16 = 1, kF16 = 2, kI32 = 3, kI64 = 4, kU8 = 5 };
enum class RedOp : int { kSum = 0, kAvg = 1, kMax = 2, kMin = 3, kProd = 4 };

ncclDataType_t to_nccl(DType t);
ncclRedOp_t to_nccl(RedOp o);
size_t dtype_size(DType t);

// How a communicator is built for the 8x MI355X xGMI mesh (every GPU: 7 point-to-point links).
// `ctas` pins RCCL's channel count (ncclConfig_t minCTAs = maxCTAs; each channel is one ring
// permutation over the mesh, so 7 / 14 / 28 channels put 1 / 2 / 4 rings on every link);
// `algo` / `proto` pin NCCL_ALGO / NCCL_PROTO for this communicator only (read by RCCL's tuner
// at init; restored afterwards).  Defaults (0 / "") leave RCCL's own tuning.
struct CommConfig {
  int ctas = 0;
  std::string algo, proto;
  std::string name() const;
};

class Comm {
 public:
  Comm(const std::string& unique_id, int rank, int world_size, int device, const CommConfig& cfg = CommConfig());
  explicit Comm(ncclComm_t c, int rank, int world_size, int device);  // adopt (replica engine)
  ~Comm();
  Comm(const Comm&) = delete;
  Comm& operator=(const Comm&) = delete;

  static std::string new_unique_id();
  // RCCL's version code (ncclGetVersion: major * 10000 + minor * 100 + patch)
  static int version();
  // Deadline of every communicator init (ncclCommInitRank / InitRankConfig / InitAll), seconds
  // (<= 0: none).  Default: MXDDP_RCCL_INIT_TIMEOUT_S, else 120.  An init that has not returned
  // by then -- a rank that never joined, a wedged bootstrap -- prints the rank, world size,
  // device and variant on stderr and ends the process with kInitTimeoutExit: the init is
  // blocking (the mode every later collective and graph capture relies on), so there is no
  // communicator handle to abort yet; ending the process is what releases the GPU and the
  // other ranks' rendezvous.
  static void set_init_timeout(double seconds);
  static double init_timeout();
  static constexpr int kInitTimeoutExit = 75;
  // ncclCommInitAll over `devices` in one process (replica / MirroredStrategy mode)
  static std::vector<Comm*> init_all(const std::vector<int>& devices);

  void all_reduce(const void* send, void* recv, size_t count, DType t, RedOp op, hipStream_t st);
  void broadcast(const void* send, void* recv, size_t count, DType t, int root, hipStream_t st);
  void reduce_scatter(const void* send, void* recv, size_t recv_count, DType t, RedOp op, hipStream_t st);
  void all_gather(const void* send, void* recv, size_t send_count, DType t, hipStream_t st);
  void all_to_all(const void* send, void* recv, size_t count_per_peer, DType t, hipStream_t st);
  void send(const void* buf, size_t count, DType t, int peer, hipStream_t st);
  void recv(void* buf, size_t count, DType t, int peer, hipStream_t st);
  // Raise if RCCL reported an asynchronous error (failure detection at step boundaries).
  void check_async_error() const;
  void abort();

  static void group_start();
  static void group_end();

  // what RCCL itself says about the communicator (ncclCommCount / ncclCommCuDevice)
  int nranks() const;
  int hip_device() const;

  int rank() const { return rank_; }
  int world_size() const { return ws_; }
  int device() const { return device_; }
  const CommConfig& config() const { return cfg_; }
  ncclComm_t raw() const { return comm_; }

 private:
  ncclComm_t comm_ = nullptr;
  int rank_ = 0, ws_ = 1, device_ = 0;
  bool aborted_ = false;
  CommConfig cfg_;
};

}  // namespace mx
