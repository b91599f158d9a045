// Device-side pieces of the peer all-reduce (design: peer.h) shared by the standalone kernels
// (peer_kernels.hip) and by kernels that run the exchange in some of their own blocks -- the
// fused MNIST conv-backward launch co-schedules the fc-bucket exchange with the conv work
// (mnist_conv_bwd.hip), so the all-reduce overlaps the backward without a second stream.
#pragma once
#include "common.h"
#include "peer.h"

namespace mx {

constexpr int kPeerThreads = 256;

__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ uint32_t* flag_at(uint32_t* sig, int set, int b, int p) {
  return sig + ((size_t)set * kPeerMaxBlocks + b) * kPeerMaxRanks + p;
}

// lanes 0..ws-1 (except `rank`) of wave 0 each wait for one peer's flag; bounded.  Fail fast:
// once the error word is set (a peer timed out in this or an earlier launch) no lane waits
// again -- the bucket is garbage either way and the host raises at its next check -- so a
// broken transport costs ONE timeout, not one per block per later launch.
__device__ __forceinline__ void wait_peers(const PeerArgs& a, int set, int b, uint32_t ep) {
  const int t = threadIdx.x;
  if (t < a.ws && t != a.rank && __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0) {
    uint32_t* f = flag_at(a.sig[a.rank], set, b, t);
    const long long t0 = wall_clock64();
    unsigned spins = 0;
    while (static_cast<int32_t>(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - ep) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if (wall_clock64() - t0 > a.timeout) {
        __hip_atomic_store(a.err, 1 + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      // another block / lane already timed out: stop waiting (host-mapped word, polled rarely)
      if ((++spins & 255u) == 0 && __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) break;
    }
  }
  if ((a.fence & 2) && t < kWave) {  // acquire (only needed when the exchange memory is cached)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    vm_drain();
  }
  __syncthreads();
}

// every wave's stores drained, then one lane per peer publishes `ep` in that peer's flag
__device__ __forceinline__ void signal_peers(const PeerArgs& a, int set, int b, uint32_t ep) {
  vm_drain();
  __syncthreads();
  const int t = threadIdx.x;
  if (t < kWave) {
    if (a.fence & 1) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      vm_drain();
    }
    // fence bit 2 (PeerComm::set_withhold, tests only): this rank never publishes its flags,
    // i.e. it behaves like a peer that stopped arriving
    if (t < a.ws && t != a.rank && !(a.fence & 4))
      __hip_atomic_store(flag_at(a.sig[t], set, b, a.rank), ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}


// One block's share (slice b) of the two-shot float all-reduce, world size at run time (the
// standalone kernel's per-W template, for a caller that cannot be instantiated per W).  Same
// slots, flags, epochs and partition as peer_all_reduce_kernel<float, W> with the same block
// count, so the two can alternate call by call.  `s_ep` is one word of the caller's LDS (a
// static __shared__ here would add to the host kernel's static LDS and make its 160 KB dynamic
// allocation fail).
__device__ __forceinline__ void peer_two_shot_f32_block(const PeerArgs& a, const PeerPartition& part, int b,
                                                        uint32_t* s_ep) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const int r = a.rank, t = threadIdx.x, W = a.ws;
  if (t == 0) *s_ep = a.epoch[b] + 1;
  __syncthreads();
  const uint32_t ep = *s_ep;
  float* data = static_cast<float*>(a.data);
  const long long c = part.chunk, lo = (long long)b * part.slice;
  const long long slot = a.slot_bytes / 4;
  const long long half = (long long)(ep & 1u) * 2 * W * slot;
  const long long hi = lo + part.slice < c ? lo + part.slice : c;
  // 1. scatter: my chunk p (slice b) -> rank p's scatter slot r, for every peer p
  for (int j = 1; j < W; ++j) {
    const int p = (r + j) % W;
    const long long np = a.count - (long long)p * c;
    const long long e = (np < hi ? np : hi) - lo;
    const long long n = e > 0 ? e : 0;
    const float* src = data + (long long)p * c + lo;
    float* dst = reinterpret_cast<float*>(a.xbuf[p]) + half + (long long)r * slot + lo;
    for (long long i = t; i < n / 4; i += kPeerThreads)
      reinterpret_cast<v4u*>(dst)[i] = reinterpret_cast<const v4u*>(src)[i];
    for (long long i = n / 4 * 4 + t; i < n; i += kPeerThreads) dst[i] = src[i];
  }
  signal_peers(a, 0, b, ep);
  wait_peers(a, 0, b, ep);
  // 2. reduce my chunk r (slice b) over the ranks in order 0..W-1, push it to every gather slot r
  {
    const long long np = a.count - (long long)r * c;
    const long long e = (np < hi ? np : hi) - lo;
    const long long nr = e > 0 ? e : 0;
    float* mine = data + (long long)r * c + lo;
    const float* scat = reinterpret_cast<const float*>(a.xbuf[r]) + half + lo;
    for (long long i = t; i < nr; i += kPeerThreads) {
      float acc = 0.f;
      for (int p = 0; p < W; ++p) {
        const float v = p == r ? mine[i] : __builtin_nontemporal_load(scat + (long long)p * slot + i);
        acc = p == 0 ? v : acc + v;
      }
      if (a.scale != 1.f) acc *= a.scale;
      mine[i] = acc;
      for (int j = 1; j < W; ++j) {
        const int p = (r + j) % W;
        (reinterpret_cast<float*>(a.xbuf[p]) + half + (long long)(W + r) * slot + lo)[i] = acc;
      }
    }
  }
  signal_peers(a, 1, b, ep);
  wait_peers(a, 1, b, ep);
  // 3. gather the other ranks' reduced chunks from my gather slots
  for (int j = 1; j < W; ++j) {
    const int p = (r + j) % W;
    const long long np = a.count - (long long)p * c;
    const long long e = (np < hi ? np : hi) - lo;
    const long long n = e > 0 ? e : 0;
    float* out = data + (long long)p * c + lo;
    const float* gat = reinterpret_cast<const float*>(a.xbuf[r]) + half + (long long)(W + p) * slot + lo;
    for (long long i = t; i < n / 4; i += kPeerThreads)
      reinterpret_cast<v4u*>(out)[i] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(gat) + i);
    for (long long i = n / 4 * 4 + t; i < n; i += kPeerThreads) out[i] = __builtin_nontemporal_load(gat + i);
  }
  if (t == 0) a.epoch[b] = ep;
}

}  // namespace mx
