// Two-shot peer all-reduce kernel (design: peer.h).
//
// One workgroup = 256 threads = 4 waves; block b owns slice b of every rank's chunk, so the
// only synchronisation is between block b of this rank and block b of each peer:
//
//   flag set 0 (scatter done)  sig[0][b][p] on rank q == "rank p stored its chunk q slice b
//                               into q's scatter slot p"
//   flag set 1 (reduce done)   sig[1][b][p] on rank q == "rank p stored reduced chunk p
//                               slice b into q's gather slot p"
//
// Flags carry a per-block call counter (epoch), so they never need resetting and graph
// replays work with fixed kernel arguments.  Exchange slots are double-buffered by call
// parity: consecutive calls may have different bucket sizes, hence a different block ->
// region mapping, so block b of rank p in call k+1 may write bytes that ANOTHER block of rank
// q still reads in call k.  Call k+1 therefore uses the other half, which q last read in call
// k-1 -- and that call has fully completed on q, since q's block b reached call k (stream
// order) before it released p's block b into call k+1 (flag set 1 of call k).
#include "common.h"
#include "peer.h"
#include "peer_device.h"

namespace mx {

namespace {

constexpr int kThreads = kPeerThreads;

// 16-byte register vector (a native vector type: HIP's uint4 is a union-based struct that
// keeps arrays of it out of registers)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// elements of T per 16-byte vector
template <class T>
struct Vec {
  static constexpr int N = 16 / sizeof(T);
};

__device__ __forceinline__ float bf16_to_f(uint32_t h) { return __uint_as_float(h << 16); }
__device__ __forceinline__ uint32_t f_to_bf16(float f) {  // round to nearest even
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u) return (u >> 16) | ((u & 0xffffu) ? 0x40u : 0u);  // inf / nan
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

// accumulate a 16-byte vector into 8 (bf16) or 4 (f32) float lanes
template <class T>
__device__ __forceinline__ void acc16(float* a, u32x4 v, bool first) {
  const uint32_t w[4] = {v[0], v[1], v[2], v[3]};
  if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = first ? __uint_as_float(w[i]) : a[i] + __uint_as_float(w[i]);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float lo = bf16_to_f(w[i] & 0xffffu), hi = bf16_to_f(w[i] >> 16);
      a[2 * i] = first ? lo : a[2 * i] + lo;
      a[2 * i + 1] = first ? hi : a[2 * i + 1] + hi;
    }
  }
}

template <class T>
__device__ __forceinline__ u32x4 pack16(const float* a) {
  u32x4 v;
  if constexpr (sizeof(T) == 4) {
    v = u32x4{__float_as_uint(a[0]), __float_as_uint(a[1]), __float_as_uint(a[2]), __float_as_uint(a[3])};
  } else {
    v = u32x4{f_to_bf16(a[0]) | (f_to_bf16(a[1]) << 16), f_to_bf16(a[2]) | (f_to_bf16(a[3]) << 16),
              f_to_bf16(a[4]) | (f_to_bf16(a[5]) << 16), f_to_bf16(a[6]) | (f_to_bf16(a[7]) << 16)};
  }
  return v;
}

template <class T>
__device__ __forceinline__ float ld_elem(const T* p, bool nt) {
  if constexpr (sizeof(T) == 4) {
    const uint32_t u = nt ? __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(p))
                          : *reinterpret_cast<const uint32_t*>(p);
    return __uint_as_float(u);
  } else {
    const uint16_t u = nt ? __builtin_nontemporal_load(reinterpret_cast<const uint16_t*>(p))
                          : *reinterpret_cast<const uint16_t*>(p);
    return bf16_to_f(u);
  }
}
template <class T>
__device__ __forceinline__ void st_elem(T* p, float f) {
  if constexpr (sizeof(T) == 4) *reinterpret_cast<float*>(p) = f;
  else *reinterpret_cast<uint16_t*>(p) = static_cast<uint16_t>(f_to_bf16(f));
}

template <class T, int W>
__global__ __launch_bounds__(kThreads) void peer_all_reduce_kernel(PeerArgs a, PeerPartition part) {
  constexpr int V = Vec<T>::N;
  const int b = blockIdx.x, r = a.rank, t = threadIdx.x;
  __shared__ uint32_t s_ep;
  if (t == 0) s_ep = a.epoch[b] + 1;
  __syncthreads();
  const uint32_t ep = s_ep;
  T* data = static_cast<T*>(a.data);
  const long long c = part.chunk, lo = (long long)b * part.slice;
  const long long slot = a.slot_bytes / (long long)sizeof(T);  // elements per slot
  const long long half = (long long)(ep & 1u) * 2 * W * slot;    // this call's buffer half
  const long long hi = lo + part.slice < c ? lo + part.slice : c;
  // per peer j = 1..W-1 (rank p = (r + j) % W, rotated so the W-1 links start on different
  // peers): elements of chunk p this block owns, and the pointers it touches (SGPRs)
  long long n[W];
  const T* src[W];   // phase 1: my chunk p         | phase 3: my gather slot p
  T* dst[W];         // phase 1: rank p's scatter slot r | phase 2: rank p's gather slot r
  const T* gat[W];
#pragma unroll
  for (int j = 0; j < W; ++j) {
    const int p = (r + j) % W;
    const long long np = a.count - (long long)p * c;
    const long long e = (np < hi ? np : hi) - lo;
    n[j] = e > 0 ? e : 0;
    src[j] = data + (long long)p * c + lo;
    dst[j] = reinterpret_cast<T*>(a.xbuf[p]) + half + (long long)r * slot + lo;
    gat[j] = reinterpret_cast<const T*>(a.xbuf[r]) + half + (long long)(W + p) * slot + lo;
  }
  // vectors every peer's chunk has (all but the last chunk are full): unconditional, unrolled
  long long nvmin = n[1] / V;
#pragma unroll
  for (int j = 2; j < W; ++j) nvmin = n[j] / V < nvmin ? n[j] / V : nvmin;

  // 1. scatter: chunk p slice b -> rank p's scatter slot r, all W-1 links at once (every
  //    thread has one 16-byte load per peer in flight before it stores)
  for (long long i = t; i < nvmin; i += kThreads) {
    u32x4 v[W - 1];
#pragma unroll
    for (int j = 1; j < W; ++j) v[j - 1] = reinterpret_cast<const u32x4*>(src[j])[i];
#pragma unroll
    for (int j = 1; j < W; ++j) reinterpret_cast<u32x4*>(dst[j])[i] = v[j - 1];
  }
#pragma unroll
  for (int j = 1; j < W; ++j) {  // the short (last) chunk's remainder
    for (long long i = nvmin + t; i < n[j] / V; i += kThreads)
      reinterpret_cast<u32x4*>(dst[j])[i] = reinterpret_cast<const u32x4*>(src[j])[i];
    for (long long i = n[j] / V * V + t; i < n[j]; i += kThreads) dst[j][i] = src[j][i];
  }
  signal_peers(a, 0, b, ep);
  wait_peers(a, 0, b, ep);

  // 2. reduce chunk r slice b over all ranks in rank order 0..W-1 (identical on every rank),
  //    write it back and push it into every peer's gather slot r
  {
    const long long nr = n[0];
    T* mine = data + (long long)r * c + lo;
    const T* scat = reinterpret_cast<const T*>(a.xbuf[r]) + half + lo;
    for (long long i = t; i < nr / V; i += kThreads) {
      u32x4 v[W];
#pragma unroll
      for (int p = 0; p < W; ++p)
        v[p] = p == r ? reinterpret_cast<const u32x4*>(mine)[i]
                      : __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(scat + (long long)p * slot) + i);
      float acc[V];
#pragma unroll
      for (int p = 0; p < W; ++p) acc16<T>(acc, v[p], p == 0);
      if (a.scale != 1.f) {
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] *= a.scale;
      }
      const u32x4 out = pack16<T>(acc);
      reinterpret_cast<u32x4*>(mine)[i] = out;
#pragma unroll
      for (int j = 1; j < W; ++j)
        reinterpret_cast<u32x4*>(dst[j] + (long long)W * slot)[i] = out;  // gather slot r of rank p
    }
    for (long long i = nr / V * V + t; i < nr; i += kThreads) {
      float acc = 0.f;
#pragma unroll
      for (int p = 0; p < W; ++p) {
        const float v = p == r ? ld_elem<T>(mine + i, false) : ld_elem<T>(scat + (long long)p * slot + i, true);
        acc = p == 0 ? v : acc + v;
      }
      if (a.scale != 1.f) acc *= a.scale;
      st_elem<T>(mine + i, acc);
      const T rounded = mine[i];
#pragma unroll
      for (int j = 1; j < W; ++j) (dst[j] + (long long)W * slot)[i] = rounded;
    }
  }
  signal_peers(a, 1, b, ep);
  wait_peers(a, 1, b, ep);

  // 3. gather: reduced chunk p slice b from gather slot p
  for (long long i = t; i < nvmin; i += kThreads) {
    u32x4 v[W - 1];
#pragma unroll
    for (int j = 1; j < W; ++j) v[j - 1] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(gat[j]) + i);
#pragma unroll
    for (int j = 1; j < W; ++j) reinterpret_cast<u32x4*>(const_cast<T*>(src[j]))[i] = v[j - 1];
  }
#pragma unroll
  for (int j = 1; j < W; ++j) {
    T* out = const_cast<T*>(src[j]);
    for (long long i = nvmin + t; i < n[j] / V; i += kThreads)
      reinterpret_cast<u32x4*>(out)[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(gat[j]) + i);
    for (long long i = n[j] / V * V + t; i < n[j]; i += kThreads) out[i] = __builtin_nontemporal_load(gat[j] + i);
  }
  if (t == 0) a.epoch[b] = ep;
}

// One-shot variant for small buckets (the MNIST conv bucket is 75 KB): every rank pushes its
// WHOLE slice b to every peer's scatter slot r, ONE flag round, then each rank sums all W slots
// in rank order locally -- the same operands in the same order everywhere, so every rank ends
// with identical values.  Each link carries S bytes instead of 2 S / W, but one synchronisation
// round is saved, which is what a small all-reduce costs.  Same slots / flags / parity as the
// two-shot kernel (only flag set 0), so the two may alternate freely call by call.
template <class T, int W>
__global__ __launch_bounds__(kThreads) void peer_all_reduce_oneshot_kernel(PeerArgs a, long long slice) {
  constexpr int V = Vec<T>::N;
  const int b = blockIdx.x, r = a.rank, t = threadIdx.x;
  __shared__ uint32_t s_ep;
  if (t == 0) s_ep = a.epoch[b] + 1;
  __syncthreads();
  const uint32_t ep = s_ep;
  const long long slot = a.slot_bytes / (long long)sizeof(T);
  const long long half = (long long)(ep & 1u) * 2 * W * slot;
  const long long lo = (long long)b * slice;
  const long long rem = a.count - lo;
  const long long n = rem < 0 ? 0 : (rem < slice ? rem : slice);
  T* mine = static_cast<T*>(a.data) + lo;
  T* dst[W];
#pragma unroll
  for (int j = 1; j < W; ++j) dst[j] = reinterpret_cast<T*>(a.xbuf[(r + j) % W]) + half + (long long)r * slot + lo;
  // 1. push: one load, W-1 remote stores per 16-byte vector
  for (long long i = t; i < n / V; i += kThreads) {
    const u32x4 v = reinterpret_cast<const u32x4*>(mine)[i];
#pragma unroll
    for (int j = 1; j < W; ++j) reinterpret_cast<u32x4*>(dst[j])[i] = v;
  }
  for (long long i = n / V * V + t; i < n; i += kThreads) {
    const T v = mine[i];
#pragma unroll
    for (int j = 1; j < W; ++j) dst[j][i] = v;
  }
  signal_peers(a, 0, b, ep);
  wait_peers(a, 0, b, ep);
  // 2. sum the W contributions in rank order 0..W-1
  const T* scat = reinterpret_cast<const T*>(a.xbuf[r]) + half + lo;
  for (long long i = t; i < n / V; i += kThreads) {
    u32x4 v[W];
#pragma unroll
    for (int p = 0; p < W; ++p)
      v[p] = p == r ? reinterpret_cast<const u32x4*>(mine)[i]
                    : __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(scat + (long long)p * slot) + i);
    float acc[V];
#pragma unroll
    for (int p = 0; p < W; ++p) acc16<T>(acc, v[p], p == 0);
    if (a.scale != 1.f) {
#pragma unroll
      for (int e = 0; e < V; ++e) acc[e] *= a.scale;
    }
    reinterpret_cast<u32x4*>(mine)[i] = pack16<T>(acc);
  }
  for (long long i = n / V * V + t; i < n; i += kThreads) {
    float acc = 0.f;
#pragma unroll
    for (int p = 0; p < W; ++p) {
      const float v = p == r ? ld_elem<T>(mine + i, false) : ld_elem<T>(scat + (long long)p * slot + i, true);
      acc = p == 0 ? v : acc + v;
    }
    if (a.scale != 1.f) acc *= a.scale;
    st_elem<T>(mine + i, acc);
  }
  if (t == 0) a.epoch[b] = ep;
}

}  // namespace

PeerPartition PeerPartition::make(long long count, int ws, int blocks, int vec) {
  PeerPartition p;
  p.chunk = ((count + ws - 1) / ws + vec - 1) / vec * vec;
  p.slice = ((p.chunk + blocks - 1) / blocks + vec - 1) / vec * vec;
  return p;
}

void peer_all_reduce_launch(const PeerArgs& a, DType t, int blocks, hipStream_t st, long long oneshot_bytes) {
  const int esz = static_cast<int>(dtype_size(t));
  const int vec = 16 / esz;
  const PeerPartition part = PeerPartition::make(a.count, a.ws, blocks, vec);
  MX_CHECK(part.chunk * esz <= a.slot_bytes, "peer all-reduce: bucket larger than the exchange slot");
  MX_CHECK(reinterpret_cast<uintptr_t>(a.data) % 16 == 0, "peer all-reduce: data must be 16-byte aligned");
  MX_CHECK(t == DType::kF32 || t == DType::kBF16, "peer all-reduce: f32 or bf16 only");
  const bool f = t == DType::kF32;
  // every rank makes the same choice (a function of the count only)
  const bool one = a.count * esz <= oneshot_bytes && a.count * esz <= a.slot_bytes;
  const long long slice = ((a.count + blocks - 1) / blocks + vec - 1) / vec * vec;
#define MX_PEER_CASE(NW)                                                                                    \
  case NW:                                                                                                  \
    if (one && f) MX_LAUNCH((peer_all_reduce_oneshot_kernel<float, NW>), dim3(blocks), dim3(kThreads), 0, st, a, slice); \
    else if (one) MX_LAUNCH((peer_all_reduce_oneshot_kernel<uint16_t, NW>), dim3(blocks), dim3(kThreads), 0, st, a, slice); \
    else if (f) MX_LAUNCH((peer_all_reduce_kernel<float, NW>), dim3(blocks), dim3(kThreads), 0, st, a, part); \
    else MX_LAUNCH((peer_all_reduce_kernel<uint16_t, NW>), dim3(blocks), dim3(kThreads), 0, st, a, part);    \
    break;
  switch (a.ws) {
    MX_PEER_CASE(2)
    MX_PEER_CASE(3)
    MX_PEER_CASE(4)
    MX_PEER_CASE(5)
    MX_PEER_CASE(6)
    MX_PEER_CASE(7)
    MX_PEER_CASE(8)
    default: throw std::runtime_error("peer all-reduce: 2..8 ranks");
  }
#undef MX_PEER_CASE
}

}  // namespace mx
