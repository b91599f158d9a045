// Grid-barrier cost on MI355X: flat counter vs per-XCD hierarchical counters, for a range of
// grid sizes.  Every spin is bounded (sets an error flag instead of hanging).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

struct Bar { unsigned count, gen, err, pad; unsigned xc[8][16]; };
__device__ Bar g_bar;

// MODE 0/1: release/acquire fences at agent scope (L2 write-back + invalidate per wave);
// MODE 2/3: data exchanged with sc1 (device-coherent) stores/loads, so the barrier only waits
// for this wave's stores to be acknowledged (s_waitcnt vmcnt(0)); 1/3 use per-XCD counters.
template <int MODE>
__device__ __forceinline__ void gsync(int sleep) {
  if (MODE < 2) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned gen = __hip_atomic_load(&g_bar.gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    bool last;
    if ((MODE & 1) == 0) {
      last = __hip_atomic_fetch_add(&g_bar.count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    } else {
      // per-XCD group: blocks b with b % 8 == x (dispatch round-robins XCDs)
      const unsigned x = blockIdx.x & 7, n = (gridDim.x - x + 7) / 8;
      last = false;
      if (__hip_atomic_fetch_add(&g_bar.xc[x][0], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == n - 1) {
        __hip_atomic_store(&g_bar.xc[x][0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned groups = gridDim.x < 8 ? gridDim.x : 8;
        last = __hip_atomic_fetch_add(&g_bar.count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == groups - 1;
      }
    }
    if (last) {
      __hip_atomic_store(&g_bar.count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&g_bar.gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      unsigned spins = 0;
      while (__hip_atomic_load(&g_bar.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen) {
        if (sleep) __builtin_amdgcn_s_sleep(1);
        if (++spins == (1u << 22)) { __hip_atomic_fetch_or(&g_bar.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); break; }
      }
    }
    if (MODE < 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

__device__ unsigned g_slot[4096];

template <int MODE>
__global__ void k(int iters, int sleep, float* sink) {
  float acc = 0.f;
  for (int i = 0; i < iters; ++i) {
    // exchange: block b publishes (i, b), reads its neighbour's after the barrier
    if (threadIdx.x == 0) __hip_atomic_store(&g_slot[blockIdx.x], (unsigned)(i * 4096 + blockIdx.x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    gsync<MODE>(sleep);
    if (threadIdx.x == 0) {
      const unsigned nb = (blockIdx.x + 1) % gridDim.x;
      const unsigned got = __hip_atomic_load(&g_slot[nb], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (got != (unsigned)(i * 4096) + nb) __hip_atomic_fetch_or(&g_bar.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    gsync<MODE>(sleep);  // nobody overwrites a slot before its reader has read it
    acc += 1.f;
  }
  if (threadIdx.x == 0) sink[blockIdx.x] = acc;
}

int main() {
  hipDeviceProp_t prop; hipGetDeviceProperties(&prop, 0); printf("CUs %d\n", prop.multiProcessorCount);
  float* sink; hipMalloc(&sink, 4096 * 4);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const int grids[] = {8, 64, 128, 256, 512};
  for (int mode = 0; mode < 4; ++mode)
    for (int sl = 0; sl < 1; ++sl)
      for (int g : grids) for (int bt : {256, 1024}) {
        if (bt == 1024 && g > 256) continue;
        const int iters = 200;
        auto launch = [&](int it) {
          if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(g), dim3(bt), 0, 0, it, sl, sink);
          else if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(g), dim3(bt), 0, 0, it, sl, sink);
          else if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(g), dim3(bt), 0, 0, it, sl, sink);
          else hipLaunchKernelGGL(k<3>, dim3(g), dim3(bt), 0, 0, it, sl, sink);
        };
        launch(2); hipDeviceSynchronize();
        hipEventRecord(a); launch(iters); hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        Bar h; hipMemcpyFromSymbol(&h, HIP_SYMBOL(g_bar), sizeof(h));
        printf("mode=%s %s sleep=%d grid=%4d block=%4d  %.2f us/barrier  err=%u\n", (mode & 1) ? "xcd " : "flat", mode >= 2 ? "sc1" : "fence", sl, g, bt,
               ms * 1000.f / (2 * iters), h.err);
        if (h.err) return 1;
      }
  // empty-kernel launch cost for reference
  hipEventRecord(a);
  for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(k<0>, dim3(512), dim3(256), 0, 0, 0, 0, sink);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  printf("back-to-back empty launches: %.2f us each\n", ms * 1000.f / 200);
  return 0;
}
