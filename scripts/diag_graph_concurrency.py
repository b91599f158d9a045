"""Do parallel branches of a captured hipGraph run concurrently on this ROCm?  Two 1-block spin
kernels (torch.cuda._sleep) captured on forked streams vs in sequence; prints both replay times."""
import time

import torch

cyc = 2_000_000  # ~1 ms at ~2 GHz
torch.cuda._sleep(1000)
torch.cuda.synchronize()


def timed(g, n=5):
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


main = torch.cuda.Stream()
side = torch.cuda.Stream()
g_seq = torch.cuda.CUDAGraph()
with torch.cuda.graph(g_seq, stream=main):
    torch.cuda._sleep(cyc)
    torch.cuda._sleep(cyc)
g_par = torch.cuda.CUDAGraph()
with torch.cuda.graph(g_par, stream=main):
    side.wait_stream(main)
    torch.cuda._sleep(cyc)
    with torch.cuda.stream(side):
        torch.cuda._sleep(cyc)
    main.wait_stream(side)
one = torch.cuda.CUDAGraph()
with torch.cuda.graph(one, stream=main):
    torch.cuda._sleep(cyc)
print({"one_ms": round(timed(one), 3), "sequential_ms": round(timed(g_seq), 3), "parallel_ms": round(timed(g_par), 3)})
# eager two streams for comparison
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    side.wait_stream(main)
    with torch.cuda.stream(main):
        torch.cuda._sleep(cyc)
    with torch.cuda.stream(side):
        torch.cuda._sleep(cyc)
    main.wait_stream(side)
torch.cuda.synchronize()
print({"eager_two_streams_ms": round((time.perf_counter() - t0) / 5 * 1e3, 3)})
