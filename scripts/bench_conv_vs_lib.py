"""Library yardsticks for every distinct ResNet-50 conv shape: stock PyTorch-ROCm
(``F.conv2d`` channels_last bf16 = MIOpen) forward / data gradient / weight gradient, and for the
1x1 stride-1 layers the same three directions as plain ``torch.mm`` GEMMs (hipBLASLt).  Printed
next to ``scripts/bench_nhwc_layers.py``'s numbers for mxddp's own kernels, run in the same call,
it says per layer whether a library path would beat the hand-written kernel.

    python scripts/bench_conv_vs_lib.py [batch] [iters]
"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench_nhwc_layers import shapes  # noqa: E402


def _time(fn, iters):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def main():
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda")
    bf = torch.bfloat16
    print(f"{'count':>5} {'N':>3} {'H':>4} {'C':>5} {'K':>5} {'R':>2} {'s':>2} | "
          f"{'miopen fwd':>10} {'dgrad':>7} {'wgrad':>7} | {'blas fwd':>8} {'TF':>5} {'dgrad':>7} {'wgrad':>7}")
    tot = {"mf": 0.0, "md": 0.0, "mw": 0.0}
    for cnt, N, H, W, C, K, R, s, p in shapes(batch):
        P, Q = (H + 2 * p - R) // s + 1, (W + 2 * p - R) // s + 1
        flops = 2.0 * N * P * Q * K * C * R * R
        x = torch.randn(N, C, H, W, device=dev, dtype=bf).to(memory_format=torch.channels_last)
        w = (torch.randn(K, C, R, R, device=dev) * 0.05).to(bf).to(memory_format=torch.channels_last)
        dy = torch.randn(N, K, P, Q, device=dev, dtype=bf).to(memory_format=torch.channels_last)
        mf = _time(lambda: F.conv2d(x, w, stride=s, padding=p), iters)
        md = _time(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, (s, s), (p, p), (1, 1), False, (0, 0), 1,
                                                               (True, False, False)), iters)
        mw = _time(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, (s, s), (p, p), (1, 1), False, (0, 0), 1,
                                                               (False, True, False)), iters)
        tot["mf"] += cnt * mf
        tot["md"] += cnt * md
        tot["mw"] += cnt * mw
        line = (f"{cnt:>5} {N:>3} {H:>4} {C:>5} {K:>5} {R:>2} {s:>2} | {mf:>10.1f} {md:>7.1f} {mw:>7.1f} |")
        if R == 1 and s == 1:
            M = N * P * Q
            a = torch.randn(M, C, device=dev, dtype=bf)
            bt = torch.randn(C, K, device=dev, dtype=bf)
            g = torch.randn(M, K, device=dev, dtype=bf)
            bf_ = _time(lambda: torch.mm(a, bt), iters)
            bd = _time(lambda: torch.mm(g, bt.t()), iters)
            bw = _time(lambda: torch.mm(g.t(), a), iters)
            line += f" {bf_:>8.1f} {flops / bf_ / 1e6:>5.0f} {bd:>7.1f} {bw:>7.1f}"
        print(line, flush=True)
        del x, w, dy
    print(f"per-step totals (us): miopen fwd={tot['mf']:.0f} dgrad={tot['md']:.0f} wgrad={tot['mw']:.0f}")


if __name__ == "__main__":
    main()
