"""Localise differences between residual-join / BN-statistics variants of two bf16 NHWC
Bottleneck blocks (the setting of tests/test_gpu_nhwc.py's join tests): for each variant, the
gradients of the block input and of every parameter are compared with a baseline run, and the
baseline is repeated to measure run-to-run nondeterminism.  Prints, per tensor, the max error
relative to the tensor's max and where it sits (pixel / channel for the input gradient).
Diagnostic only.

    python scripts/diag_join.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from mxddp import native  # noqa: E402
from mxddp.models.resnet import Bottleneck  # noqa: E402
from mxddp.ops import nhwc  # noqa: E402


def run(blocks, x, stats, lazy, unroll):
    native().nhwc_bn_set_unroll(unroll)
    nhwc._BN_STATS_IN_DGRAD = stats
    nhwc._LAZY_JOIN = lazy
    for blk in blocks:
        blk.zero_grad()
    xg = x.clone().requires_grad_()
    y = xg
    for blk in blocks:
        y = blk.forward_nhwc(y)
    gy = torch.randn(y.shape, generator=torch.Generator().manual_seed(8)).to(torch.bfloat16).to(x.device)
    y.backward(gy)
    torch.cuda.synchronize()
    names = ["x"] + [f"b{i}.{n}" for i, blk in enumerate(blocks) for n, _ in blk.named_parameters()]
    vals = [xg.grad.float().cpu()] + [p.grad.float().cpu() for blk in blocks for p in blk.parameters()]
    return dict(zip(names, vals)), y.float().cpu()


def compare(tag, ref, out):
    worst = []
    for k, a in ref.items():
        b = out[k]
        d = (a - b).abs()
        rel = (d.max() / (a.abs().max() + 1e-6)).item()
        worst.append((rel, k, d))
    worst.sort(key=lambda t: -t[0])
    print(f"{tag}: " + ", ".join(f"{k} {r:.2e}" for r, k, _ in worst[:4]))
    r, k, d = worst[0]
    if r > 1e-2 and d.dim() == 4:
        idx = (d == d.max()).nonzero()[0].tolist()
        n_bad = int((d > 0.1 * d.max()).sum())
        chans = sorted(set((d > 0.1 * d.max()).nonzero()[:, 3].tolist()))[:16]
        pix = sorted(set(((d > 0.1 * d.max()).nonzero()[:, 0] * 10000 + (d > 0.1 * d.max()).nonzero()[:, 1] * 100 +
                          (d > 0.1 * d.max()).nonzero()[:, 2]).tolist()))[:16]
        print(f"   {k}: max at {idx}, {n_bad} elements > 10% of max; channels {chans}; (n,h,w) {pix}")


def main():
    dev = torch.device("cuda")
    torch.manual_seed(12)
    for nblk, shape in ((2, (2, 14, 14, 256)), (3, (2, 14, 14, 256)), (2, (4, 8, 8, 256))):
        blocks = [Bottleneck(256, 64).to(dev) for _ in range(nblk)]
        x = torch.randn(*shape).to(torch.bfloat16).to(dev)
        print(f"== {nblk} blocks, input {shape}")
        base, y0 = run(blocks, x, False, False, 2)
        again, y1 = run(blocks, x, False, False, 2)
        print(f"forward output repeat: {((y0 - y1).abs().max()).item():.3e}")
        compare("repeat (no stats, materialised join, unroll 2)", base, again)
        compare("unroll 4", base, run(blocks, x, False, False, 4)[0])
        compare("lazy join", base, run(blocks, x, False, True, 2)[0])
        compare("dgrad statistics, materialised join", base, run(blocks, x, True, False, 2)[0])
        compare("dgrad statistics + lazy join", base, run(blocks, x, True, True, 2)[0])
    nhwc._BN_STATS_IN_DGRAD = nhwc._BN_STATS_IN_CONV
    nhwc._LAZY_JOIN = True
    native().nhwc_bn_set_unroll(4)


if __name__ == "__main__":
    main()
