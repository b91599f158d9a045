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


def reference(blocks, x):
    """fp32 CPU autograd of the same blocks (NCHW, torch ops, training-mode BN on batch
    statistics), with the bf16 input and output gradient of the GPU runs."""
    import torch.nn.functional as F

    xr = x.float().cpu().permute(0, 3, 1, 2).contiguous().requires_grad_()
    params = []
    y = xr
    for blk in blocks:
        ws = [blk.conv1.weight, blk.conv2.weight, blk.conv3.weight]
        bns = [blk.bn1, blk.bn2, blk.bn3]
        w = [t.detach().float().cpu().requires_grad_() for t in ws]
        gb = [(b.weight.detach().float().cpu().requires_grad_(), b.bias.detach().float().cpu().requires_grad_())
              for b in bns]
        params.append((w, gb))
        h = F.conv2d(y, w[0])
        h = F.relu(F.batch_norm(h, None, None, gb[0][0], gb[0][1], training=True, eps=bns[0].eps))
        h = F.conv2d(h, w[1], stride=blk.conv2.stride, padding=blk.conv2.padding)
        h = F.relu(F.batch_norm(h, None, None, gb[1][0], gb[1][1], training=True, eps=bns[1].eps))
        h = F.conv2d(h, w[2])
        h = F.batch_norm(h, None, None, gb[2][0], gb[2][1], training=True, eps=bns[2].eps)
        y = F.relu(h + y)
    gy = torch.randn(tuple(y.permute(0, 2, 3, 1).shape), generator=torch.Generator().manual_seed(8))
    gy = gy.to(torch.bfloat16).float().permute(0, 3, 1, 2)
    y.backward(gy)
    out = {"x": xr.grad.permute(0, 2, 3, 1).contiguous()}
    for i, (blk, (w, gb)) in enumerate(zip(blocks, params)):
        grads = {"conv1.weight": w[0].grad, "conv2.weight": w[1].grad, "conv3.weight": w[2].grad,
                 "bn1.weight": gb[0][0].grad, "bn1.bias": gb[0][1].grad, "bn2.weight": gb[1][0].grad,
                 "bn2.bias": gb[1][1].grad, "bn3.weight": gb[2][0].grad, "bn3.bias": gb[2][1].grad}
        for n, _ in blk.named_parameters():
            out[f"b{i}.{n}"] = grads[n]
    return out


def compare(tag, ref, out):
    worst = []
    for k, a in ref.items():
        b = out[k]
        d = (a - b).abs()
        rel = (d.max() / (a.abs().max() + 1e-6)).item()
        nrm = ((a - b).norm() / (a.norm() + 1e-12)).item()
        worst.append((rel, k, d, nrm))
    worst.sort(key=lambda t: -t[0])
    print(f"{tag}: max-rel " + ", ".join(f"{k} {r:.2e}" for r, k, _, _ in worst[:4]) +
          f" | norm-rel max {max(t[3] for t in worst):.2e} (" +
          ", ".join(f"{t[1]} {t[3]:.2e}" for t in sorted(worst, key=lambda t: -t[3])[:3]) + ")")
    r, k, d, _ = worst[0]
    if r > 1e-2 and d.dim() == 4:
        idx = (d == d.max()).nonzero()[0].tolist()
        n_bad = int((d > 0.1 * d.max()).sum())
        chans = sorted(set((d > 0.1 * d.max()).nonzero()[:, 3].tolist()))[:16]
        pix = sorted(set(((d > 0.1 * d.max()).nonzero()[:, 0] * 10000 + (d > 0.1 * d.max()).nonzero()[:, 1] * 100 +
                          (d > 0.1 * d.max()).nonzero()[:, 2]).tolist()))[:16]
        print(f"   {k}: max at {idx}, {n_bad} elements > 10% of max; channels {chans}; (n,h,w) {pix}")


def forward_trace(blk, x):
    """Every intermediate of one block's NHWC forward (training mode), for the determinism probe."""
    N = nhwc
    out = []
    join = N.GradJoin()
    a, xs = N.fork(x, join)
    c1 = N.conv2d(a, blk.conv1.weight, join=join, bn=blk.bn1)
    out.append(("conv1", c1))
    h1 = N.batch_norm(c1, blk.bn1, relu=True)
    out.append(("bn1", h1))
    c2 = N.conv2d(h1, blk.conv2.weight, blk.conv2.stride, blk.conv2.padding, bn=blk.bn2)
    out.append(("conv2", c2))
    h2 = N.batch_norm(c2, blk.bn2, relu=True)
    out.append(("bn2", h2))
    c3 = N.conv2d(h2, blk.conv3.weight, bn=blk.bn3)
    out.append(("conv3", c3))
    y = N.batch_norm(c3, blk.bn3, relu=True, res=xs, join=join)
    out.append(("bn3", y))
    return [(n, t.detach().float().cpu()) for n, t in out]


def determinism_probe(dev):
    torch.manual_seed(21)
    for shape in ((4, 8, 8, 256), (2, 14, 14, 256)):
        blk = Bottleneck(256, 64).to(dev)
        x = torch.randn(*shape).to(torch.bfloat16).to(dev)
        runs = [forward_trace(blk, x) for _ in range(4)]
        for i, (name, t0) in enumerate(runs[0]):
            diffs = [(r[i][1] - t0).abs().max().item() for r in runs[1:]]
            print(f"determinism {shape} {name}: max |run k - run 0| = {', '.join(f'{d:.3e}' for d in diffs)}")


def main():
    dev = torch.device("cuda")
    determinism_probe(dev)
    torch.manual_seed(12)
    for nblk, shape in ((2, (2, 14, 14, 256)), (3, (2, 14, 14, 256)), (2, (4, 8, 8, 256))):
        blocks = [Bottleneck(256, 64).to(dev) for _ in range(nblk)]
        x = torch.randn(*shape).to(torch.bfloat16).to(dev)
        print(f"== {nblk} blocks, input {shape}")
        fp32 = reference(blocks, x)
        base, y0 = run(blocks, x, False, False, 2)
        compare("baseline vs fp32 CPU reference", fp32, base)
        compare("lazy join vs fp32 CPU reference", fp32, run(blocks, x, False, True, 2)[0])
        compare("statistics + lazy join vs fp32 CPU reference", fp32, run(blocks, x, True, True, 2)[0])
        again, y1 = run(blocks, x, False, False, 2)
        print(f"forward output repeat: {((y0 - y1).abs().max()).item():.3e}")
        compare("repeat (no stats, materialised join, unroll 2)", base, again)
        compare("unroll 4", base, run(blocks, x, False, False, 4)[0])
        compare("lazy join", base, run(blocks, x, False, True, 2)[0])
        compare("dgrad statistics, materialised join", base, run(blocks, x, True, False, 2)[0])
        compare("dgrad statistics + lazy join", base, run(blocks, x, True, True, 2)[0])
    nhwc._BN_STATS_IN_DGRAD = False
    nhwc._LAZY_JOIN = True
    native().nhwc_bn_set_unroll(4)


if __name__ == "__main__":
    main()
