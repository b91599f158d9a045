"""Effective bandwidth of the bf16 NHWC BatchNorm kernels on one ResNet-50-sized tensor, per
variant (ReLU mask from the forward's coefficients / as bits, residual add, backward with and
without the residual gradient), against a plain bf16 copy of the same bytes: which part of the
BN step is slow.  Forward variants run with precomputed statistics rows, so the timed work is the
finalize + apply; backward variants include their statistics pass.

    python scripts/bench_bn.py [N H W C] [iters]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from mxddp import native  # noqa: E402


def timed(fn, iters):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / iters


def main():
    a = [int(v) for v in sys.argv[1:5]] if len(sys.argv) >= 5 else [256, 56, 56, 256]
    iters = int(sys.argv[5]) if len(sys.argv) > 5 else 20
    N, H, W, C = a
    Cn = native()
    dev = torch.device("cuda")
    st = torch.cuda.current_stream().cuda_stream
    npix = N * H * W
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    res = torch.randn_like(x)
    y = torch.empty_like(x)
    dy = torch.randn_like(x)
    dx = torch.empty_like(x)
    dres = torch.empty_like(x)
    g = torch.rand(C, device=dev) + 0.5
    b = torch.randn(C, device=dev) * 0.1
    mean = torch.empty(C, device=dev)
    inv = torch.empty(C, device=dev)
    rm = torch.zeros(C, device=dev)
    rv = torch.ones(C, device=dev)
    dg = torch.empty(C, device=dev)
    db = torch.empty(C, device=dev)
    coef = torch.empty(2 * C, device=dev)
    mask = torch.empty(npix * C // 8, device=dev, dtype=torch.uint8)
    scr = torch.empty(Cn.nhwc_bn_scratch_floats(npix, C), device=dev)
    part = torch.zeros(2 * C, device=dev)  # one precomputed statistics row: finalize + apply only
    part[1::2] = npix
    nbytes = x.numel() * 2
    rows = []

    def fwd(relu, r, m, pre=True):
        return lambda: Cn.nhwc_bn_fwd(x.data_ptr(), r.data_ptr() if r is not None else 0, y.data_ptr(), g.data_ptr(),
                                      b.data_ptr(), mean.data_ptr(), inv.data_ptr(), rm.data_ptr(), rv.data_ptr(), 0,
                                      npix, C, 0.1, 1e-5, relu, scr.data_ptr(), st,
                                      coef.data_ptr() if (relu and r is None and not m) else 0,
                                      mask.data_ptr() if m else 0, part.data_ptr() if pre else 0, 1 if pre else 0, 0)

    def bwd(relu, fc, m, dr):
        return lambda: Cn.nhwc_bn_bwd(dy.data_ptr(), x.data_ptr(), y.data_ptr(), g.data_ptr(), mean.data_ptr(),
                                      inv.data_ptr(), dx.data_ptr(), dres.data_ptr() if dr else 0, dg.data_ptr(),
                                      db.data_ptr(), npix, C, relu, False, scr.data_ptr(), st,
                                      coef.data_ptr() if fc else 0, mask.data_ptr() if m else 0, 0, 0)

    fwd(True, None, False)()  # coefficients for the backward's mask
    fwd(True, res, True)()    # mask bits
    cases = [
        ("copy (torch, read + write)", lambda: y.copy_(x), 2 * nbytes),
        ("fwd apply, no ReLU", fwd(False, None, False), 2 * nbytes),
        ("fwd apply, ReLU (coefficients kept)", fwd(True, None, False), 2 * nbytes),
        ("fwd apply, residual + ReLU + mask bits", fwd(True, res, True), 3 * nbytes + nbytes // 16),
        ("fwd with statistics pass, ReLU", fwd(True, None, False, pre=False), 3 * nbytes),
        ("bwd (stats + apply), no ReLU", bwd(False, False, False, False), 5 * nbytes),
        ("bwd, ReLU from coefficients", bwd(True, True, False, False), 5 * nbytes),
        ("bwd, ReLU from mask bits + dres", bwd(True, False, True, True), 6 * nbytes + nbytes // 8),
    ]
    print(f"tensor {N}x{H}x{W}x{C} bf16 = {nbytes / 1e6:.1f} MB")
    for name, fn, byts in cases:
        us = timed(fn, iters)
        rows.append((name, us, byts / us / 1e6))
        print(f"{name:42s} {us:8.1f} us  {byts / us / 1e6:6.2f} TB/s (nominal bytes)", flush=True)
    # apply-kernel grid cap (2048 = the round-3 grids; 0 = the default, tensor-sized)
    for cap in (2048, 8192, 32768):
        Cn.nhwc_bn_set_grid_cap(cap)
        f_us = timed(fwd(True, None, False), iters)
        b_us = timed(bwd(True, True, False, False), iters)
        print(f"grid cap {cap:6d}: fwd apply ReLU {f_us:7.1f} us ({2 * nbytes / f_us / 1e6:5.2f} TB/s), "
              f"bwd {b_us:7.1f} us ({5 * nbytes / b_us / 1e6:5.2f} TB/s)", flush=True)
    Cn.nhwc_bn_set_grid_cap(32768)

if __name__ == "__main__":
    main()
