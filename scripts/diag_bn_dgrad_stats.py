"""Backward BN statistics from a convolution's data-gradient epilogue (ConvNArgs::bx) vs the
same sums computed in torch from the stored gradient: per kernel path (LDS-DMA 128 / 256 tile,
generic, stride-2 parity classes), prints the rows written and the max deviation of the
per-channel sum(g) and sum(g * (x - mean)).  Diagnostic only.

    python scripts/diag_bn_dgrad_stats.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from mxddp import native  # noqa: E402


def run(tag, N, H, W, C, K, R, s, pd, glds, glds256, relu_bits):
    Cn = native()
    dev = torch.device("cuda")
    st = torch.cuda.current_stream().cuda_stream
    torch.manual_seed(1)
    P, Q = (H + 2 * pd - R) // s + 1, (W + 2 * pd - R) // s + 1
    dy = torch.randn(N, P, Q, K, device=dev).to(torch.bfloat16)
    w = torch.randn(K, C, R, R, device=dev) * 0.05
    wtd = torch.empty(C * R * R * K, device=dev, dtype=torch.bfloat16)
    Cn.nhwc_repack_weight(w.data_ptr(), 0, wtd.data_ptr(), K, C, R, R, C, st)
    x = (torch.randn(N, H, W, C, device=dev) + 0.3).to(torch.bfloat16)
    mean = x.float().mean(dim=(0, 1, 2))
    mask = torch.randint(0, 256, (N * H * W * C // 8,), dtype=torch.uint8, device=dev) if relu_bits else None
    n = Cn.nhwc_conv_dgrad_scratch_floats(N, H, W, C, K, R, R, s, s, pd, pd, P, Q)
    scr = torch.empty(max(n, 1), device=dev)
    rows_cap = Cn.nhwc_conv_dgrad_bn_rows(N, H, W, C, K, R, R, s, s, pd, pd, P, Q)
    bpart = torch.full((rows_cap * 2 * C,), float("nan"), device=dev)
    dx = torch.empty(N, H, W, C, device=dev, dtype=torch.bfloat16)
    Cn.nhwc_conv_set_glds(glds)
    Cn.nhwc_conv_set_glds256(glds256)
    try:
        rows = Cn.nhwc_conv_dgrad(dy.data_ptr(), wtd.data_ptr(), dx.data_ptr(), N, H, W, C, K, R, R, s, s, pd, pd, P,
                                  Q, scr.data_ptr() if n else 0, st, 0, bpart.data_ptr(), x.data_ptr(),
                                  mean.data_ptr(), 0, mask.data_ptr() if relu_bits else 0, bool(relu_bits))
        torch.cuda.synchronize()
    finally:
        Cn.nhwc_conv_set_glds256(0)
        Cn.nhwc_conv_set_glds(1)
    g = dx.float().reshape(-1, C)
    if relu_bits:
        bits = (mask.view(-1, 1) >> torch.arange(8, device=dev, dtype=torch.uint8)) & 1
        g = g * bits.view(-1, C).float()
    ref1 = g.sum(0)
    ref2 = (g * (x.float().reshape(-1, C) - mean)).sum(0)
    if rows <= 0:
        print(f"{tag:34s} rows=0 (no epilogue statistics)")
        return
    p = bpart[: rows * 2 * C].view(rows, C, 2)
    nan_rows = int(torch.isnan(p).any(dim=(1, 2)).sum())
    s1, s2 = p[..., 0].sum(0), p[..., 1].sum(0)
    e1 = ((s1 - ref1).abs().max() / (ref1.abs().max() + 1e-6)).item()
    e2 = ((s2 - ref2).abs().max() / (ref2.abs().max() + 1e-6)).item()
    print(f"{tag:34s} rows={rows:5d} (cap {rows_cap}) nan_rows={nan_rows} err_sum_g={e1:.2e} err_sum_gx={e2:.2e}")


def main():
    # (tag, N, H, W, C, K, R, stride, pad, glds mode, glds256 mode, relu bits)
    cases = [
        ("glds128 1x1 C128 K256", 4, 16, 16, 128, 256, 1, 1, 0, 2, 0, False),
        ("glds128 1x1 C128 K256 relu", 4, 16, 16, 128, 256, 1, 1, 0, 2, 0, True),
        ("glds256 1x1 C256 K256", 2, 10, 10, 256, 256, 1, 1, 0, 2, 2, False),
        ("glds256 3x3 C256 K128", 2, 10, 10, 256, 128, 3, 1, 1, 2, 2, False),
        ("glds256 3x3 C256 K128 relu", 2, 10, 10, 256, 128, 3, 1, 1, 2, 2, True),
        ("generic 1x1 C64 K64", 4, 16, 16, 64, 64, 1, 1, 0, 0, 0, False),
        ("generic 3x3 s2 C64 K128 relu", 4, 16, 16, 64, 128, 3, 2, 1, 0, 0, True),
        ("generic 3x3 s2 C64 K128", 4, 16, 16, 64, 128, 3, 2, 1, 0, 0, False),
    ]
    for c in cases:
        run(*c)


def bn_pre_path():
    """nhwc_bn_bwd with precomputed partial rows (one row of torch sums) vs its own statistics pass."""
    Cn = native()
    dev = torch.device("cuda")
    st = torch.cuda.current_stream().cuda_stream
    torch.manual_seed(2)
    N, H, W, C = 2, 10, 10, 256
    npix = N * H * W
    x = (torch.randn(N, H, W, C, device=dev) + 0.3).to(torch.bfloat16)
    dy = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    gamma = torch.rand(C, device=dev) + 0.5
    beta = torch.randn(C, device=dev) * 0.2
    mean = torch.empty(C, device=dev)
    invstd = torch.empty(C, device=dev)
    y = torch.empty_like(x)
    scr = torch.empty(Cn.nhwc_bn_scratch_floats(npix, C), device=dev)
    Cn.nhwc_bn_fwd(x.data_ptr(), 0, y.data_ptr(), gamma.data_ptr(), beta.data_ptr(), mean.data_ptr(),
                   invstd.data_ptr(), 0, 0, 0, npix, C, 0.1, 1e-5, False, scr.data_ptr(), st, 0, 0, 0, 0, 0)
    outs = []
    for use_pre in (False, True):
        dx = torch.empty_like(x)
        dg = torch.empty(C, device=dev)
        db = torch.empty(C, device=dev)
        pre = None
        if use_pre:
            g = dy.float().reshape(-1, C)
            pre = torch.stack([g.sum(0), (g * (x.float().reshape(-1, C) - mean)).sum(0)], 1).reshape(-1).contiguous()
        Cn.nhwc_bn_bwd(dy.data_ptr(), x.data_ptr(), 0, gamma.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                       dx.data_ptr(), 0, dg.data_ptr(), db.data_ptr(), npix, C, False, False, scr.data_ptr(), st, 0, 0,
                       pre.data_ptr() if use_pre else 0, 1 if use_pre else 0)
        torch.cuda.synchronize()
        outs.append((dx.float(), dg.clone(), db.clone()))
    for name, a, b in zip(("dx", "dgamma", "dbeta"), *outs):
        print(f"bn_bwd pre path {name:7s} rel err {((a - b).abs().max() / (b.abs().max() + 1e-6)).item():.2e}")


if __name__ == "__main__":
    main()
    bn_pre_path()
