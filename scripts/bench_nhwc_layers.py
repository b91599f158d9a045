"""Per-layer timing of the channels-last bf16 convolution kernels on every distinct ResNet-50
conv shape at batch 32 (forward, data gradient, weight gradient): microseconds and TFLOP/s per
direction, so the conv-kernel work can be prioritised by where the step time goes.

    python scripts/bench_nhwc_layers.py [batch] [iters] [tile256] [glds_short] [wgrad_tile256] [glds_deep]

Every switch defaults to the build's production choice; env GK2=0/1/2 picks the two-stage
128 x 128 conv tile kernel (nhwc_conv_set_gk2).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from mxddp import native  # noqa: E402


def shapes(batch):
    """(count per step, N, H, W, C, K, R, stride, pad) of every ResNet-50 conv (224 input)."""
    out = [(1, batch, 224, 224, 8, 64, 7, 2, 3)]
    inp, hw = 64, 56
    for planes, blocks, stride in ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)):
        for b in range(blocks):
            s = stride if b == 0 else 1
            out.append((1, batch, hw, hw, inp, planes, 1, 1, 0))
            out.append((1, batch, hw, hw, planes, planes, 3, s, 1))
            ohw = hw // s
            out.append((1, batch, ohw, ohw, planes, planes * 4, 1, 1, 0))
            if b == 0:
                out.append((1, batch, hw, hw, inp, planes * 4, 1, s, 0))
            inp, hw = planes * 4, ohw
    agg = {}
    for c, *k in out:
        agg[tuple(k)] = agg.get(tuple(k), 0) + c
    return [(c,) + k for k, c in agg.items()]


def main():
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    tile256 = int(sys.argv[3]) if len(sys.argv) > 3 else 1  # 1: the 256 x 256-tile kernel where it fits (default)
    dev = torch.device("cuda")
    Cn = native()
    Cn.nhwc_conv_set_glds256(tile256)
    if len(sys.argv) > 4:  # the two-stage 128-pixel LDS-DMA variant for short reductions (default 1)
        Cn.nhwc_conv_set_glds_short(int(sys.argv[4]))
    if len(sys.argv) > 5:  # 256 x 256 weight-gradient tiles (default 1)
        Cn.nhwc_wgrad_set_tile256(int(sys.argv[5]))
    if len(sys.argv) > 6:  # 128 x 128 LDS-DMA tiles for deep reductions on few tiles (default 1)
        Cn.nhwc_conv_set_glds_deep(int(sys.argv[6]))
    if "GK2" in os.environ:  # two-stage 128 x 128 tiles: 0 8-wave 64 x 32, 1 / 2 gk2 (16x16x32 / 32x32x16)
        Cn.nhwc_conv_set_gk2(int(os.environ["GK2"]))
    st = torch.cuda.current_stream().cuda_stream
    tot = {"fwd": 0.0, "dgrad": 0.0, "dgrad_st": 0.0, "wgrad": 0.0}
    # floor: max(HBM bytes at 8 TB/s, FLOPs at the 2.5 PF bf16 dense peak), the same for all three
    # directions to first order (each reads / writes one activation pair and the weights)
    print(f"{'count':>5} {'N':>3} {'H':>4} {'C':>5} {'K':>5} {'R':>2} {'s':>2} | "
          f"{'fwd us':>8} {'TF':>5} | {'dgrad us':>8} {'TF':>5} | {'+bnst us':>8} | {'wgrad us':>8} {'TF':>5} | "
          f"{'floor us':>8}")
    for cnt, N, H, W, C, K, R, s, p in shapes(batch):
        P, Q = (H + 2 * p - R) // s + 1, (W + 2 * p - R) // s + 1
        x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
        w = torch.randn(K, C, R, R, device=dev) * 0.05
        wt = torch.empty(K * R * R * C, device=dev, dtype=torch.bfloat16)
        wtd = torch.empty(C * R * R * K, device=dev, dtype=torch.bfloat16)
        Cn.nhwc_repack_weight(w.data_ptr(), wt.data_ptr(), wtd.data_ptr(), K, C, R, R, C, st)
        y = torch.empty(N, P, Q, K, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(N, P, Q, K, device=dev).to(torch.bfloat16)
        dx = torch.empty_like(x)
        dw = torch.empty_like(w)
        sf = Cn.nhwc_conv_scratch_floats(N * P * Q, K, R * R * C)
        sd = Cn.nhwc_conv_dgrad_scratch_floats(N, H, W, C, K, R, R, s, s, p, p, P, Q)
        sw = Cn.nhwc_wgrad_scratch_floats(N, C, K, R, R, P, Q)
        scr = torch.empty(max(sf, sd, sw, 1), device=dev)
        # the data gradient with the producing BN's backward statistics in its epilogue (ReLU mask
        # from the forward's coefficients), as the training step runs it
        bmean = torch.randn(C, device=dev)
        bcoef = torch.randn(2 * C, device=dev)
        brows = Cn.nhwc_conv_dgrad_bn_rows(N, H, W, C, K, R, R, s, s, p, p, P, Q)
        bpart = torch.empty(brows * 2 * C, device=dev)
        flops = 2.0 * N * P * Q * K * C * R * R
        hbm_bytes = 2.0 * (N * H * W * C + N * P * Q * K) + 2.0 * K * C * R * R
        floor_us = max(hbm_bytes / 8e12, flops / 2.5e15) * 1e6
        runs = {
            "fwd": lambda: Cn.nhwc_conv_fwd(x.data_ptr(), wt.data_ptr(), y.data_ptr(), N, H, W, C, K, R, R, s, s, p, p,
                                            P, Q, scr.data_ptr() if sf else 0, st),
            "dgrad": lambda: Cn.nhwc_conv_dgrad(dy.data_ptr(), wtd.data_ptr(), dx.data_ptr(), N, H, W, C, K, R, R, s, s,
                                                p, p, P, Q, scr.data_ptr() if sd else 0, st),
            "dgrad_st": lambda: Cn.nhwc_conv_dgrad(dy.data_ptr(), wtd.data_ptr(), dx.data_ptr(), N, H, W, C, K, R, R, s,
                                                   s, p, p, P, Q, scr.data_ptr() if sd else 0, st, 0, bpart.data_ptr(),
                                                   x.data_ptr(), bmean.data_ptr(), bcoef.data_ptr(), 0, True, 0),
            "wgrad": lambda: Cn.nhwc_conv_wgrad(dy.data_ptr(), x.data_ptr(), dw.data_ptr(), N, H, W, C, C, K, R, R, s,
                                                s, p, p, P, Q, False, scr.data_ptr(), st),
        }
        res = {}
        for name, fn in runs.items():
            if name.startswith("dgrad") and C == 8:
                res[name] = (0.0, 0.0)
                continue
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1000.0 / iters
            res[name] = (us, flops / us / 1e6)
            tot[name] += us * cnt
        print(f"{cnt:5d} {N:3d} {H:4d} {C:5d} {K:5d} {R:2d} {s:2d} | "
              f"{res['fwd'][0]:8.1f} {res['fwd'][1]:5.0f} | {res['dgrad'][0]:8.1f} {res['dgrad'][1]:5.0f} | "
              f"{res['dgrad_st'][0]:8.1f} | {res['wgrad'][0]:8.1f} {res['wgrad'][1]:5.0f} | {floor_us:8.1f}", flush=True)
    print("per-step totals (us): " + " ".join(f"{k}={v:.0f}" for k, v in tot.items()) +
          f" all (without dgrad_st)={sum(v for k, v in tot.items() if k != 'dgrad_st'):.0f}")


if __name__ == "__main__":
    main()
