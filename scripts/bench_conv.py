"""Per-shape timing of the 3x3 s1 convolutions of PyramidNet-110 (B = 64): fwd / dgrad / wgrad of
the Winograd and direct-LDS paths vs stock PyTorch-ROCm (MIOpen).  Prints one JSON line per shape."""
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
import mxddp  # noqa: E402

C_ = mxddp.native()
SHAPES = [(16, 21, 32), (56, 61, 32), (66, 71, 32), (96, 101, 32), (106, 111, 16), (126, 131, 16),
          (146, 151, 16), (161, 166, 16), (181, 186, 16), (191, 196, 8), (211, 216, 8), (231, 236, 8),
          (251, 256, 8), (266, 271, 8)]
if "--shapes" in sys.argv:  # e.g. --shapes 146,151,16:266,271,8
    SHAPES = [tuple(int(v) for v in t.split(",")) for t in sys.argv[sys.argv.index("--shapes") + 1].split(":")]
N = 64
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream().cuda_stream


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


ONLY_WINO = "--only-wino" in sys.argv  # compare forward variants (MXDDP_WINO_FWD) quickly

for (C, K, W) in SHAPES:
    x = torch.randn(N, C, W, W, device=dev)
    w = torch.randn(K, C, 3, 3, device=dev) * 0.05
    dy = torch.randn(N, K, W, W, device=dev)
    y = torch.empty(N, K, W, W, device=dev)
    dx = torch.empty_like(x)
    dw = torch.empty_like(w)
    geo = (N, C, W, W, K, 3, 3, 1, 1, 1, 1, 1, 1)
    res = {"C": C, "K": K, "W": W, "gflop_direct_each": round(2 * 9 * C * K * W * W * N / 1e9, 3)}
    for algo, name in ((0, "wino"),) if ONLY_WINO else ((0, "wino"), (1, "direct")):
        C_.set_conv_algo(algo)
        scr = torch.empty(max(1, C_.conv_scratch_floats(*geo)), device=dev)
        ws = torch.empty(max(1, C_.conv_wgrad_scratch_floats(*geo)), device=dev)
        res[name + "_fwd"] = round(timeit(lambda: C_.conv2d_fwd(x.data_ptr(), w.data_ptr(), 0, y.data_ptr(), *geo, False, st, scr.data_ptr())), 1)
        res[name + "_dgrad"] = round(timeit(lambda: C_.conv2d_dgrad(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), *geo, 0, False, st, scr.data_ptr())), 1)
        res[name + "_wgrad"] = round(timeit(lambda: C_.conv2d_wgrad(dy.data_ptr(), x.data_ptr(), dw.data_ptr(), *geo, False, st, ws.data_ptr())), 1)
    C_.set_conv_algo(0)
    if ONLY_WINO:
        print(json.dumps(res), flush=True)
        continue
    res["miopen_fwd"] = round(timeit(lambda: F.conv2d(x, w, None, 1, 1)), 1)
    res["miopen_dgrad"] = round(timeit(lambda: torch.nn.grad.conv2d_input(x.shape, w, dy, 1, 1)), 1)
    res["miopen_wgrad"] = round(timeit(lambda: torch.nn.grad.conv2d_weight(x, w.shape, dy, 1, 1)), 1)
    print(json.dumps(res), flush=True)
