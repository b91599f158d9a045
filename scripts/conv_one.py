"""Run one 3x3 conv shape's fwd / dgrad / wgrad (current algo) a fixed number of times, for
rocprofv3 counter passes.  usage: conv_one.py C K W [iters]"""
import sys

import torch

sys.path.insert(0, ".")
import mxddp  # noqa: E402

C_ = mxddp.native()
C, K, W = map(int, sys.argv[1:4])
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 20
N = 64
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream().cuda_stream
x = torch.randn(N, C, W, W, device=dev)
w = torch.randn(K, C, 3, 3, device=dev) * 0.05
dy = torch.randn(N, K, W, W, device=dev)
y, dx, dw = torch.empty_like(dy), torch.empty_like(x), torch.empty_like(w)
geo = (N, C, W, W, K, 3, 3, 1, 1, 1, 1, 1, 1)
scr = torch.empty(max(1, C_.conv_scratch_floats(*geo)), device=dev)
ws = torch.empty(max(1, C_.conv_wgrad_scratch_floats(*geo)), device=dev)
for _ in range(iters):
    C_.conv2d_fwd(x.data_ptr(), w.data_ptr(), 0, y.data_ptr(), *geo, False, st, scr.data_ptr())
    C_.conv2d_dgrad(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), *geo, 0, False, st, scr.data_ptr())
    C_.conv2d_wgrad(dy.data_ptr(), x.data_ptr(), dw.data_ptr(), *geo, False, st, ws.data_ptr())
torch.cuda.synchronize()
print("done")
