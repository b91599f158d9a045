"""Where does the split-K conv data gradient deviate from the fp32 reference? (keras conv3 shape)"""
import torch
import torch.nn.functional as F

from mxddp import ops

cuda = torch.device("cuda", 0)
for relu in (False, True):
    N, C, H, W, K, R, S, st, pd = 64, 64, 5, 5, 64, 3, 3, 1, 0
    torch.manual_seed(0)
    x = torch.randn(N, C, H, W)
    w = torch.randn(K, C, R, S) * 0.1
    b = torch.randn(K)
    xr, wr, br = (t.clone().double().requires_grad_() for t in (x, w, b))
    yr = F.conv2d(xr, wr, br, st, pd)
    if relu:
        yr = F.relu(yr)
    gy = torch.randn_like(yr)
    yr.backward(gy)
    xg, wg, bg = (t.to(cuda).requires_grad_() for t in (x, w, b))
    y = ops.conv2d(xg, wg, bg, st, pd, relu=relu)
    y.backward(gy.float().to(cuda))
    torch.cuda.synchronize()
    d = (xg.grad.cpu().double() - xr.grad).abs()
    i = int(d.argmax())
    print(f"relu={relu} y err {(y.cpu().double() - yr).abs().max().item():.3e} dx max err {d.max().item():.3e} at "
          f"{list(torch.unravel_index(torch.tensor(i), d.shape))} ref {xr.grad.flatten()[i].item():.4f} "
          f"n_bad(>1e-3)={(d > 1e-3).sum().item()} dw err {(wg.grad.cpu().double() - wr.grad).abs().max().item():.3e}")
    if relu:
        mask_gpu = (y.detach().cpu() > 0)
        mask_ref = (yr.detach() > 0)
        print("mask disagreements", (mask_gpu != mask_ref).sum().item())
        # recompute dgrad on GPU from the reference-masked gradient
        g = (gy * mask_ref).float().to(cuda)
        dx2 = torch.nn.grad.conv2d_input(x.shape, w.to(cuda), g, st, pd)
        print("torch dgrad from ref mask err", (dx2.cpu().double() - xr.grad).abs().max().item())
