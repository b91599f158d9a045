import torch, torch.nn.functional as F
from mxddp import ops
cuda = torch.device("cuda", 0)
def run(shape, offset, relu):
    torch.manual_seed(4)
    C = shape[1]
    x = torch.randn(*shape) * 2 + offset
    g, b = torch.rand(C) + 0.5, torch.randn(C)
    rm, rv = torch.zeros(C), torch.ones(C)
    xr, gr, br = (t.clone().requires_grad_() for t in (x, g, b))
    yr = F.batch_norm(xr, rm, rv, gr, br, True, 0.1, 1e-5)
    if relu: yr = F.relu(yr)
    gy = torch.randn_like(yr)
    yr.backward(gy)
    rmg, rvg = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    xg, gg, bg = (t.to(cuda).requires_grad_() for t in (x, g, b))
    y = ops.batch_norm(xg, gg, bg, rmg, rvg, True, 0.1, 1e-5, relu=relu)
    y.backward(gy.to(cuda))
    e = (gg.grad.cpu() - gr.grad).abs()
    eb = (bg.grad.cpu() - br.grad).abs()
    print(shape, relu, "dgamma maxerr %.3g (max|dg| %.3g) worst ch %d; dbeta maxerr %.3g; dx rel %.3g" % (
        e.max(), gr.grad.abs().max(), e.argmax(), eb.max(), ((xg.grad.cpu()-xr.grad).abs().max()/xr.grad.abs().max()).item()))
run((32, 64, 56, 56), 1.0, True)
run((32, 64, 56, 56), 1.0, False)
run((32, 64, 56, 56), 1.0, True)
run((8, 64, 56, 56), 1.0, True)
run((32, 8, 56, 56), 1.0, True)
