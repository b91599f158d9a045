"""Reproduce the order-dependent BN dgamma error: run test_gpu_ops.py's tests in file order via
pytest's API up to the failing case, then inspect per-channel errors."""
import sys

import pytest
import torch
import torch.nn.functional as F

from mxddp import ops

cuda = torch.device("cuda", 0)


def run(shape, offset, relu, tag):
    torch.manual_seed(4)
    C = shape[1]
    x = torch.randn(*shape) * 2 + offset
    g, b = torch.rand(C) + 0.5, torch.randn(C)
    rm, rv = torch.zeros(C), torch.ones(C)
    xr, gr, br = (t.clone().requires_grad_() for t in (x, g, b))
    yr = F.batch_norm(xr, rm, rv, gr, br, True, 0.1, 1e-5)
    if relu:
        yr = F.relu(yr)
    gy = torch.randn_like(yr)
    yr.backward(gy)
    rmg, rvg = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    xg, gg, bg = (t.to(cuda).requires_grad_() for t in (x, g, b))
    y = ops.batch_norm(xg, gg, bg, rmg, rvg, True, 0.1, 1e-5, relu=relu)
    y.backward(gy.to(cuda))
    e = (gg.grad.cpu() - gr.grad).abs()
    bad = (e > 1e-3 * gr.grad.abs().max()).nonzero().flatten().tolist()
    print(tag, shape, relu, "dgamma max err %.3g / %.3g, bad channels %s" % (e.max(), gr.grad.abs().max(), bad[:20]))
    if bad:
        c = bad[0]
        print("   ch", c, "ours", gg.grad[c].item(), "ref", gr.grad[c].item(), "dbeta ours/ref", bg.grad[c].item(),
              br.grad[c].item())
    return bad


# 1) the failing case alone, 2) after the whole ops file (minus itself)
run((32, 64, 56, 56), 1.0, True, "fresh")
rc = pytest.main(["-q", "-m", "gpu", "tests/test_gpu_ops.py", "-k", "not test_batchnorm", "-p", "no:cacheprovider"])
print("pytest rc", rc)
for i in range(3):
    run((32, 64, 56, 56), 1.0, True, f"after-ops-{i}")
run((32, 64, 56, 56), 1.0, False, "after-ops-norelu")
from mxddp.ops import _BN_ACC
for k, v in _BN_ACC.items():
    print("acc", k, "parity", v[1], "hiwater", v[2], "nonzero next:", (v[0][v[1]] != 0).sum().item())
