"""bf16-operand MFMA path (mixed precision, BASELINE config 5): conv / linear fwd+bwd vs the
PyTorch fp32 reference, with bf16-level tolerance (8-bit mantissa operands, fp32 accumulate)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from mxddp import ops  # noqa: E402


@pytest.fixture
def bf16(cuda):
    ops.set_compute_dtype("bf16")
    yield
    ops.set_compute_dtype("fp32")


def _rel(a, b):
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


@pytest.mark.parametrize("case", [(2, 64, 14, 14, 40, 3, 3, 1, 1), (2, 3, 33, 31, 17, 7, 7, 2, 3),
                                  (3, 32, 26, 26, 64, 3, 3, 1, 0), (2, 256, 7, 7, 64, 1, 1, 1, 0)])
def test_conv2d_bf16(cuda, bf16, case):
    N, C, H, W, K, R, S, st, pd = case
    torch.manual_seed(0)
    x, w = torch.randn(N, C, H, W), torch.randn(K, C, R, S) * 0.1
    xr, wr = x.clone().requires_grad_(), w.clone().requires_grad_()
    yr = F.conv2d(xr, wr, None, st, pd)
    gy = torch.randn_like(yr)
    yr.backward(gy)
    xg, wg = x.to(cuda).requires_grad_(), w.to(cuda).requires_grad_()
    y = ops.conv2d(xg, wg, None, st, pd)
    y.backward(gy.to(cuda))
    assert ops.compute_dtype() == "bf16"
    assert _rel(y.detach().cpu(), yr.detach()) < 2e-2
    assert _rel(xg.grad.cpu(), xr.grad) < 2e-2
    assert _rel(wg.grad.cpu(), wr.grad) < 2e-2


def test_linear_bf16(cuda, bf16):
    torch.manual_seed(1)
    x, w = torch.randn(64, 2048), torch.randn(1000, 2048) * 0.02
    y = ops.linear(x.to(cuda), w.to(cuda))
    assert _rel(y.cpu(), F.linear(x, w)) < 2e-2
