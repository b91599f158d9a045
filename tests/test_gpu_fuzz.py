"""Hypothesis-fuzzed shapes for the HIP kernels (SURVEY §4.2 tier T1): random batch / channel /
spatial sizes that are not tile multiples (PyramidNet's channel counts are 16 + 5k), random
stride / padding / kernel size, asymmetric random operands, every result against a plain
PyTorch fp32 CPU reference of the same op (forward and all gradients).  Examples are drawn
with a fixed seed (derandomize) so a GPU run is reproducible; each test stays well under a
second per example."""
import pytest
import torch
import torch.nn.functional as F
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

pytestmark = pytest.mark.gpu

from mxddp import ops  # noqa: E402

FUZZ = settings(max_examples=20, deadline=None, derandomize=True,
                suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])


def _rel(a, b):
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


@st.composite
def conv_shapes(draw):
    k = draw(st.sampled_from([1, 3, 3, 3, 5, 7]))
    stride = draw(st.sampled_from([1, 1, 2]))
    pad = draw(st.integers(0, k // 2))
    h = draw(st.integers(k, 20))
    w = draw(st.integers(k, 20))
    return (draw(st.integers(1, 4)), draw(st.integers(1, 48)), h, w, draw(st.integers(1, 48)), k, stride, pad)


@FUZZ
@given(shape=conv_shapes(), relu=st.booleans())
def test_conv2d_fuzz(cuda, shape, relu):
    N, C, H, W, K, k, s, p = shape
    g = torch.Generator().manual_seed(N * 7919 + C * 131 + K)
    x = torch.randn(N, C, H, W, generator=g)
    w = torch.randn(K, C, k, k, generator=g) / (k * C ** 0.5)
    b = torch.randn(K, generator=g)
    xr, wr, br = (t.clone().requires_grad_() for t in (x, w, b))
    yr = F.conv2d(xr, wr, br, s, p)
    if relu:
        yr = F.relu(yr)
    gy = torch.randn(yr.shape, generator=g)
    yr.backward(gy)
    xg, wg, bg = (t.to(cuda).requires_grad_() for t in (x, w, b))
    y = ops.conv2d(xg, wg, bg, s, p, relu=relu)
    y.backward(gy.to(cuda))
    torch.cuda.synchronize()
    assert y.shape == yr.shape
    for got, want in ((y, yr.detach()), (xg.grad, xr.grad), (wg.grad, wr.grad), (bg.grad, br.grad)):
        assert _rel(got.cpu(), want) < 2e-4, shape


@FUZZ
@given(M=st.integers(1, 130), N=st.integers(1, 140), K=st.integers(1, 600), relu=st.booleans())
def test_linear_fuzz(cuda, M, N, K, relu):
    g = torch.Generator().manual_seed(M * 1009 + N * 31 + K)
    x, w, b = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) / K ** 0.5, torch.randn(N, generator=g)
    xr, wr, br = (t.clone().requires_grad_() for t in (x, w, b))
    yr = F.linear(xr, wr, br)
    if relu:
        yr = F.relu(yr)
    gy = torch.randn(yr.shape, generator=g)
    yr.backward(gy)
    xg, wg, bg = (t.to(cuda).requires_grad_() for t in (x, w, b))
    y = ops.linear(xg, wg, bg, relu=relu)
    y.backward(gy.to(cuda))
    torch.cuda.synchronize()
    for got, want in ((y, yr.detach()), (xg.grad, xr.grad), (wg.grad, wr.grad), (bg.grad, br.grad)):
        assert _rel(got.cpu(), want) < 2e-4, (M, N, K)


@FUZZ
@given(N=st.integers(1, 6), C=st.integers(1, 40), H=st.integers(1, 17), W=st.integers(1, 17), relu=st.booleans())
def test_batch_norm_train_fuzz(cuda, N, C, H, W, relu):
    if N * H * W < 2:
        return  # train-mode BN needs two values per channel (torch raises too)
    g = torch.Generator().manual_seed(N * 97 + C * 13 + H * 5 + W)
    x = torch.randn(N, C, H, W, generator=g) * 2 + 0.5
    gamma, beta = torch.randn(C, generator=g), torch.randn(C, generator=g)
    xr, gr, brr = (t.clone().requires_grad_() for t in (x, gamma, beta))
    rmr, rvr = torch.zeros(C), torch.ones(C)
    yr = F.batch_norm(xr, rmr, rvr, gr, brr, training=True, momentum=0.1, eps=1e-5)
    if relu:
        yr = F.relu(yr)
    gy = torch.randn(yr.shape, generator=g)
    yr.backward(gy)
    xg, gg, bg = (t.to(cuda).requires_grad_() for t in (x, gamma, beta))
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    y = ops.batch_norm(xg, gg, bg, rm, rv, True, momentum=0.1, eps=1e-5, relu=relu)
    y.backward(gy.to(cuda))
    torch.cuda.synchronize()
    # running statistics (unbiased variance) as torch.nn.BatchNorm2d
    assert _rel(rm.cpu(), rmr) < 1e-5 and _rel(rv.cpu(), rvr) < 1e-5
    for got, want in ((y, yr.detach()), (xg.grad, xr.grad), (gg.grad, gr.grad), (bg.grad, brr.grad)):
        # floor on the scale: with 2 values per channel dx cancels to ~0 exactly (x_hat = +-1)
        err = (got.cpu() - want).abs().max().item() / max(want.abs().max().item(), 1e-3)
        assert err < 5e-4, (N, C, H, W)


@FUZZ
@given(N=st.integers(1, 4), C=st.integers(1, 20), H=st.integers(2, 19), W=st.integers(2, 19),
       kind=st.sampled_from(["max", "avg", "avg_ceil"]))
def test_pool_fuzz(cuda, N, C, H, W, kind):
    g = torch.Generator().manual_seed(N * 11 + C * 7 + H * 3 + W)
    x = torch.randn(N, C, H, W, generator=g)
    xr = x.clone().requires_grad_()
    if kind == "max":
        yr = F.max_pool2d(xr, 2)
    else:
        yr = F.avg_pool2d(xr, 2, ceil_mode=kind == "avg_ceil")
    gy = torch.randn(yr.shape, generator=g)
    yr.backward(gy)
    xg = x.to(cuda).requires_grad_()
    y = ops.max_pool2d(xg, 2) if kind == "max" else ops.avg_pool2d(xg, 2, ceil_mode=kind == "avg_ceil")
    y.backward(gy.to(cuda))
    torch.cuda.synchronize()
    assert y.shape == yr.shape
    assert _rel(y.cpu(), yr.detach()) < 1e-5 and _rel(xg.grad.cpu(), xr.grad) < 1e-5
