"""PyramidNet's BN -> conv3x3 with the BN normalise pass folded into the Winograd convolution
(ops.bn_conv, opt-in: ops.set_bn_fold / MXDDP_BN_FOLD=1).  The convolution forms
relu?(x * scale + shift) while staging its input -- the BN apply kernel's own fmaf -- and the BN
backward recomputes its ReLU mask from x, so a residual block on 16 x 16 / 8 x 8 images trains
BIT FOR BIT like the unfolded chain: forward output, every gradient, running statistics.  Within
rounding: 32 x 32 layers (the folded forward runs the per-window kernel, the unfolded one the
patch-staged kernel) and the stride-2 conv1's weight gradient (float atomics).  Plus the fold
against the fp32 CPU reference of the same block, and a whole PyramidNet-110 step with the fold
on and off.
"""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

from mxddp import ops  # noqa: E402

# (N, Cin, Cout, stride, W): stage 1 / 2 / 3 widths, odd channel counts, both stride-2 entries,
# the patch-staged 32 x 32 kernel and the window kernels (16 x 16, 8 x 8)
BLOCKS = [
    (8, 16, 21, 1, 32),
    (4, 96, 101, 1, 32),
    (8, 101, 106, 2, 32),
    (16, 106, 111, 1, 16),
    (16, 186, 191, 2, 16),
    (32, 191, 196, 1, 8),
]


def _run(block, x, gy):
    x = x.clone().requires_grad_(True)
    y = block(x)
    y.backward(gy)
    grads = {n: p.grad.clone() for n, p in block.named_parameters()}
    bufs = {n: b.clone() for n, b in block.named_buffers()}
    return y.detach(), x.grad.detach(), grads, bufs


@pytest.mark.parametrize("cfg", BLOCKS, ids=[f"{c[1]}-{c[2]}-s{c[3]}-w{c[4]}" for c in BLOCKS])
def test_folded_block_is_bitwise_the_unfolded_one(cuda, cfg):
    from mxddp.models.pyramidnet import ResidualBlock

    N, Cin, Cout, stride, W = cfg
    torch.manual_seed(0)
    b0 = ResidualBlock(Cin, Cout, stride)
    with torch.no_grad():  # non-trivial affine parameters and running statistics
        for m in b0.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.3, 0.3)
                m.running_mean.uniform_(-0.1, 0.1)
    b0 = b0.to(cuda).train()
    b1 = copy.deepcopy(b0)
    x = (torch.randn(N, Cin, W, W) * 1.3 + 0.2).to(cuda)
    Wo = W // stride
    gy = torch.randn(N, Cout, Wo, Wo).to(cuda)
    prev = ops._BN_FOLD
    try:
        ops.set_bn_fold(True)
        # the fold must actually be taken on the stride-1 conv2 of every block
        assert ops._fold_ok(torch.empty(N, Cout, Wo, Wo, device=cuda), b0.bn2, b0.conv2)
        r1 = _run(b1, x, gy)
        ops.set_bn_fold(False)
        r0 = _run(b0, x, gy)
    finally:
        ops.set_bn_fold(prev)
    torch.cuda.synchronize()
    if W == 32:
        # 32 x 32 layers: the unfolded forward runs the patch-staged kernel, the folded one the
        # per-window kernel (different MFMA chunk order): equal within rounding
        # (a rounding difference in conv1's output can flip bn2's ReLU mask on a few elements, so
        # the gradients are compared norm-wise)
        def rel(a, b):
            return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()

        assert rel(r1[0], r0[0]) < 1e-5 and rel(r1[1], r0[1]) < 1e-4
        for k in r0[2]:
            assert rel(r1[2][k], r0[2][k]) < 1e-4, (k, rel(r1[2][k], r0[2][k]))
        for k in r0[3]:
            assert rel(r1[3][k], r0[3][k]) < 1e-5, k
        return
    assert torch.equal(r1[0], r0[0]), (r1[0] - r0[0]).abs().max().item()
    assert torch.equal(r1[1], r0[1]), (r1[1] - r0[1]).abs().max().item()
    for k in r0[2]:
        if stride == 2 and k == "conv1.weight":  # the stride-2 conv's weight gradient: float atomics
            torch.testing.assert_close(r1[2][k], r0[2][k], rtol=1e-3, atol=1e-4)
            continue
        assert torch.equal(r1[2][k], r0[2][k]), (k, (r1[2][k] - r0[2][k]).abs().max().item())
    for k in r0[3]:
        assert torch.equal(r1[3][k], r0[3][k]), k


def test_folded_block_matches_fp32_reference(cuda):
    """The folded block against the same block run by plain torch ops on the CPU."""
    from mxddp.models.pyramidnet import ResidualBlock

    torch.manual_seed(1)
    ref = ResidualBlock(21, 26, 1).train()
    dev = copy.deepcopy(ref).to(cuda).train()
    x = torch.randn(4, 21, 16, 16)
    gy = torch.randn(4, 26, 16, 16)
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)  # CPU: every mxddp op falls back to torch
    yr.backward(gy)
    prev = ops._BN_FOLD
    try:
        ops.set_bn_fold(True)
        xd = x.to(cuda).requires_grad_(True)
        yd = dev(xd)
        yd.backward(gy.to(cuda))
    finally:
        ops.set_bn_fold(prev)
    torch.testing.assert_close(yd.cpu(), yr.detach(), rtol=2e-4, atol=2e-4)
    torch.testing.assert_close(xd.grad.cpu(), xr.grad, rtol=2e-3, atol=2e-3)
    for (n, p), (_, q) in zip(dev.named_parameters(), ref.named_parameters()):
        torch.testing.assert_close(p.grad.cpu(), q.grad, rtol=2e-3, atol=2e-3, msg=n)
    for (n, b), (_, c) in zip(dev.named_buffers(), ref.named_buffers()):
        torch.testing.assert_close(b.cpu().to(c.dtype), c, rtol=1e-4, atol=1e-5, msg=n)


def test_pyramidnet_step_fold_on_off(cuda):
    """A whole PyramidNet-110 forward + backward, fold on vs off: equal up to the run-to-run
    spread of the model's float-atomic kernels (fc split-K, average-pool backward)."""
    from mxddp.models import build_model

    torch.manual_seed(0)
    m0 = build_model("pyramidnet110").to(cuda).train()
    m1 = copy.deepcopy(m0)
    x = torch.randn(8, 3, 32, 32, device=cuda)
    out = {}
    prev = ops._BN_FOLD
    try:
        for on, m in ((True, m1), (False, m0)):
            ops.set_bn_fold(on)
            y = m(x)
            y.float().square().mean().backward()
            out[on] = (y.detach(), {n: p.grad.clone() for n, p in m.named_parameters()})
    finally:
        ops.set_bn_fold(prev)
    torch.testing.assert_close(out[True][0], out[False][0], rtol=1e-4, atol=1e-4)
    for k, g in out[False][1].items():
        torch.testing.assert_close(out[True][1][k], g, rtol=2e-3, atol=2e-4, msg=k)
