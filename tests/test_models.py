"""T0: model topology golden values on the CPU path."""
import pytest
import torch

from mxddp.models import MODELS, build_model
from mxddp.models.layers import count_params
from mxddp.models.pyramidnet import channel_schedule

GOLDEN_PARAMS = {
    "mnist_cnn": 1_199_882,
    "keras_cnn": 93_322,
    "mlp": 1_796_010,
    "pyramidnet110": 24_253_410,
    "resnet50": 25_557_032,
}


@pytest.mark.parametrize("name", sorted(GOLDEN_PARAMS))
def test_param_counts(name):
    assert count_params(build_model(name)) == GOLDEN_PARAMS[name]


def test_pyramidnet_state_dict_layout():
    sd = build_model("pyramidnet110").state_dict()
    keys = list(sd)
    assert len(keys) == 880
    assert keys[:4] == ["conv1.weight", "bn1.weight", "bn1.bias", "bn1.running_mean"]
    assert keys[-3:] == ["bn_out.num_batches_tracked", "fc_out.weight", "fc_out.bias"]
    assert sum(1 for k in keys if k.endswith("num_batches_tracked")) == 155  # 155 BN layers
    assert sum(1 for k in keys if k.endswith("conv1.weight") or k.endswith("conv2.weight")) == 103


def test_pyramidnet_channel_schedule():
    sched, out = channel_schedule()
    assert len(sched) == 51 and out == 271
    assert sched[0] == (16, 21, 1)
    assert sched[17][2] == 2 and sched[17][0] == 101 and sched[17][1] == 106  # stage-2 entry
    assert sched[34][2] == 2 and sched[34][0] == 186 and sched[34][1] == 191  # stage-3 entry
    assert len({(a, b) for a, b, _ in sched}) == 51


@pytest.mark.parametrize("name,shape", [("mnist_cnn", (2, 1, 28, 28)), ("keras_cnn", (2, 1, 28, 28)),
                                        ("mlp", (2, 1, 28, 28)), ("pyramidnet110", (2, 3, 32, 32))])
def test_forward_backward_cpu(name, shape):
    m = build_model(name)
    x = torch.randn(shape)
    out = m(x)
    assert out.shape == (2, 10)
    out.sum().backward()
    assert all(p.grad is not None for p in m.parameters())


def test_resnet50_forward_small():
    m = build_model("resnet50")
    out = m(torch.randn(1, 3, 64, 64))
    assert out.shape == (1, 1000)


def test_state_dict_loads_into_plain_torch_module():
    """Checkpoint compatibility: our MnistCNN state_dict loads into a torch.nn reference net."""
    import torch.nn as nn

    class Ref(nn.Module):
        def __init__(self):
            super().__init__()
            self.conv1 = nn.Conv2d(1, 32, 3, 1)
            self.conv2 = nn.Conv2d(32, 64, 3, 1)
            self.fc1 = nn.Linear(9216, 128)
            self.fc2 = nn.Linear(128, 10)

    ref = Ref()
    ref.load_state_dict(build_model("mnist_cnn").state_dict(), strict=True)


def test_registry_specs():
    assert set(MODELS) == set(GOLDEN_PARAMS)
    assert MODELS["keras_cnn"].optimizer == "adam" and MODELS["pyramidnet110"].optimizer == "sgd"


@pytest.mark.parametrize("stride", [1, 2])
def test_pyramidnet_block_matches_reference_formula(stride):
    """ResidualBlock (the shortcut fused into the BNs on stride 1) computes the reference block
    (pytorch/model.py:40-50): bn1 -> conv(s) -> bn2 -> ReLU -> conv -> bn3, + pad/pool shortcut."""
    import torch.nn.functional as F

    from mxddp.models.pyramidnet import ResidualBlock

    torch.manual_seed(3)
    blk = ResidualBlock(6, 11, stride)
    x = torch.randn(3, 6, 8, 8, requires_grad=True)
    out = blk(x)

    def bn(m, t):
        return F.batch_norm(t, None, None, m.weight, m.bias, True, 0.1, m.eps)

    xr = x.detach().clone().requires_grad_()
    h = bn(blk.bn3, blk.conv2(F.relu(bn(blk.bn2, F.conv2d(bn(blk.bn1, xr), blk.conv1.weight, None, stride, 1)))))
    sc = F.pad(xr, (0, 0, 0, 0, 0, 5))
    if stride == 2:
        sc = F.avg_pool2d(sc, 2, 2, ceil_mode=True)
    ref = h + sc
    assert torch.allclose(out, ref, atol=1e-5)
    g = torch.randn_like(ref)
    out.backward(g)
    ref.backward(g)
    assert torch.allclose(x.grad, xr.grad, atol=1e-5)


def test_resnet_stock_baseline_never_takes_the_native_nhwc_path(monkeypatch):
    """bench.py --impl torch (the stock PyTorch-ROCm baseline) runs under ops.torch_reference_mode
    with the compute dtype set to bf16: ResNet must then take its torch-op path, not mxddp's NHWC
    kernels (which made the round-3/4 "stock" ResNet-50 numbers mxddp's own)."""
    from types import SimpleNamespace

    from mxddp import ops
    from mxddp.models import resnet as R

    monkeypatch.setattr(ops, "compute_dtype", lambda: "bf16")
    x = SimpleNamespace(is_cuda=True)
    assert R._nhwc_mode(x)
    with ops.torch_reference_mode():
        assert not R._nhwc_mode(x)
    assert R._nhwc_mode(x)


def test_bn_conv_cpu_fallback_and_input_affine():
    """ops.bn_conv off the GPU is the plain conv(bn(x)) chain (tap included), and ops.conv2d's
    in_ss (a folded BN's per-channel scale / shift, fused ReLU) matches applying it first."""
    import copy

    import torch
    import torch.nn.functional as F

    from mxddp import ops
    from mxddp.models.pyramidnet import ResidualBlock

    torch.manual_seed(0)
    blk = ResidualBlock(16, 21, 1).train()
    ref = copy.deepcopy(blk)
    x = torch.randn(2, 16, 8, 8)
    y, xs = ops.bn_conv(x, blk.bn1, blk.conv1, tap=True)
    y_ref = ref.conv1(ref.bn1(x))
    assert torch.equal(y, y_ref) and torch.equal(xs, x)
    w = torch.randn(5, 16, 3, 3)
    ss = torch.stack([torch.rand(16) + 0.5, torch.randn(16) * 0.1], dim=1)
    for relu in (False, True):
        h = x * ss[:, 0].view(1, -1, 1, 1) + ss[:, 1].view(1, -1, 1, 1)
        h = F.relu(h) if relu else h
        torch.testing.assert_close(ops.conv2d(x, w, None, 1, 1, in_ss=ss, in_relu=relu), F.conv2d(h, w, None, 1, 1))
