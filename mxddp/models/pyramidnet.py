"""PyramidNet-110 (alpha=270) for CIFAR-10: the reference's PyTorch model
(pytorch/model.py:6-118, factory ``pyramidnet()`` at :115-118).

Additive widening: the channel count grows by alpha / (3 * 18) = 5.0 per residual block
from 16 to 271 over three stages of 17 blocks (``range(num_layers - 1)``, model.py:89).
Block = BN -> conv3x3(stride) -> BN -> ReLU -> conv3x3 -> BN, plus a parameter-free
shortcut that zero-pads channels and 2x2-avg-pools (ceil) on stride 2 (model.py:17-21).
No ReLU after the residual add.  Module / parameter names match the reference exactly,
so ``state_dict`` has the same 880 keys (24,253,410 parameters) and checkpoints are
interchangeable.  In the mxddp version the BN->ReLU pair is one kernel, the identity
shortcut (stride 1) is fused into bn3's normalise pass and bn1's backward, and the stride-2
pad+pool+add shortcut is one kernel.
"""
from __future__ import annotations

import torch.nn as nn

from .. import ops
from .layers import AvgPool2d, BatchNorm2d, Conv2d, Linear


class IdentityPadding(nn.Module):
    """Parameter-free shortcut descriptor; the add itself is fused (ops.shortcut_pad_add)."""

    def __init__(self, in_channels: int, out_channels: int, stride: int = 1):
        super().__init__()
        self.pooling = AvgPool2d(2, 2, ceil_mode=True) if stride == 2 else None
        self.add_channels = out_channels - in_channels
        self.stride = stride


class ResidualBlock(nn.Module):
    def __init__(self, in_channels: int, out_channels: int, stride: int = 1):
        super().__init__()
        self.bn1 = BatchNorm2d(in_channels)
        self.conv1 = Conv2d(in_channels, out_channels, 3, stride, 1, bias=False)
        self.bn2 = BatchNorm2d(out_channels, fuse_relu=True)
        self.conv2 = Conv2d(out_channels, out_channels, 3, 1, 1, bias=False)
        self.bn3 = BatchNorm2d(out_channels)
        self.relu = nn.ReLU(inplace=True)  # fused into bn2; kept for module-tree parity
        self.down_sample = IdentityPadding(in_channels, out_channels, stride)
        self.stride = stride

    def forward(self, x):
        # bn1 -> conv1 and bn2 -> ReLU -> conv2 with the BN normalise pass folded into the
        # convolution's input staging where it runs the Winograd path (ops.bn_conv; the stride-2
        # conv1 keeps its BN pass)
        if self.stride == 1:
            # identity shortcut fused into the BNs: bn3 adds x (zero-padded channels) while it
            # normalises, and bn1's backward adds the shortcut's gradient to its dx
            h, xs = ops.bn_conv(x, self.bn1, self.conv1, tap=True)
            return self.bn3(ops.bn_conv(h, self.bn2, self.conv2), residual=xs)
        out = self.bn3(ops.bn_conv(self.conv1(self.bn1(x)), self.bn2, self.conv2))
        return ops.shortcut_pad_add(out, x, self.stride)


def channel_schedule(num_layers: int = 18, alpha: float = 270.0, start: int = 16):
    """[(in, out, stride)] for every block, reproducing the reference's float accumulation."""
    addrate = alpha / (3 * num_layers * 1.0)
    cin = float(start)
    sched = []
    for stage_stride in (1, 2, 2):
        stride = stage_stride
        for _ in range(num_layers - 1):
            cout = cin + addrate
            sched.append((int(round(cin)), int(round(cout)), stride))
            cin = cout
            stride = 1
    return sched, int(round(cin))


class PyramidNet(nn.Module):
    input_shape = (3, 32, 32)
    num_classes = 10

    def __init__(self, num_layers: int = 18, alpha: float = 270.0, num_classes: int = 10):
        super().__init__()
        self.num_layers = num_layers
        self.addrate = alpha / (3 * num_layers * 1.0)
        self.conv1 = Conv2d(3, 16, 3, 1, 1, bias=False)
        self.bn1 = BatchNorm2d(16)
        sched, self.out_channels = channel_schedule(num_layers, alpha)
        per = num_layers - 1
        self.layer1 = nn.Sequential(*[ResidualBlock(*s) for s in sched[:per]])
        self.layer2 = nn.Sequential(*[ResidualBlock(*s) for s in sched[per:2 * per]])
        self.layer3 = nn.Sequential(*[ResidualBlock(*s) for s in sched[2 * per:]])
        self.bn_out = BatchNorm2d(self.out_channels, fuse_relu=True)
        self.relu_out = nn.ReLU(inplace=True)  # fused into bn_out
        self.avgpool = AvgPool2d(8, stride=1)
        self.fc_out = Linear(self.out_channels, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def forward(self, x):
        x = self.bn1(self.conv1(x))
        x = self.layer3(self.layer2(self.layer1(x)))
        x = self.avgpool(self.bn_out(x))
        return self.fc_out(x.flatten(1))


def pyramidnet(num_classes: int = 10) -> PyramidNet:
    return PyramidNet(num_layers=18, alpha=270, num_classes=num_classes)
