"""nn.Module layers whose forward runs the mxddp HIP kernels.

Each layer subclasses the matching ``torch.nn`` module, so parameter / buffer names,
shapes, default initialisation and therefore ``state_dict`` keys are identical to the
reference's torch.nn models (checkpoint compatibility).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops


class Conv2d(nn.Conv2d):
    def __init__(self, *a, fuse_relu: bool = False, **k):
        super().__init__(*a, **k)
        self.fuse_relu = fuse_relu

    def forward(self, x):
        if self.groups != 1 or self.padding_mode != "zeros" or isinstance(self.padding, str):
            raise NotImplementedError("mxddp Conv2d: groups=1, zero padding only")
        return ops.conv2d(x, self.weight, self.bias, self.stride, self.padding, self.dilation, relu=self.fuse_relu)


class Linear(nn.Linear):
    def __init__(self, *a, fuse_relu: bool = False, **k):
        super().__init__(*a, **k)
        self.fuse_relu = fuse_relu

    def forward(self, x):
        return ops.linear(x, self.weight, self.bias, relu=self.fuse_relu)


class ReLU(nn.ReLU):
    def forward(self, x):
        return ops.relu(x)


class MaxPool2d(nn.MaxPool2d):
    def forward(self, x):
        return ops.max_pool2d(x, self.kernel_size, self.stride, self.padding, self.ceil_mode)


class AvgPool2d(nn.AvgPool2d):
    def forward(self, x):
        if not self.count_include_pad or self.divisor_override is not None:
            raise NotImplementedError("mxddp AvgPool2d: count_include_pad=True only")
        return ops.avg_pool2d(x, self.kernel_size, self.stride, self.padding, self.ceil_mode)


class BatchNorm2d(nn.BatchNorm2d):
    def __init__(self, *a, fuse_relu: bool = False, **k):
        super().__init__(*a, **k)
        self.fuse_relu = fuse_relu

    def forward(self, x, residual=None, tap=False):
        """``residual`` / ``tap``: the PyramidNet shortcut fusions of ops.batch_norm."""
        training = self.training or not self.track_running_stats
        nbt = self.num_batches_tracked if (self.training and self.track_running_stats) else None
        mom = self.momentum if self.momentum is not None else 0.1
        return ops.batch_norm(x, self.weight, self.bias,
                              self.running_mean if self.track_running_stats else None,
                              self.running_var if self.track_running_stats else None,
                              training, mom, self.eps, relu=self.fuse_relu, num_batches=nbt,
                              residual=residual, tap=tap)


def count_params(model: nn.Module) -> int:
    return sum(p.numel() for p in model.parameters() if p.requires_grad)


@torch.no_grad()
def keras_init_(model: nn.Module) -> None:
    """Keras defaults: glorot_uniform kernels, zero biases (tensorflow2/mnist_single.py:16-26)."""
    for m in model.modules():
        if isinstance(m, (nn.Conv2d, nn.Linear)):
            nn.init.xavier_uniform_(m.weight)
            if m.bias is not None:
                nn.init.zeros_(m.bias)


@torch.no_grad()
def chainer_init_(model: nn.Module) -> None:
    """Chainer L.Linear defaults: LeCunNormal(scale=1) weights, zero bias (chainer/train_mnist.py:19-21)."""
    for m in model.modules():
        if isinstance(m, nn.Linear):
            fan_in = m.weight.shape[1]
            m.weight.normal_(0.0, (1.0 / fan_in) ** 0.5)
            if m.bias is not None:
                m.bias.zero_()
