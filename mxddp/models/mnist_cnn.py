"""North-star MNIST CNN (BASELINE.json "MNIST CNN DDP").

conv(1->32,3)+ReLU -> conv(32->64,3)+ReLU -> maxpool2 -> flatten(9216) -> fc(9216->128)+ReLU
-> fc(128->10); the loss is log_softmax + NLL, fused (``mxddp.ops.cross_entropy``).
1,199,882 parameters.  This module is the layer-by-layer path; the fully fused native
training step for the same parameters is ``mxddp.engine.FusedMnistTrainer``.
"""
from __future__ import annotations

import torch.nn as nn

from .. import ops
from .layers import Conv2d, Linear


class MnistCNN(nn.Module):
    input_shape = (1, 28, 28)
    num_classes = 10

    def __init__(self):
        super().__init__()
        self.conv1 = Conv2d(1, 32, 3, 1, fuse_relu=True)
        self.conv2 = Conv2d(32, 64, 3, 1, fuse_relu=True)
        self.fc1 = Linear(9216, 128, fuse_relu=True)
        self.fc2 = Linear(128, 10)

    def forward(self, x):
        x = self.conv2(self.conv1(x))
        x = ops.max_pool2d(x, 2)
        x = self.fc1(x.flatten(1))
        return self.fc2(x)  # logits; log_softmax is fused into the loss
