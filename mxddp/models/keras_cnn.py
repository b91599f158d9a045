"""Reference TF2 Keras CNN (tensorflow2/mnist_single.py:16-26), 93,322 parameters.

Conv2D(32,3,relu) -> MaxPool2 -> Conv2D(64,3,relu) -> MaxPool2 -> Conv2D(64,3,relu) ->
Flatten -> Dense(64,relu) -> Dense(10,softmax).  Valid padding, biases on, Keras
glorot-uniform / zero init.  The softmax is fused into the sparse-categorical CE loss
(same math, better numerics); ``predict`` applies it explicitly.  Layout is NCHW, so the
Flatten order is (c,h,w) rather than Keras' (h,w,c): a fixed permutation of fc1's inputs.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .layers import Conv2d, Linear, keras_init_


class KerasCNN(nn.Module):
    input_shape = (1, 28, 28)
    num_classes = 10

    def __init__(self):
        super().__init__()
        self.conv1 = Conv2d(1, 32, 3, fuse_relu=True)
        self.conv2 = Conv2d(32, 64, 3, fuse_relu=True)
        self.conv3 = Conv2d(64, 64, 3, fuse_relu=True)
        self.fc1 = Linear(576, 64, fuse_relu=True)
        self.fc2 = Linear(64, 10)
        keras_init_(self)

    def forward(self, x):
        x = ops.max_pool2d(self.conv1(x), 2)
        x = ops.max_pool2d(self.conv2(x), 2)
        x = self.conv3(x)
        return self.fc2(self.fc1(x.flatten(1)))

    @torch.no_grad()
    def predict(self, x):
        return torch.softmax(self.forward(x), dim=1)
