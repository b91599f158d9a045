"""Reference Chainer MLP (chainer/train_mnist.py:13-26): 784 -> 1000 -> 1000 -> 10, ReLU.

1,796,010 parameters with ``n_units=1000``; wrapped by L.Classifier (softmax CE +
accuracy) in the reference, which is ``mxddp.ops.cross_entropy(..., return_correct=True)``
here.  Chainer LeCunNormal / zero init.  Parameter names l1, l2, l3 as in Chainer.
"""
from __future__ import annotations

import torch.nn as nn

from .layers import Linear, chainer_init_


class MLP(nn.Module):
    input_shape = (1, 28, 28)
    num_classes = 10

    def __init__(self, n_units: int = 1000, n_out: int = 10, n_in: int = 784):
        super().__init__()
        self.l1 = Linear(n_in, n_units, fuse_relu=True)
        self.l2 = Linear(n_units, n_units, fuse_relu=True)
        self.l3 = Linear(n_units, n_out)
        chainer_init_(self)

    def forward(self, x):
        return self.l3(self.l2(self.l1(x.flatten(1))))
