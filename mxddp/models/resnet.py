"""ResNet-50 (BASELINE.json config 5 only: not in the reference).  torchvision-style
topology and parameter names (conv1/bn1/layer1..4/fc, Bottleneck with downsample.0/.1),
25,557,032 parameters, on mxddp kernels.  ReLU is fused into the BN that precedes it.

Two execution paths over the same parameters (identical ``state_dict``):

* NCHW fp32 (CPU, and GPU at compute dtype fp32): ``mxddp.ops`` layer kernels;
* channels-last bf16 (GPU at compute dtype bf16, the config-5 benchmark): activations bf16
  NHWC end to end (``mxddp.ops.nhwc``), vectorized implicit-GEMM MFMA convolutions, BN with the
  Bottleneck's residual add + ReLU fused into its apply kernel, fp32 master weights / grads.
"""
from __future__ import annotations

import torch.nn as nn

from .. import ops
from .layers import BatchNorm2d, Conv2d, Linear, MaxPool2d


def _nhwc_mode(x) -> bool:
    # not under ops.torch_reference_mode (bench.py --impl torch): the stock baseline must run
    # PyTorch's own kernels end to end, never mxddp's NHWC ones
    return x.is_cuda and ops.compute_dtype() == "bf16" and not ops.torch_reference_active()


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: nn.Module | None = None):
        super().__init__()
        self.conv1 = Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = BatchNorm2d(planes, fuse_relu=True)
        self.conv2 = Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = BatchNorm2d(planes, fuse_relu=True)
        self.conv3 = Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        out = self.bn3(self.conv3(self.bn2(self.conv2(self.bn1(self.conv1(x))))))
        return ops.relu(out + idt)

    def convs(self):
        c = [self.conv1, self.conv2, self.conv3]
        return c + ([self.downsample[0]] if self.downsample is not None else [])

    def forward_nhwc(self, x, pack=None):
        from ..ops import nhwc as N

        # the shortcut's input gradient is added inside conv1's data-gradient epilogue: the
        # identity gradient left by bn3's backward, or the projection conv's data gradient.  The
        # projection branch is built AFTER the main branch so its backward nodes carry the higher
        # sequence numbers and autograd runs them first (its dx exists when conv1's dgrad runs).
        join = N.GradJoin()
        x, xs = N.fork(x, join)
        # bn=: each conv's epilogue computes its BN's partial statistics where its kernel allows
        out = N.batch_norm(N.conv2d(x, self.conv1.weight, pack=pack, join=join, bn=self.bn1), self.bn1, relu=True)
        out = N.batch_norm(N.conv2d(out, self.conv2.weight, self.conv2.stride, self.conv2.padding, pack, bn=self.bn2),
                           self.bn2, relu=True)
        out = N.conv2d(out, self.conv3.weight, pack=pack, bn=self.bn3)
        if self.downsample is None:
            return N.batch_norm(out, self.bn3, relu=True, res=xs, join=join)
        dc, dbn = self.downsample[0], self.downsample[1]
        idt = N.batch_norm(N.conv2d(xs, dc.weight, dc.stride, dc.padding, pack, deposit=join, bn=dbn), dbn)
        return N.batch_norm(out, self.bn3, relu=True, res=idt)


class ResNet(nn.Module):
    input_shape = (3, 224, 224)

    def __init__(self, layers=(3, 4, 6, 3), num_classes: int = 1000):
        super().__init__()
        self.num_classes = num_classes
        self.inplanes = 64
        self.conv1 = Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = BatchNorm2d(64, fuse_relu=True)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = MaxPool2d(3, 2, 1)
        self.layer1 = self._make(64, layers[0], 1)
        self.layer2 = self._make(128, layers[1], 2)
        self.layer3 = self._make(256, layers[2], 2)
        self.layer4 = self._make(512, layers[3], 2)
        self.fc = Linear(512 * 4, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _make(self, planes, blocks, stride):
        down = None
        if stride != 1 or self.inplanes != planes * 4:
            down = nn.Sequential(Conv2d(self.inplanes, planes * 4, 1, stride, bias=False), BatchNorm2d(planes * 4))
        layers = [Bottleneck(self.inplanes, planes, stride, down)]
        self.inplanes = planes * 4
        layers += [Bottleneck(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x):
        if _nhwc_mode(x):
            return self.forward_nhwc(x)
        x = self.maxpool(self.bn1(self.conv1(x)))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = ops.avg_pool2d(x, (x.shape[2], x.shape[3]))
        return self.fc(x.flatten(1))


    def _weight_pack(self):
        """All 53 conv weights repacked to bf16 in one launch per forward (mxddp.ops.nhwc.WeightPack);
        the pack is rebuilt only when a weight's storage or the grad mode changes."""
        import torch

        from ..ops import nhwc as N

        grad = torch.is_grad_enabled()
        specs = [(self.conv1.weight, 8, False)]
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            for blk in layer:
                specs += [(c.weight, c.weight.shape[1], grad) for c in blk.convs()]
        pack = getattr(self, "_nhwc_pack", None)
        if pack is None or not pack.matches(specs):
            pack = N.WeightPack(specs)
            self._nhwc_pack = pack
        pack.refresh()
        return pack

    def forward_nhwc(self, x):
        from ..ops import nhwc as N

        pack = self._weight_pack()
        y = N.to_nhwc(x)
        # the stem kernel's epilogue computes bn1's statistics (csrc/nhwc_bf16.hip conv_nhwc_stem_kernel)
        y = N.conv2d(y, self.conv1.weight, self.conv1.stride, self.conv1.padding, pack, bn=self.bn1)
        y = N.batch_norm(y, self.bn1, relu=True)
        y = N.max_pool2d(y, 3, 2, 1)
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            for blk in layer:
                y = blk.forward_nhwc(y, pack)
        return self.fc(N.global_avg_pool(y))


def resnet50(num_classes: int = 1000) -> ResNet:
    return ResNet((3, 4, 6, 3), num_classes)
