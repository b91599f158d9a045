"""Model zoo: every model family of the reference plus the BASELINE extras.

| name           | reference                                   | params      |
|----------------|---------------------------------------------|-------------|
| mnist_cnn      | north star (BASELINE.json), not in the ref  | 1,199,882   |
| keras_cnn      | tensorflow2/mnist_single.py:16-26           | 93,322      |
| mlp            | chainer/train_mnist.py:13-26                | 1,796,010   |
| pyramidnet110  | pytorch/model.py:53-118                     | 24,253,410  |
| resnet50       | BASELINE.json config 5, not in the ref      | 25,557,032  |
"""
from __future__ import annotations

from dataclasses import dataclass

import torch.nn as nn

from .keras_cnn import KerasCNN
from .mlp import MLP
from .mnist_cnn import MnistCNN
from .pyramidnet import PyramidNet, pyramidnet
from .resnet import ResNet, resnet50


@dataclass(frozen=True)
class ModelSpec:
    name: str
    factory: type | object
    input_shape: tuple
    num_classes: int
    dataset: str          # natural dataset family: mnist | cifar10 | imagenet
    optimizer: str        # reference optimizer: sgd | adam
    lr: float
    momentum: float
    weight_decay: float


MODELS = {
    "mnist_cnn": ModelSpec("mnist_cnn", MnistCNN, (1, 28, 28), 10, "mnist", "sgd", 0.1, 0.9, 1e-4),
    "keras_cnn": ModelSpec("keras_cnn", KerasCNN, (1, 28, 28), 10, "mnist", "adam", 1e-3, 0.0, 0.0),
    "mlp": ModelSpec("mlp", MLP, (1, 28, 28), 10, "mnist", "adam", 1e-3, 0.0, 0.0),
    "pyramidnet110": ModelSpec("pyramidnet110", pyramidnet, (3, 32, 32), 10, "cifar10", "sgd", 0.1, 0.9, 1e-4),
    "resnet50": ModelSpec("resnet50", resnet50, (3, 224, 224), 1000, "imagenet", "sgd", 0.1, 0.9, 1e-4),
}


def get_spec(name: str) -> ModelSpec:
    try:
        return MODELS[name]
    except KeyError:
        raise ValueError(f"unknown model {name!r}; choose from {sorted(MODELS)}") from None


def build_model(name: str, **kwargs) -> nn.Module:
    return get_spec(name).factory(**kwargs)


__all__ = ["MODELS", "ModelSpec", "get_spec", "build_model", "MnistCNN", "KerasCNN", "MLP", "PyramidNet",
           "pyramidnet", "ResNet", "resnet50"]
