"""Python face of the native fused Chainer-MLP training step (``mxddp._C.MlpEngine``).

The reference trains ``MLP(1000, 10)`` (chainer/train_mnist.py:13-26) with Chainer Adam (:69)
on one device, and with ``ParallelUpdater`` over several GPUs of one process
(chainer/train_mnist_gpu.py:87-93).  ``FusedMlpTrainer.step()`` runs one such training step as
five fused gfx950 launches (csrc/mlp_kernels.hip: l1 / l2 forward, head, l2 + l3 backward with
Adam folded in, l1 backward with Adam folded in) -- or, with gradient collectives, the two
gradient buckets all-reduced over RCCL / the xGMI peer transport and the flat Adam -- captured
in hipGraphs so a step is one graph launch.  ``FusedMlpReplicas`` is the ParallelUpdater.

Parameters are one flat fp32 buffer in ``models.MLP`` ``state_dict`` order (l1, l2, l3), so
checkpoints are interchangeable with the layer model's.
"""
from __future__ import annotations

import torch

from . import native
from .fused import AdamTrainerBase, FusedReplicas
from .models.mlp import MLP

_LAYOUT = [  # (name, shape) in state_dict order == flat offsets of MlpLayout (mlp_kernels.h)
    ("l1.weight", (1000, 784)), ("l1.bias", (1000,)),
    ("l2.weight", (1000, 1000)), ("l2.bias", (1000,)),
    ("l3.weight", (10, 1000)), ("l3.bias", (10,)),
]


class FusedMlpTrainer(AdamTrainerBase):
    LAYOUT = _LAYOUT
    MODEL = MLP

    def __init__(self, batch: int = 64, device: torch.device | int = 0, comm=None, seed: int = 1, lr: float = 1e-3,
                 betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0, eps_hat: bool = True,
                 use_graph: bool = True, init_model: MLP | None = None, steps_per_graph: int | None = None,
                 graph_mode: int | None = None, peer=None, force_collectives: bool = False, transport: str = "auto",
                 rccl_variants=None):
        C = native()
        if not 1 <= batch <= C.MLP_MAX_BATCH:
            raise ValueError(f"FusedMlpTrainer: batch must be in [1, {C.MLP_MAX_BATCH}]")
        if init_model is not None and tuple(init_model.l1.weight.shape) != (1000, 784):
            raise ValueError("FusedMlpTrainer: the native step is built for the reference's 1000 units")
        n = self._init_flat(batch, device, comm, seed, init_model)
        assert n == C.MLP_NUM_PARAMS
        self._init_adam(n, lr)
        wsb = C.mlp_workspace_bytes(batch)
        self.workspace = torch.zeros(wsb // 4 + 64, dtype=torch.float32, device=self.device)
        torch.cuda.synchronize(self.device)
        self.eng = C.MlpEngine(batch, self.params.data_ptr(), self.grads.data_ptr(), self.m.data_ptr(),
                               self.v.data_ptr(), self.adam_state.data_ptr(), self.workspace.data_ptr(), wsb, comm,
                               seed, self.lr.data_ptr(), self.metrics.data_ptr(), float(betas[0]), float(betas[1]),
                               float(eps), float(weight_decay), bool(eps_hat))
        self._init_runtime(comm, peer, transport, force_collectives, rccl_variants, use_graph, graph_mode,
                           steps_per_graph)


class FusedMlpReplicas(FusedReplicas):
    """ParallelUpdater parity (chainer/train_mnist_gpu.py:87-93): one FusedMlpTrainer per device,
    the global batch split across them, gradients averaged over the in-process peer transport."""

    def __init__(self, devices, batch: int = 64, lr: float = 1e-3, seed: int = 1, init_model=None,
                 use_graph: bool = True, steps_per_graph: int | None = None, blocks: int = 32):
        if init_model is None:
            torch.manual_seed(seed)
            init_model = MLP()
        self.batch = batch
        super().__init__(devices, lambda d, pc: FusedMlpTrainer(batch=batch, device=d, peer=pc, seed=seed, lr=lr,
                                                                init_model=init_model, use_graph=use_graph,
                                                                steps_per_graph=steps_per_graph, graph_mode=1),
                         blocks=blocks)
