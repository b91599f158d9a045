"""Python face of the native fused Keras-CNN training step (``mxddp._C.KerasEngine``).

The reference trains its TF2 Keras CNN (tensorflow2/mnist_single.py:16-26) with Keras Adam
(:78) on one device, under MirroredStrategy (tensorflow2/mnist_mirror_strategy.py:12,68-79) and
under MultiWorkerMirroredStrategy.  ``FusedKerasTrainer.step()`` runs one such training step as
four fused gfx950 kernels (csrc/keras_kernels.hip) -- on-device batch, forward, backward,
finalize + Adam -- plus the gradient all-reduce when there are replicas / ranks, captured in
hipGraphs so a step is one graph launch.  Loss and accuracy accumulate on the device.  The DDP
launch strategy (transport, RCCL communicator variant, eager or graph) is timed per machine by
``autotune()`` (fused.py), as for the MNIST engine.

Parameters are one flat fp32 buffer in KerasCNN ``state_dict`` order, so ``state_dict()`` is
key-for-key the layer model's (``models.KerasCNN``) and checkpoints are interchangeable.
"""
from __future__ import annotations

import torch

from . import native
from .fused import AdamTrainerBase, FusedReplicas
from .models.keras_cnn import KerasCNN

_LAYOUT = [  # (name, shape) in state_dict order == flat offsets of KerasLayout (keras_kernels.h)
    ("conv1.weight", (32, 1, 3, 3)), ("conv1.bias", (32,)),
    ("conv2.weight", (64, 32, 3, 3)), ("conv2.bias", (64,)),
    ("conv3.weight", (64, 64, 3, 3)), ("conv3.bias", (64,)),
    ("fc1.weight", (64, 576)), ("fc1.bias", (64,)),
    ("fc2.weight", (10, 64)), ("fc2.bias", (10,)),
]


class FusedKerasTrainer(AdamTrainerBase):
    """The fused Keras-CNN step.  DDP (world size > 1, or collectives forced): finalize into g,
    ONE all-reduce of the 373 KB gradient, Adam -- over RCCL (any comm.py variant) or the xGMI
    peer transport, eager launches or one hipGraph per group of steps, picked by autotune().
    With the peer transport the exchange can also run inside the Adam launch ("co": one-shot
    push of every rank's gradient, per-block flags, rank-ordered sum, Adam; one launch fewer)."""
    LAYOUT = _LAYOUT
    MODEL = KerasCNN
    STRATEGIES = ("one",)

    def _candidate_strategies(self, transport: str) -> list:
        return ["one"] + (["co"] if transport == "peer" else [])

    def _set_buckets(self, strat: str):
        """one: a separate all-reduce of the whole gradient between the finalize and Adam; co
        (peer transport): the exchange co-scheduled with Adam in one launch."""
        co = strat == "co" and self.eng.set_coscheduled(True)
        if not co:
            self.eng.set_coscheduled(False)
        self.bucket_strategy = "co" if co else "one"

    def __init__(self, batch: int = 64, device: torch.device | int = 0, comm=None, seed: int = 1, lr: float = 1e-3,
                 betas=(0.9, 0.999), eps: float = 1e-7, weight_decay: float = 0.0, eps_hat: bool = True,
                 use_graph: bool = True, init_model: KerasCNN | None = None, steps_per_graph: int | None = None,
                 peer=None, force_collectives: bool = False, graph_mode: int | None = None, transport: str = "auto",
                 rccl_variants=None):
        C = native()
        if batch % 8:
            raise ValueError("FusedKerasTrainer: batch must be a multiple of 8")
        n = self._init_flat(batch, device, comm, seed, init_model)
        assert n == C.KERAS_NUM_PARAMS
        self._init_adam(n, lr)
        wsb = C.keras_workspace_bytes(batch)
        self.workspace = torch.zeros(wsb // 4 + 64, dtype=torch.float32, device=self.device)
        torch.cuda.synchronize(self.device)
        self.eng = C.KerasEngine(batch, self.params.data_ptr(), self.grads.data_ptr(), self.m.data_ptr(),
                                 self.v.data_ptr(), self.adam_state.data_ptr(), self.workspace.data_ptr(), wsb, comm,
                                 seed, self.lr.data_ptr(), self.metrics.data_ptr(), float(betas[0]), float(betas[1]),
                                 float(eps), float(weight_decay), bool(eps_hat))
        self._init_runtime(comm, peer, transport, force_collectives, rccl_variants, use_graph, graph_mode,
                           steps_per_graph)
        self.bucket_strategy = "one"

    def _after_param_load(self):
        self.eng.repack()  # conv2 weights live pre-packed in MFMA fragment order


class FusedKerasReplicas(FusedReplicas):
    """In-process replica data parallelism (MirroredStrategy, tensorflow2/mnist_mirror_strategy.py:12)
    for the Keras CNN on the fused engine: one FusedKerasTrainer per device, the global batch split
    across them, gradients averaged by the peer transport opened in-process (device peer access),
    so every replica's step -- forward, backward, all-reduce, Adam -- is one graph launch and the
    replicas synchronise on the GPUs.  All replicas' work is launched before the host waits."""

    def __init__(self, devices, batch: int = 64, lr: float = 1e-3, seed: int = 1, init_model=None,
                 use_graph: bool = True, steps_per_graph: int | None = None, blocks: int = 32,
                 strategy: str = "co"):
        if init_model is None:
            torch.manual_seed(seed)
            init_model = KerasCNN()
        self.batch = batch
        n = len(devices)
        if strategy == "co" and n > 2 and len({torch.device(d) for d in devices}) < n:
            # replicas sharing one GPU (a rehearsal of an n-GPU node): the co-scheduled exchange is
            # n x 182 blocks of 512 threads that must ALL be resident at once (each block waits on
            # the peers' matching block), more than one GPU holds at n = 8 -- the separate
            # exchange kernel (32 blocks per replica) is used instead
            strategy = "one"

        def make(d, pc):
            t = FusedKerasTrainer(batch=batch, device=d, peer=pc, seed=seed, lr=lr, init_model=init_model,
                                  use_graph=use_graph, steps_per_graph=steps_per_graph, graph_mode=1)
            if pc is not None:
                t._set_buckets(strategy)  # "co": exchange inside the Adam launch; "one": separate
            return t

        super().__init__(devices, make, blocks=blocks, peer_bytes=4 << 20)
