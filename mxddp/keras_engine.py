"""Python face of the native fused Keras-CNN training step (``mxddp._C.KerasEngine``).

The reference trains its TF2 Keras CNN (tensorflow2/mnist_single.py:16-26) with Keras Adam
(:78) on one device, under MirroredStrategy (tensorflow2/mnist_mirror_strategy.py:12,68-79) and
under MultiWorkerMirroredStrategy.  ``FusedKerasTrainer.step()`` runs one such training step as
four fused gfx950 kernels (csrc/keras_kernels.hip) -- on-device batch, forward, backward,
finalize + Adam -- plus the gradient all-reduce when there are replicas / ranks, captured in
hipGraphs so a step is one graph launch.  Loss and accuracy accumulate on the device.

Parameters are one flat fp32 buffer in KerasCNN ``state_dict`` order, so ``state_dict()`` is
key-for-key the layer model's (``models.KerasCNN``) and checkpoints are interchangeable.
"""
from __future__ import annotations

import os

import torch

from . import native
from .models.keras_cnn import KerasCNN

_LAYOUT = [  # (name, shape) in state_dict order == flat offsets of KerasLayout (keras_kernels.h)
    ("conv1.weight", (32, 1, 3, 3)), ("conv1.bias", (32,)),
    ("conv2.weight", (64, 32, 3, 3)), ("conv2.bias", (64,)),
    ("conv3.weight", (64, 64, 3, 3)), ("conv3.bias", (64,)),
    ("fc1.weight", (64, 576)), ("fc1.bias", (64,)),
    ("fc2.weight", (10, 64)), ("fc2.bias", (10,)),
]


class FusedKerasTrainer:
    def __init__(self, batch: int = 64, device: torch.device | int = 0, comm=None, seed: int = 1, lr: float = 1e-3,
                 betas=(0.9, 0.999), eps: float = 1e-7, weight_decay: float = 0.0, eps_hat: bool = True,
                 use_graph: bool = True, init_model: KerasCNN | None = None, steps_per_graph: int | None = None,
                 peer=None, force_collectives: bool = False):
        C = native()
        if batch % 8:
            raise ValueError("FusedKerasTrainer: batch must be a multiple of 8")
        self.device = torch.device("cuda", device) if isinstance(device, int) else device
        self.batch = batch
        self.comm = comm
        self.use_graph = use_graph
        self.steps_per_graph = steps_per_graph
        self._external = False
        self._captured = False
        n = C.KERAS_NUM_PARAMS
        if init_model is None:
            torch.manual_seed(seed)
            init_model = KerasCNN()
        sd = init_model.state_dict()
        flat = torch.cat([sd[k].detach().reshape(-1).float().cpu() for k, _ in _LAYOUT])
        assert flat.numel() == n
        self.params = flat.to(self.device)
        self.grads = torch.zeros(n, device=self.device)
        self.m = torch.zeros(n, device=self.device)
        self.v = torch.zeros(n, device=self.device)
        self.adam_state = torch.zeros(2, dtype=torch.int32, device=self.device)
        self.lr = torch.full((1,), lr, device=self.device)
        self._lr_host = lr
        self.metrics = torch.zeros(4, device=self.device)
        wsb = C.keras_workspace_bytes(batch)
        self.workspace = torch.zeros(wsb // 4 + 64, dtype=torch.float32, device=self.device)
        torch.cuda.synchronize(self.device)
        if comm is not None and comm.world_size > 1:  # DDP ctor semantics: rank 0's weights everywhere
            comm.broadcast(self.params.data_ptr(), self.params.data_ptr(), n, C.DType.f32, 0,
                           torch.cuda.current_stream(self.device).cuda_stream)
            torch.cuda.synchronize(self.device)
        self.eng = C.KerasEngine(batch, self.params.data_ptr(), self.grads.data_ptr(), self.m.data_ptr(),
                                 self.v.data_ptr(), self.adam_state.data_ptr(), self.workspace.data_ptr(), wsb, comm,
                                 seed, self.lr.data_ptr(), self.metrics.data_ptr(), float(betas[0]), float(betas[1]),
                                 float(eps), float(weight_decay), bool(eps_hat))
        if force_collectives:
            self.eng.set_force_collectives(True)
        if peer is not None:
            self.eng.set_peer(peer)
        self.peer = peer
        self.stream = torch.cuda.ExternalStream(self.eng.stream, device=self.device)
        self.steps = 0
        self.steps_at_reset = 0

    # --------------------------------------------------------------- stepping
    def step(self, n: int = 1):
        """n training steps (graph replays once captured; the first call warms up + captures)."""
        if n <= 0:
            return
        if self.use_graph and not self._captured:
            self.eng.step()  # lazy kernel / communicator init outside the capture
            self.eng.sync()
            spg = self.steps_per_graph or int(os.environ.get("MXDDP_STEPS_PER_GRAPH", "32"))
            self.eng.capture(1 if self._external else spg)
            self._captured = True
            n -= 1
            self.steps += 1
        if n > 0:
            self.eng.replay(n)
            self.steps += n

    def warm_graphs(self) -> int:
        if self.use_graph and not self._captured:
            self.step(1)
        k = self.eng.warm_graphs()
        self.steps += k
        return k

    def set_batch(self, x: torch.Tensor, y: torch.Tensor):
        """Use a caller-provided batch (real MNIST) instead of the on-device generator."""
        if not self._external:
            self.eng.set_external_batch(True)
            self.eng.uncapture()
            self._captured = False
            self._external = True
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            self._x_view().copy_(x.reshape(self.batch, 784), non_blocking=True)
            self._y_view().copy_(y.to(torch.int32), non_blocking=True)
        cur.wait_stream(self.stream)

    def _view(self, ptr, count, dtype=torch.float32):
        off = (ptr - self.workspace.data_ptr()) // 4
        return self.workspace[off:off + count].view(dtype)

    def _x_view(self):
        return self._view(self.eng.x_ptr, self.batch * 784).view(self.batch, 784)

    def _y_view(self):
        return self._view(self.eng.y_ptr, self.batch, torch.int32)

    def set_lr(self, lr: float):
        if lr != self._lr_host:
            with torch.cuda.stream(self.stream):
                self.lr.fill_(lr)
            self._lr_host = lr

    def synchronize(self):
        self.eng.sync()

    def read_metrics(self, reset: bool = True):
        """(loss_sum, correct) since the last reset (one host sync)."""
        self.eng.sync()
        if self.comm is not None:
            self.comm.check_async_error()
        if self.peer is not None and self.peer.error():
            raise RuntimeError(f"keras engine all-reduce: rank {self.peer.error() - 1} never arrived (timeout)")
        m = self.metrics[:2].tolist()
        if reset:
            with torch.cuda.stream(self.stream):
                self.metrics.zero_()
            self.eng.sync()
            self.steps_at_reset = self.steps
        return m[0], m[1]

    @property
    def adam_steps(self) -> int:
        # [0] committed by the next forward, [1] written by the last update (ko_kernel)
        self.eng.sync()
        return int(self.adam_state.max().item())

    def data_state(self) -> torch.Tensor:
        self.eng.sync()
        return self._view(self.eng.counter_ptr, 4, torch.int32).cpu().clone()

    def load_data_state(self, ctr: torch.Tensor):
        self.eng.sync()
        self._view(self.eng.counter_ptr, 4, torch.int32).copy_(ctr.to(torch.int32).to(self.device))
        torch.cuda.synchronize(self.device)

    # --------------------------------------------------------------- state
    def state_dict(self) -> dict:
        self.eng.sync()
        out, off = {}, 0
        for name, shape in _LAYOUT:
            k = 1
            for s in shape:
                k *= s
            out[name] = self.params[off:off + k].view(shape).detach().cpu().clone()
            off += k
        return out

    def optimizer_state(self) -> dict:
        self.eng.sync()
        return {"lr": self._lr_host, "m": self.m.cpu(), "v": self.v.cpu(), "steps": int(self.adam_state.max().item())}

    def load_optimizer_state(self, st: dict):
        self.eng.sync()
        self.m.copy_(st["m"].to(self.device))
        self.v.copy_(st["v"].to(self.device))
        self.adam_state.fill_(int(st["steps"]))
        self.set_lr(float(st["lr"]))
        torch.cuda.synchronize(self.device)

    def load_state_dict(self, sd: dict):
        flat = torch.cat([sd[k].detach().reshape(-1).float().cpu() for k, _ in _LAYOUT])
        self.eng.sync()
        self.params.copy_(flat.to(self.device))
        torch.cuda.synchronize(self.device)
        self.eng.repack()  # conv2 weights live pre-packed in MFMA fragment order
        self.eng.sync()

    def to_module(self) -> KerasCNN:
        m = KerasCNN()
        m.load_state_dict(self.state_dict())
        return m


class FusedKerasReplicas:
    """In-process replica data parallelism (MirroredStrategy, tensorflow2/mnist_mirror_strategy.py:12)
    for the Keras CNN on the fused engine: one FusedKerasTrainer per device, the global batch split
    across them, gradients averaged by the peer transport opened in-process (device peer access),
    so every replica's step -- forward, backward, all-reduce, Adam -- is one graph launch and the
    replicas synchronise on the GPUs.  All replicas' work is launched before the host waits."""

    def __init__(self, devices, batch: int = 64, lr: float = 1e-3, seed: int = 1, init_model=None,
                 use_graph: bool = True, steps_per_graph: int | None = None, blocks: int = 32):
        C = native()
        self.devices = [torch.device(d) for d in devices]
        n = len(self.devices)
        if init_model is None:
            torch.manual_seed(seed)
            init_model = KerasCNN()
        self.peers = [None] * n
        if n > 1:
            self.peers = []
            for i, d in enumerate(self.devices):
                with torch.cuda.device(d):
                    self.peers.append(C.PeerComm(i, n, d.index, 4 << 20, blocks))
            for pc, d in zip(self.peers, self.devices):
                with torch.cuda.device(d):
                    pc.open_local(self.peers)
        self.trainers = []
        for pc, d in zip(self.peers, self.devices):
            with torch.cuda.device(d):
                self.trainers.append(FusedKerasTrainer(batch=batch, device=d, peer=pc, seed=seed, lr=lr,
                                                       init_model=init_model, use_graph=use_graph,
                                                       steps_per_graph=steps_per_graph))
        self.batch = batch
        self._captured = False
        self.use_graph = use_graph

    def _each(self, fn):
        for t, d in zip(self.trainers, self.devices):
            with torch.cuda.device(d):
                fn(t)

    def step(self, n: int = 1):
        if n <= 0:
            return
        if self.use_graph and not self._captured:
            self._each(lambda t: t.eng.step())  # every replica launched before any host wait
            self._each(lambda t: t.eng.sync())
            spg = self.trainers[0].steps_per_graph or int(os.environ.get("MXDDP_STEPS_PER_GRAPH", "32"))
            ext = self.trainers[0]._external
            self._each(lambda t: t.eng.capture(1 if ext else spg))
            self._each(lambda t: setattr(t, "_captured", True))
            self._each(lambda t: setattr(t, "steps", t.steps + 1))
            self._captured = True
            n -= 1
        if n > 0:
            self._each(lambda t: t.eng.replay(n))
            self._each(lambda t: setattr(t, "steps", t.steps + n))

    def set_batch(self, x: torch.Tensor, y: torch.Tensor):
        xs, ys = x.chunk(len(self.trainers)), y.chunk(len(self.trainers))
        for t, d, xi, yi in zip(self.trainers, self.devices, xs, ys):
            with torch.cuda.device(d):
                if not t._external:
                    t.eng.set_external_batch(True)
                    t.eng.uncapture()
                    t._external = True
                    self._captured = False
                t.set_batch(xi.to(d, non_blocking=True), yi.to(d, non_blocking=True))

    def synchronize(self):
        self._each(lambda t: t.eng.sync())
        for pc in self.peers:
            if pc is not None and pc.error():
                raise RuntimeError(f"replica all-reduce: replica {pc.error() - 1} never arrived (timeout)")

    def read_metrics(self):
        self.synchronize()
        ls = cs = 0.0
        for t, d in zip(self.trainers, self.devices):
            with torch.cuda.device(d):
                a, b = t.read_metrics()
            ls, cs = ls + a, cs + b
        return ls, cs

    def state_dict(self) -> dict:
        return self.trainers[0].state_dict()

    def to_module(self):
        return self.trainers[0].to_module()
