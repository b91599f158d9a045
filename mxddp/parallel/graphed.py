"""Whole training step captured in ONE hipGraph, at any world size.

The reference's DDP step (pytorch/distributed_data_parallel.py:118-152) is ~1,500 kernel launches
for PyramidNet and ~700 for ResNet-50, issued one by one from Python through autograd.  On MI355X
that host path, not the GPU, bounds small-batch steps.  ``GraphedStep`` records the step once --
zero-grad, the DDP per-forward BN-buffer broadcast, forward, loss, backward with every bucket
all-reduce the reducer issues (RCCL or the xGMI peer transport, on the reducer's side stream,
joined by its finalize), the flat optimizer and the on-device loss / accuracy accumulation -- and
replays it with one ``hipGraphLaunch`` per step.

What keeps a replay identical to an eager step:

* every input is copied into static device buffers first (the batch), and every host-side
  value the step reads is already on the device (learning rate, Adam step count, synthetic-data
  counters, BN ``num_batches_tracked``);
* ``before_replay`` runs host bookkeeping that eager steps do inside ``opt.step()`` (a StepLR
  change of the learning rate is written to the device tensor the graph reads);
* collectives run in the same order on every rank because every rank captured the same step;
* steps whose batch shape differs from the captured one (the last partial batch of an epoch) run
  eagerly -- the same code, so the numerics match.

``gloo`` data planes are host-staged and cannot be captured: such steps stay eager.
"""
from __future__ import annotations

import torch

from .. import native

_CAPTURE_STREAMS: dict = {}
_CAPTURING = [0]


def capturing() -> bool:
    """True while a GraphedStep records its step (hooks use it to check they run inside it)."""
    return _CAPTURING[0] > 0


def capture_stream(device: torch.device, slot: int = 0) -> torch.cuda.Stream:
    """One stream per device on which every mxddp hipGraph is captured.  Stream-owned scratch
    (the split-K partial planes of ops_gemm.hip) is reserved for it here, outside any capture:
    a GEMM captured on a stream without planes would have to run unsplit.  ``slot``: graphs that
    REPLAY CONCURRENTLY on one device (replicas sharing a GPU) need capture streams of their own,
    or their captured GEMMs would share one set of partial planes."""
    device = torch.device(device)
    s = _CAPTURE_STREAMS.get((device, slot))
    if s is None:
        s = torch.cuda.Stream(device)
        native().reserve_splitk_planes(s.cuda_stream)
        _CAPTURE_STREAMS[(device, slot)] = s
    return s


class GraphedStep:
    def __init__(self, step_fn, device: torch.device, warmup: int = 2, before_replay=None, enabled: bool = True):
        """``step_fn(x, y)`` runs one full training step on device tensors and returns a tuple
        of device tensors (static after capture).  The first ``warmup`` calls run eagerly (lazy
        kernel / allocator / communicator initialisation must not happen inside a capture)."""
        self.step_fn = step_fn
        self.device = device
        self.warmup = warmup
        self.before_replay = before_replay
        self.enabled = enabled and device.type == "cuda"
        self.graph = None
        self.calls = 0
        self.replays = 0
        self._x = self._y = self._out = None

    @property
    def captured(self) -> bool:
        return self.graph is not None

    def __call__(self, x: torch.Tensor, y: torch.Tensor):
        self.calls += 1
        if not self.enabled:
            return self.step_fn(x, y)
        if self.graph is not None and x.shape == self._x.shape and y.shape == self._y.shape:
            self._x.copy_(x, non_blocking=True)
            self._y.copy_(y, non_blocking=True)
            if self.before_replay is not None:
                self.before_replay()
            self.graph.replay()
            self.replays += 1
            return self._out
        if self.graph is None and self.calls > self.warmup:
            return self._capture(x, y)
        return self.step_fn(x, y)

    def _capture(self, x, y):
        cur = torch.cuda.current_stream(self.device)
        self._x = x.detach().clone()
        self._y = y.detach().clone()
        side = capture_stream(self.device)
        side.wait_stream(cur)
        g = torch.cuda.CUDAGraph()
        # thread-local capture mode: the communicator and reducer issue their own stream work
        # (side comm stream, RCCL kernels) from this thread inside the capture
        _CAPTURING[0] += 1
        try:
            with torch.cuda.graph(g, stream=side, capture_error_mode="thread_local"):
                self._out = self.step_fn(self._x, self._y)
        finally:
            _CAPTURING[0] -= 1
        cur.wait_stream(side)
        self.graph = g
        # the capture only RECORDED the step: run it once so this call trains like any other
        if self.before_replay is not None:
            self.before_replay()
        g.replay()
        self.replays += 1
        return self._out
