"""Flat parameter / gradient storage.

All trainable parameters of a module are re-homed into ONE contiguous fp32 buffer (and
their ``.grad`` into a second one), in registration order, each parameter padded to a
64-byte boundary.  Consequences:

* the optimizer is one multi-tensor kernel over the flat buffer (mxddp.optim);
* DDP buckets are contiguous slices of the grad buffer (no copy-in/copy-out), and
  backward-order buckets are simply slices taken from the END of the buffer;
* the buffers are sized once and stay resident in HBM (288 GB per MI355X: nothing is
  ever re-allocated per step).
"""
from __future__ import annotations

import torch
import torch.nn as nn

_ALIGN = 16  # elements (64 bytes)
_GRAD_SLACK = 1024  # elements >= 8 ranks x 32 channels x 4


def _al(n: int) -> int:
    return (n + _ALIGN - 1) // _ALIGN * _ALIGN


def _noop():
    return None


class FlatParams:
    def __init__(self, module: nn.Module, device: torch.device | None = None):
        self.params = [p for p in module.parameters() if p.requires_grad]
        self.names = [n for n, p in module.named_parameters() if p.requires_grad]
        device = device or (self.params[0].device if self.params else torch.device("cpu"))
        self.offsets, off = [], 0
        for p in self.params:
            self.offsets.append(off)
            off += _al(p.numel())
        self.numel = max(off, _ALIGN)
        self.data = torch.zeros(self.numel, dtype=torch.float32, device=device)
        # zeroed slack after the gradients: the DDP reducer pads the all-reduce of the bucket that
        # ends there to a multiple of world_size x channels x 16 B (Reducer::set_padding)
        self.capacity = self.numel + _GRAD_SLACK
        self._grad_store = torch.zeros(self.capacity, dtype=torch.float32, device=device)
        self.grad = self._grad_store[:self.numel]
        with torch.no_grad():
            for p, o in zip(self.params, self.offsets):
                self.data[o:o + p.numel()].copy_(p.detach().reshape(-1))
                p.data = self.data[o:o + p.numel()].view_as(p)
        # marker for direct gradient writing (mxddp.ops._grad_sink): GPU backward kernels
        # accumulate into p.grad (a view of self.grad) instead of returning a gradient
        for p in self.params:
            p._mx_grad_ready = _noop
        self.attach_grads()

    def attach_grads(self) -> None:
        """(Re)point every param.grad at its slice of the flat grad buffer."""
        for p, o in zip(self.params, self.offsets):
            g = self.grad[o:o + p.numel()].view_as(p)
            if p.grad is None or p.grad.data_ptr() != g.data_ptr():
                p.grad = g

    def zero_grad(self) -> None:
        self.grad.zero_()  # the slack stays zero: only all-reduces of zeros ever touch it
        self.attach_grads()

    def span(self, i: int) -> tuple[int, int]:
        return self.offsets[i], self.params[i].numel()


def flatten_buffers(module: nn.Module, device: torch.device | None = None):
    """Re-home floating-point buffers (BN running stats) into one flat tensor so the DDP
    per-forward buffer broadcast (reference default broadcast_buffers=True) is ONE
    collective.  Integer buffers (num_batches_tracked) stay separate (identical on all
    ranks because every rank runs the same number of steps)."""
    bufs = [(n, b) for n, b in module.named_buffers() if b is not None and b.is_floating_point()]
    if not bufs:
        return None
    device = device or bufs[0][1].device
    total = sum(_al(b.numel()) for _, b in bufs)
    flat = torch.zeros(total, dtype=torch.float32, device=device)
    off = 0
    for name, b in bufs:
        n = b.numel()
        flat[off:off + n].copy_(b.reshape(-1))
        b.data = flat[off:off + n].view_as(b)
        off += _al(n)
    return flat
