"""Flat multi-tensor optimizers (one HIP kernel per step over the whole model).

``SGD`` follows torch.optim.SGD exactly (momentum buffer = grad at the first step,
coupled weight decay), as used by the reference (pytorch/distributed_data_parallel.py:94-95).
``Adam`` follows torch.optim.Adam; ``eps_hat=True`` gives the Keras / Chainer placement
of epsilon (tensorflow2/mnist_single.py:78, chainer/train_mnist.py:69).

The learning rate lives in a 1-element device tensor so schedulers (StepLR,
pytorch/distributed_data_parallel.py:97) keep working under hipGraph replay.
``grad_scale`` folds DDP's 1/world_size average into the update when the reducer
sums instead of averaging.  After a GPU step the banked Winograd filters of the model's 3x3
convs are re-transformed in one launch (ops.refresh_filters).
"""
from __future__ import annotations

import torch

from . import native
from . import ops as _ops
from .parallel.flat import FlatParams


class _FlatOptimizer:
    def __init__(self, flat: FlatParams, lr: float):
        self.flat = flat
        self.param_groups = [{"lr": lr, "initial_lr": lr}]
        dev = flat.data.device
        self._lr_dev = torch.full((1,), lr, dtype=torch.float32, device=dev)
        self._lr_host = lr
        self.grad_scale = 1.0

    def _sync_lr(self):
        """Write a changed host learning rate to the device tensor the kernels read.  Never
        inside a stream capture: the fill would be recorded into the graph and every replay
        would write the capture-time lr back over the value ``before_replay`` set.  The sync is
        left pending instead (``_lr_host`` unchanged), so the next eager step or
        ``before_replay`` applies it."""
        lr = self.param_groups[0]["lr"]
        if lr != self._lr_host:
            if self._lr_dev.is_cuda and torch.cuda.is_current_stream_capturing():
                return
            self._lr_dev.fill_(lr)
            self._lr_host = lr

    def zero_grad(self, set_to_none: bool = False):
        self.flat.zero_grad()

    @property
    def lr(self):
        return self.param_groups[0]["lr"]


class SGD(_FlatOptimizer):
    def __init__(self, flat: FlatParams, lr: float = 0.1, momentum: float = 0.0, weight_decay: float = 0.0):
        super().__init__(flat, lr)
        self.momentum, self.weight_decay = momentum, weight_decay
        self.buf = torch.zeros_like(flat.data) if momentum else flat.data.new_zeros(16)
        # completed steps: on a GPU a device counter advanced inside the step (graph replays
        # count too), on the CPU a host int
        self._steps_host = 0
        self._steps_dev = torch.zeros(1, dtype=torch.int64, device=flat.data.device) if flat.data.is_cuda else None

    @property
    def steps(self) -> int:
        if self._steps_dev is not None:
            return int(self._steps_dev.item())
        return self._steps_host

    @steps.setter
    def steps(self, n: int):
        self._steps_host = int(n)
        if self._steps_dev is not None:
            self._steps_dev.fill_(int(n))

    @torch.no_grad()
    def step(self):
        self._sync_lr()
        f = self.flat
        if f.data.is_cuda:
            _ops.flush_wgrad(f.data.device)  # deferred weight-gradient reductions land first
            native().sgd_step(f.data.data_ptr(), f.grad.data_ptr(), self.buf.data_ptr(), self._lr_dev.data_ptr(),
                              float(self.grad_scale), float(self.momentum), float(self.weight_decay), f.numel,
                              False, torch.cuda.current_stream(f.data.device).cuda_stream)
            _ops.refresh_filters(f.data.device)
        else:
            g = f.grad * self.grad_scale + self.weight_decay * f.data
            if self.momentum:
                self.buf.mul_(self.momentum).add_(g)  # buf starts at 0 -> buf = g at step 1
                g = self.buf
            f.data.sub_(self.lr * g)
        if self._steps_dev is not None:
            self._steps_dev.add_(1)
        else:
            self._steps_host += 1

    def state_dict(self):
        return {"lr": self.lr, "momentum_buffer": self.buf.detach().cpu().clone(), "steps": self.steps}

    def load_state_dict(self, sd):
        self.param_groups[0]["lr"] = sd["lr"]
        self.buf.copy_(sd["momentum_buffer"])
        self.steps = sd["steps"]


class Adam(_FlatOptimizer):
    """On a GPU the step count lives on the device (``_state``: completed steps, the count being
    applied) and the kernels advance it, so ``step()`` issues two launches (update, one-block
    commit) and no host value: a captured hipGraph replays Adam exactly (bias corrections and the
    eps_hat form included)."""

    def __init__(self, flat: FlatParams, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, eps_hat: bool = False):
        super().__init__(flat, lr)
        self.b1, self.b2 = betas
        self.eps, self.weight_decay, self.eps_hat = eps, weight_decay, eps_hat
        self.m = torch.zeros_like(flat.data)
        self.v = torch.zeros_like(flat.data)
        self._steps_host = 0  # CPU path / host mirror of the eager step count
        self._state = torch.zeros(2, dtype=torch.int32, device=flat.data.device)

    @property
    def steps(self) -> int:
        if self.flat.data.is_cuda:
            return int(self._state[0].item())
        return self._steps_host

    @torch.no_grad()
    def step(self):
        self._sync_lr()
        f = self.flat
        if f.data.is_cuda:
            _ops.flush_wgrad(f.data.device)  # deferred weight-gradient reductions land first
            native().adam_step(f.data.data_ptr(), f.grad.data_ptr(), self.m.data_ptr(), self.v.data_ptr(),
                               self._lr_dev.data_ptr(), self._state.data_ptr(), float(self.grad_scale),
                               self.b1, self.b2, float(self.eps), float(self.weight_decay), bool(self.eps_hat),
                               f.numel, torch.cuda.current_stream(f.data.device).cuda_stream)
            _ops.refresh_filters(f.data.device)
        else:
            self._steps_host += 1
            t = self._steps_host
            eps = self.eps / (1.0 - self.b2 ** t) ** 0.5 if self.eps_hat else self.eps
            g = f.grad * self.grad_scale + self.weight_decay * f.data
            self.m.mul_(self.b1).add_(g, alpha=1 - self.b1)
            self.v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            bc1 = 1 - self.b1 ** t
            bc2 = 1 - self.b2 ** t
            denom = (self.v.sqrt() / bc2 ** 0.5).add_(eps)
            f.data.addcdiv_(self.m, denom, value=-self.lr / bc1)

    def state_dict(self):
        return {"lr": self.lr, "m": self.m.cpu().clone(), "v": self.v.cpu().clone(), "steps": self.steps}

    def load_state_dict(self, sd):
        self.param_groups[0]["lr"] = sd["lr"]
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        self._steps_host = int(sd["steps"])
        self._state.fill_(int(sd["steps"]))


class StepLR:
    """torch.optim.lr_scheduler.StepLR semantics (pytorch/distributed_data_parallel.py:97,101)."""

    def __init__(self, opt: _FlatOptimizer, step_size: int, gamma: float = 0.1):
        self.opt, self.step_size, self.gamma = opt, step_size, gamma
        self.base = opt.param_groups[0]["initial_lr"]
        self.last_epoch = 0

    def step(self):
        self.last_epoch += 1
        self.opt.param_groups[0]["lr"] = self.base * self.gamma ** (self.last_epoch // self.step_size)

    def state_dict(self):
        return {"last_epoch": self.last_epoch}

    def load_state_dict(self, sd):
        self.last_epoch = sd["last_epoch"]
        self.opt.param_groups[0]["lr"] = self.base * self.gamma ** (self.last_epoch // self.step_size)
