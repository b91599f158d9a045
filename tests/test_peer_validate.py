"""Peer-transport validation logic (mxddp.parallel.peer._validate_iters) with fake transports on
the CPU: a transport that errors or disagrees with RCCL is rejected, and every rank issues the
same number of RCCL calls whatever the peer transport does (no early exit that would leave the
other ranks' collectives unmatched)."""
import types

import torch

from mxddp.parallel import peer


class _Fake:
    def __init__(self, store, fail_at=None, wrong=False):
        self.store, self.fail_at, self.wrong = store, fail_at, wrong
        self.calls, self.err = 0, 0

    def reset_error(self):
        self.err = 0

    def error(self):
        return self.err

    def all_reduce(self, ptr, n, *args):  # "sum over 2 ranks" of identical data = 2 x
        t = self.store[ptr]
        self.calls += 1
        if self.fail_at is not None and self.calls >= self.fail_at:
            self.err = 2
            return
        t.mul_(2.0 if not self.wrong else 2.5)


class _Rccl(_Fake):
    def all_reduce(self, src, dst, n, *args):
        super().all_reduce(dst, n)


def _run(pc_kw, iters=3):
    store = {}
    orig_clone = torch.Tensor.clone

    def clone(t, *a, **k):  # register every clone so the fakes can find it by data_ptr
        c = orig_clone(t, *a, **k)
        store[c.data_ptr()] = c
        return c

    torch.Tensor.clone = clone
    try:
        pc, rc = _Fake(store, **pc_kw), _Rccl(store)
        C = types.SimpleNamespace(RedOp=types.SimpleNamespace(sum=0))
        inf = types.SimpleNamespace(world_size=2)
        g = torch.Generator().manual_seed(0)
        ok = peer._validate_iters(pc, rc, C, torch.device("cpu"), torch.float32, None, 1000, iters, 0, g, inf)
    finally:
        torch.Tensor.clone = orig_clone
    return ok, rc.calls


def test_validate_accepts_matching_transport():
    assert _run({}) == (True, 3)


def test_validate_rejects_erroring_transport_without_early_exit():
    ok, rccl_calls = _run({"fail_at": 1})
    assert not ok and rccl_calls == 3


def test_validate_rejects_wrong_sums():
    ok, rccl_calls = _run({"wrong": True})
    assert not ok and rccl_calls == 3
