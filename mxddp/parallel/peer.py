"""Bootstrap + validation of the direct xGMI peer all-reduce (``mxddp._C.PeerComm``, csrc/peer.h).

The reference's DDP all-reduces gradient buckets with NCCL's ring
(pytorch/distributed_data_parallel.py:74,132).  On one 8x MI355X node every GPU has a
point-to-point xGMI link to each peer, so a two-shot all-reduce that uses all 7 links at once
(the peer transport) can beat a ring on latency-bound bucket sizes.  This module

* creates one PeerComm per rank and exchanges the HIP IPC handles of the exchange buffers
  through the control-plane process group (gloo / TCPStore), single node only;
* validates it against RCCL on random data before anything uses it (every rank must agree,
  so a transport that is wrong on ANY rank is dropped by ALL ranks together);
* is what ``FusedMnistTrainer.autotune`` and ``DistributedDataParallel`` pick from.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from .. import native
from . import comm as _comm

_PEER = None


def _agree_ok(ok: bool) -> bool:
    """True only if every rank reports ok (one host all-reduce every rank reaches)."""
    return _comm.all_reduce_max(0.0 if ok else 1.0) == 0.0


def peer_comm(cap_bytes: int = 32 << 20, blocks: int | None = None):
    """This rank's PeerComm (created on first use), or None when the job is not a single-node
    GPU job of 2..8 ranks or the IPC mapping failed on any rank."""
    global _PEER
    if _PEER is not None:
        return _PEER
    inf = _comm.info()
    if inf.world_size < 2 or inf.world_size > 8 or inf.device.type != "cuda" or not dist.is_initialized():
        return None
    if inf.local_world_size != inf.world_size:
        return None  # xGMI peers are on the same node only
    if os.environ.get("MXDDP_PEER", "1") == "0":
        return None
    C = native()
    if blocks is None:
        blocks = 64
    pc, err = None, ""
    try:
        pc = C.PeerComm(inf.rank, inf.world_size, inf.device.index, cap_bytes, blocks)
        mine = pc.handles()
    except RuntimeError as e:  # allocation / IPC export failed here
        mine, err = b"", str(e)
    allh = [None] * inf.world_size
    dist.all_gather_object(allh, mine)
    ok = all(h for h in allh)
    if ok:
        try:
            pc.open(allh)
        except RuntimeError as e:
            ok, err = False, str(e)
    if not _agree_ok(ok):
        if inf.is_main:
            print(f"[mxddp] peer transport unavailable ({err or 'on another rank'}); using RCCL", flush=True)
        return None
    _comm.barrier()
    _PEER = pc
    return pc


def validate(pc, rccl, dtype: str = "f32", numel: int = 1_181_066, iters: int = 3) -> bool:
    """Run the peer all-reduce and RCCL's on the same random per-rank data and compare.
    Collective over all ranks; returns the agreed verdict."""
    inf = _comm.info()
    C = native()
    dev = inf.device
    tdt = torch.float32 if dtype == "f32" else torch.bfloat16
    cdt = C.DType.f32 if dtype == "f32" else C.DType.bf16
    st = torch.cuda.current_stream(dev).cuda_stream
    g = torch.Generator(device="cpu").manual_seed(1234 + inf.rank)
    # a transport that does not work on this machine (flags never seen across the links) must
    # not stall the job for the full 30 s training timeout per call: 2 s while validating
    pc.set_timeout_ms(float(os.environ.get("MXDDP_PEER_VALIDATE_TIMEOUT_MS", "2000")))
    try:
        ok = _validate_iters(pc, rccl, C, dev, tdt, cdt, numel, iters, st, g, inf)
    finally:
        pc.set_timeout_ms(float(os.environ.get("MXDDP_PEER_TIMEOUT_MS", "30000")))
    return _agree_ok(ok)


def _validate_iters(pc, rccl, C, dev, tdt, cdt, numel, iters, st, g, inf) -> bool:
    # every rank runs every iteration (no early exit): the RCCL calls must stay matched across
    # ranks even when the peer transport fails on some of them
    ok = True
    for _ in range(iters):
        x = torch.randn(numel, generator=g).to(dev, tdt)
        a, b = x.clone(), x.clone()
        pc.reset_error()
        pc.all_reduce(a.data_ptr(), numel, cdt, st)
        rccl.all_reduce(b.data_ptr(), b.data_ptr(), numel, cdt, C.RedOp.sum, st)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        if pc.error():
            ok = False
            continue
        tol = 1e-5 * inf.world_size if tdt == torch.float32 else 2e-2
        err = (a.float() - b.float()).abs().max().item()
        scale = b.float().abs().max().item() + 1e-6
        ok = ok and err <= tol * scale
    return ok


def pick_transport(pc, rccl, numels: list[int], dtype: str = "f32", iters: int = 10) -> tuple[str, dict]:
    """Time one pass of all-reduces over buckets of `numels` elements with each transport (the
    DDP reducer's buckets), slowest rank decides; every rank returns the same choice.  ``rccl``
    is one communicator (name "rccl") or {variant: Comm} (names "rccl:<variant>", the xGMI-sized
    variants of comm.py); ``pc`` may be None (RCCL variants only)."""
    import time

    inf = _comm.info()
    C = native()
    dev = inf.device
    tdt = torch.float32 if dtype == "f32" else torch.bfloat16
    cdt = C.DType.f32 if dtype == "f32" else C.DType.bf16
    bufs = [torch.zeros(n, dtype=tdt, device=dev) for n in numels]
    st = torch.cuda.current_stream(dev).cuda_stream
    comms = {"rccl": rccl} if not isinstance(rccl, dict) else {f"rccl:{k}": v for k, v in rccl.items()}
    cands = list(comms) + (["peer"] if pc is not None else [])
    res = {}
    for name in cands:
        def one_pass():
            for b in bufs:
                if name == "peer":
                    pc.all_reduce(b.data_ptr(), b.numel(), cdt, st)
                else:
                    comms[name].all_reduce(b.data_ptr(), b.data_ptr(), b.numel(), cdt, C.RedOp.sum, st)
        one_pass()
        torch.cuda.synchronize(dev)
        _comm.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            one_pass()
        torch.cuda.synchronize(dev)
        res[name] = _comm.all_reduce_max(time.perf_counter() - t0) / iters * 1e3
    if pc is not None:
        if pc.error():
            res["peer"] = float("inf")
        res["peer"] = _comm.all_reduce_max(res["peer"])
    return min(res, key=res.get), res


def resync(pc) -> None:
    """Collective over all ranks: put the peer transport back at a fresh epoch sequence on
    every rank (after an exchange timed out and left the ranks' per-block epochs apart, or when
    an exchange with another block partition -- the Keras co-scheduled KX kernel -- takes over
    the buffers).  Every rank's device is idle before any rank zeroes its flags, and no rank
    exchanges again before every rank has zeroed them."""
    inf = _comm.info()
    if inf.device.type == "cuda":
        torch.cuda.synchronize(inf.device)
    _comm.barrier()
    pc.reset_state()
    _comm.barrier()


def shutdown():
    global _PEER
    _PEER = None
