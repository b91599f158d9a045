"""DistributedDataParallel on the mxddp bucket reducer.

Same contract as ``torch.nn.parallel.DistributedDataParallel`` as the reference uses it
(pytorch/distributed_data_parallel.py:74; semantics verified in SURVEY §2.2):

1. rank 0's parameters (and buffers) are broadcast at wrap time;
2. gradients are all-reduced and AVERAGED over ranks every backward, bucketed in reverse
   parameter order (first bucket 1 MB, then 25 MB caps), launched asynchronously as each
   bucket fills so communication overlaps the rest of backward;
3. floating buffers (BN running stats) are broadcast from rank 0 before every forward
   (``broadcast_buffers=True``);
4. ``.module`` is the wrapped model, so ``ddp.module.state_dict()`` has no ``module.``
   prefix (checkpoint layout, pytorch/distributed_data_parallel.py:109-113).

``grad_comm_dtype="bf16"`` (opt-in, off by default): every bucket is cast to bf16 before its
all-reduce and back to fp32 after it -- half the bytes on the links for large models (ResNet-50's
102 MB fp32 gradient travels as 51 MB); the optimizer still updates fp32 weights
from fp32 gradient buffers.

GPU: gradients live in one flat buffer (mxddp.parallel.flat); each bucket is an in-place
RCCL all-reduce on the reducer's side HIP stream (C++ ``mxddp._C.Reducer``), fenced by
events.  CPU: the same bucketing over gloo with async work handles.
"""
from __future__ import annotations

import sys

import torch
import torch.distributed as dist
import torch.nn as nn

from .. import native
from . import comm as _comm
from . import graphed as _graphed
from .flat import FlatParams, flatten_buffers


def assign_buckets(numels: list[int], offsets: list[int], total: int, bucket_cap_mb: float = 25.0,
                   first_bucket_cap_mb: float = 1.0, elem_size: int = 4):
    """Greedy reverse-order bucketing (DDP's policy).  Returns (buckets, param_bucket) with
    buckets as contiguous (offset, numel) slices of the flat buffer, bucket 0 = the LAST
    parameters (the first gradients produced by backward)."""
    buckets: list[tuple[int, int]] = []
    param_bucket = [0] * len(numels)
    cap = first_bucket_cap_mb * 1024 * 1024
    cur, cur_bytes, end = [], 0, total
    for i in reversed(range(len(numels))):
        cur.append(i)
        cur_bytes += numels[i] * elem_size
        if cur_bytes >= cap:
            start = offsets[cur[-1]]
            buckets.append((start, end - start))
            for j in cur:
                param_bucket[j] = len(buckets) - 1
            end, cur, cur_bytes = start, [], 0
            cap = bucket_cap_mb * 1024 * 1024
    if cur:
        start = offsets[cur[-1]]
        buckets.append((start, end - start))
        for j in cur:
            param_bucket[j] = len(buckets) - 1
    return buckets, param_bucket


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, device_ids=None, output_device=None, broadcast_buffers: bool = True,
                 bucket_cap_mb: float = 25.0, first_bucket_cap_mb: float = 1.0, average: bool = True,
                 timing: bool = False, transport: str = "auto", grad_comm_dtype: str = "fp32"):
        super().__init__()
        self.module = module
        inf = _comm.info()
        self.world_size, self.rank = inf.world_size, inf.rank
        self.device = next(module.parameters()).device
        self.flat = FlatParams(module, self.device)
        self.flat_buffers = flatten_buffers(module, self.device) if broadcast_buffers else None
        self.broadcast_buffers = broadcast_buffers and self.flat_buffers is not None
        numels = [p.numel() for p in self.flat.params]
        self.buckets, self.param_bucket = assign_buckets(numels, self.flat.offsets, self.flat.numel, bucket_cap_mb,
                                                         first_bucket_cap_mb)
        self.average = average
        if grad_comm_dtype not in ("fp32", "bf16"):
            raise ValueError(f"grad_comm_dtype {grad_comm_dtype!r}: fp32 or bf16")
        self.grad_comm_dtype = grad_comm_dtype
        # --dist-backend gloo on a GPU (pytorch/distributed_data_parallel.py:46): honoured --
        # the gradient buckets and broadcasts go over gloo (host-staged), not RCCL / peer
        self.gloo_data = self.device.type == "cuda" and inf.backend == "gloo" and self.world_size > 1
        native_reducer = self.device.type == "cuda" and not self.gloo_data
        self._comm = _comm.rccl_comm() if native_reducer else None
        self._sync_params()
        if native_reducer:
            C = native()
            self.reducer = C.Reducer(self._comm, self.flat.grad.data_ptr(), C.DType.f32, self.buckets,
                                     self.param_bucket, C.RedOp.avg if average else C.RedOp.sum, timing)
            if grad_comm_dtype == "bf16":
                # bf16 twin of the whole gradient store (slack included: the padded last bucket)
                self._comm_shadow = torch.zeros(self.flat.capacity, dtype=torch.bfloat16, device=self.device)
                self.reducer.set_comm_dtype(C.DType.bf16, self._comm_shadow.data_ptr())
        else:
            self.reducer = _GlooReducer(self.flat.grad, self.buckets, self.param_bucket, average, self.world_size,
                                        bf16=grad_comm_dtype == "bf16")
        self.transport = "rccl" if native_reducer else "gloo"
        self.transport_ms = None
        if native_reducer and self.world_size > 1:
            self._select_transport(transport)
        if native_reducer and self.transport == "rccl":
            self._set_padding()
        self._queued = False
        # fires on both gradient paths: returned gradients and gradients the GPU kernels wrote
        # straight into the flat buffer (mxddp.ops._grad_sink; AccumulateGrad still runs)
        self._hooks = [p.register_post_accumulate_grad_hook(self._make_hook(i)) for i, p in enumerate(self.flat.params)]

    def _select_transport(self, transport: str):
        """Gradient all-reduce transport: RCCL's ring or the direct xGMI peer all-reduce
        (parallel/peer.py).  "auto" validates the peer transport against RCCL and times both on
        this model's buckets; ranks sharing one GPU (no RCCL) must use the peer transport."""
        from . import peer as _peer

        pc = _peer.peer_comm() if transport != "rccl" or self._comm is None else None
        if self._comm is None:
            if pc is None:
                raise RuntimeError("DDP: no RCCL communicator (ranks share a GPU) and no peer transport")
            self.reducer.set_peer(pc)
            self.transport = "peer"
            return
        if pc is not None and not _peer.validate(pc, self._comm):
            if transport == "peer":
                raise RuntimeError("DDP: peer transport requested but unavailable / failed validation")
            pc = None
        if transport == "peer":
            if pc is None:
                raise RuntimeError("DDP: peer transport requested but unavailable")
            self.reducer.set_peer(pc)
            self.transport = "peer"
            return
        # time the xGMI-sized RCCL variants (and the validated peer transport) on this model's
        # buckets; every rank gets the same verdict
        variants = {}
        for v in _comm.rccl_variants():
            c, why = None, ""
            try:  # a variant RCCL refuses (config field, version) is dropped, not fatal
                c = self._comm if v == "default" else _comm.rccl_comm(variant=v)
            except Exception as e:  # noqa: BLE001 - any init failure
                why = str(e).splitlines()[0] if str(e) else type(e).__name__
            if _comm.all_reduce_max(0.0 if c is not None else 1.0) > 0:  # every rank must have it
                if why:
                    print(f"mxddp DDP: RCCL variant {v!r} dropped: {why}", file=sys.stderr, flush=True)
                continue
            variants[v] = c
        choice, self.transport_ms = _peer.pick_transport(pc, variants, [n for _, n in self.buckets])
        if choice == "peer":
            self.reducer.set_peer(pc)
            self.transport = "peer"
            return
        name = choice.split(":", 1)[1]
        self._comm = variants[name]
        self.reducer.set_comm(self._comm)
        self.transport = choice
        self._set_padding()

    def _set_padding(self):
        """Pad the last bucket's all-reduce into the flat buffer's zeroed slack (xGMI sizing)."""
        if self._comm is None or not hasattr(self.reducer, "set_padding"):
            return
        ctas = _comm.parse_variant(self._comm.variant)["ctas"]
        self.reducer.set_padding(self.flat.numel, self.flat.capacity, self.world_size * max(ctas, 32) * 4)

    # ------------------------------------------------------------------ sync helpers
    def _broadcast(self, t: torch.Tensor):
        if self.world_size == 1:
            return
        if self._comm is not None:
            C = native()
            self._comm.broadcast(t.data_ptr(), t.data_ptr(), t.numel(), C.DType.f32, 0,
                                 torch.cuda.current_stream(self.device).cuda_stream)
        elif self.gloo_data:
            dist.broadcast(t, 0)  # gloo data plane: a GPU tensor is staged through the host
        elif t.is_cuda and getattr(self, "transport", None) == "peer":
            # ranks sharing a GPU (no RCCL): broadcast = peer all-reduce of (rank 0 ? t : 0), exact
            # in fp32 and, unlike a host round trip, capturable into a hipGraph
            from . import peer as _peer

            pc = _peer.peer_comm()
            if self.rank != 0:
                t.zero_()
            C = native()
            pc.all_reduce(t.data_ptr(), t.numel(), C.DType.f32, torch.cuda.current_stream(self.device).cuda_stream,
                          C.RedOp.sum)
        elif t.is_cuda:  # before the transport is chosen (wrap time): through the gloo control plane
            h = t.cpu()
            dist.broadcast(h, 0)
            t.copy_(h)
        else:
            dist.broadcast(t, 0)

    def _sync_params(self):
        with torch.no_grad():
            self._broadcast(self.flat.data)
            if self.flat.data.is_cuda:
                from .. import ops

                ops.invalidate_filters(self.flat.data.device)  # raw write: banked filters stale
            if self.flat_buffers is not None:
                self._broadcast(self.flat_buffers)

    # ------------------------------------------------------------------ hooks
    def _make_hook(self, i: int):
        def hook(p):
            if self.device.type == "cuda" and _graphed.capturing() and not torch.cuda.is_current_stream_capturing():
                # the grad accumulator runs on the stream it was created on: one kept alive from an
                # eager step (an autograd graph held across steps) puts this bucket's all-reduce
                # outside the captured step, and every replay would skip it
                raise RuntimeError("DDP: gradient hook ran outside the hipGraph capture (an autograd graph from an "
                                   "earlier step is still alive: detach step outputs accumulated across steps)")
            if not self._queued:
                self._queued = True
                torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
            st = torch.cuda.current_stream(self.device).cuda_stream if self.device.type == "cuda" else 0
            self.reducer.mark_ready(i, st)
        return hook

    def _finalize(self):
        st = torch.cuda.current_stream(self.device).cuda_stream if self.device.type == "cuda" else 0
        self.reducer.finalize(st)
        self._queued = False

    def forward(self, *args, **kwargs):
        self.flat.attach_grads()
        if self.broadcast_buffers and self.world_size > 1 and self.module.training:
            with torch.no_grad():
                self._broadcast(self.flat_buffers)
        if self._queued:
            # the previous backward raised after its first gradient hook: its finalize callback
            # never ran, so drop that step's reducer state before starting a new one
            self.reducer.abort()
            self._queued = False
        if torch.is_grad_enabled():
            self.reducer.prepare()
        return self.module(*args, **kwargs)

    def check(self):
        """Raise if the gradient transport reported a failure (a peer that never arrived in the
        xGMI peer all-reduce, an RCCL async error): a collective that silently gave up would
        leave the ranks training on different gradients."""
        if self.transport == "peer":
            from . import peer as _peer

            pc = _peer.peer_comm()
            if pc is not None and pc.error():
                raise RuntimeError(f"DDP peer all-reduce: rank {pc.error() - 1} never arrived (timeout)")
        elif self._comm is not None and self.world_size > 1:
            self._comm.check_async_error()

    def zero_grad(self, set_to_none: bool = False):
        self.flat.zero_grad()

    @property
    def flat_params(self) -> FlatParams:
        return self.flat


class _GlooReducer:
    """CPU twin of mxddp._C.Reducer: contiguous flat-buffer buckets, async gloo all-reduce
    launched in bucket order as buckets fill, joined in finalize()."""

    def __init__(self, flat_grad, buckets, param_bucket, average, world_size, bf16: bool = False):
        self.flat, self.buckets, self.param_bucket = flat_grad, buckets, param_bucket
        self.average, self.ws, self.bf16 = average, world_size, bf16
        self.total = [0] * len(buckets)
        for b in param_bucket:
            self.total[b] += 1
        self.prepare()

    def prepare(self):
        self.pending = list(self.total)
        self.ready = [False] * len(self.buckets)
        self.marked = set()
        self.next = 0
        self.works = []

    def abort(self, timeout_s: float = 30.0):
        """Drop a step whose backward raised.  Its launched all-reduces are joined first: they
        write into the gradient buffer in place, and one finishing after the next step's
        zero_grad() would corrupt that step.  When every rank raised at the same point (the same
        buckets launched everywhere: a deterministic error) they complete at once; a rank whose
        peers never posted them is out of step for good, and that is raised after `timeout_s`
        instead of hanging (as with torch DDP, an error on one rank only is fatal to the job)."""
        import datetime

        for _off, _n, _t, w in self.works:
            try:
                w.wait(timeout=datetime.timedelta(seconds=timeout_s))
            except Exception as e:  # gloo raises on timeout
                self.prepare()
                raise RuntimeError("DDP abort: the peers did not post the failed step's bucket all-reduces -- "
                                   "the backward raised on this rank only and the ranks are out of step") from e
        self.prepare()

    def mark_ready(self, p, _stream=0):
        if p in self.marked:
            raise RuntimeError("parameter marked ready twice in one backward pass")
        self.marked.add(p)
        b = self.param_bucket[p]
        self.pending[b] -= 1
        if self.pending[b] == 0:
            self.ready[b] = True
            self._launch()

    def mark_bucket_ready(self, b, _stream=0):
        self.pending[b] = 0
        self.ready[b] = True
        self._launch()

    def _launch(self):
        while self.next < len(self.buckets) and self.ready[self.next]:
            off, n = self.buckets[self.next]
            if self.ws > 1:
                t = self.flat[off:off + n].to(torch.bfloat16) if self.bf16 else self.flat[off:off + n]
                self.works.append((off, n, t, dist.all_reduce(t, async_op=True)))
            self.next += 1

    def finalize(self, _stream=0):
        for i in range(len(self.buckets)):
            self.ready[i] = True
        self._launch()
        for off, n, t, w in self.works:
            w.wait()
            if self.bf16:
                self.flat[off:off + n].copy_(t)
            if self.average:
                self.flat[off:off + n].div_(self.ws)
        self.works = []

    @property
    def num_buckets(self):
        return len(self.buckets)
