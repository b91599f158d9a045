"""Single-process multi-GPU "replica" data parallelism.

Capability of ``nn.DataParallel`` (pytorch/data_parallel.py:70-72), TF2
``MirroredStrategy`` (tensorflow2/mnist_mirror_strategy.py:12,68-73) and Chainer
``ParallelUpdater`` (chainer/train_mnist_gpu.py:87-93): ONE process drives N GPUs, the
*global* batch is split across them (strong scaling).

MI355X-native design -- MirroredStrategy semantics rather than
DataParallel's replicate-every-step:

* replicas are created once and kept in sync (rank-0 broadcast at start); there is no
  97 MB per-step re-replication and no gather onto device 0 (the reason the reference's
  DataParallel reaches only 80 % GPU utilisation, pytorch/README.md:64);
* per-replica flat gradient buffers are averaged with ONE grouped RCCL all-reduce
  (``ncclCommInitAll`` communicators, ncclGroupStart/End) over xGMI;
* every replica runs its own flat optimizer step, so replicas never diverge;
* all replicas' backward passes are issued by a single multi-root autograd call, which
  runs the per-device graphs concurrently on the autograd engine's device threads;
* ``use_graph=True`` captures each replica's WHOLE step -- BN-buffer sync, zero-grad, forward,
  backward, gradient average over the in-process peer transport, optimizer (SGD, or Adam with
  its step count on the device), metric accumulation -- into one hipGraph per device after two
  eager warm-up steps (inputs copied into static per-device buffers), so a step is n graph
  launches and nothing else, instead of hundreds of Python-issued kernels per replica.
"""
from __future__ import annotations

import copy
import os
import warnings
import weakref

import torch
import torch.nn as nn

from .. import native
from ..fused import FusedReplicas
from .flat import FlatParams, flatten_buffers


class ReplicaGroup:
    """Replicas of ``model`` on ``devices`` kept in lockstep.  Several replicas may share one
    device (a functional rehearsal of an N-GPU node on one GPU): their exchanges are the peer
    transport, and each replica's exchange kernel spins on the GPU until every peer arrives, so
    each replica's streams (exchange, capture and -- graph mode -- the reducer's side stream)
    must land on hardware queues of their own, or a replica queued behind another's spinning
    exchange stalls until the peer timeout.  HIP gives a process GPU_MAX_HW_QUEUES queues (4 by
    default); a shared-device group that needs more warns at construction (raise the variable
    before the process first touches the GPU)."""

    STREAMS_PER_REPLICA = 3  # exchange stream, capture stream, reducer side stream (graph mode)

    def __init__(self, model: nn.Module, devices: list[torch.device], make_optimizer, broadcast_buffers: bool = True,
                 use_graph: bool = False, peer_blocks: int = 64, bucket_cap_mb: float = 25.0):
        self.devices = [torch.device(d) for d in devices]
        self.use_graph = use_graph and all(torch.device(d).type == "cuda" for d in devices)
        self._graphs = None  # per-device hipGraphs of the WHOLE step
        self._eager_steps = 0
        base = model.to(self.devices[0])
        self.replicas = [base] + [copy.deepcopy(base).to(d) for d in self.devices[1:]]
        self.flats = [FlatParams(m, d) for m, d in zip(self.replicas, self.devices)]
        self.buffers = [flatten_buffers(m, d) for m, d in zip(self.replicas, self.devices)] if broadcast_buffers else None
        self.optimizers = [make_optimizer(f) for f in self.flats]
        self.n = len(self.devices)
        # per-device on-device metric accumulators (sum of per-image loss, correct count)
        self._acc = [torch.zeros(2, device=d) for d in self.devices]
        self.comms = None
        self.peers = None
        self.reducers = None
        self._capturing = None  # replica whose step is being captured (its gradient hooks are live)
        # several replicas on ONE device (a rehearsal of an N-GPU node on one GPU): RCCL cannot
        # span them, so every exchange is the in-process peer transport
        self.shared = len(set(self.devices)) < self.n
        self._hook_handles = []
        self._align_buf = None
        if self.shared:
            need = self.n * (self.STREAMS_PER_REPLICA if self.use_graph else 1) + 1
            have = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
            if need > have:
                warnings.warn(f"ReplicaGroup: {self.n} replicas share a device and need ~{need} hardware queues "
                              f"(GPU_MAX_HW_QUEUES={have}): a replica's exchange may wait behind another's until "
                              "the peer timeout; set GPU_MAX_HW_QUEUES >= that before the GPU is first used",
                              RuntimeWarning, stacklevel=2)
        if self.n > 1:
            if any(d.type != "cuda" for d in self.devices):
                raise ValueError("replica mode across several devices needs GPUs")
            if not self.shared:
                self.comms = native().Comm.init_all([d.index for d in self.devices])
            # every replica's exchange kernels run on a stream of its own: a replica's all-reduce
            # waits on the GPU for the others', which must not be queued behind it
            self._rs = [torch.cuda.Stream(d) for d in self.devices]
            if self.use_graph or self.shared:
                # the in-graph gradient / buffer exchange: the peer transport opened in-process
                # (device peer access, no IPC) -- an ordinary kernel per device, so each replica's
                # whole step is one graph launch (RCCL's single-thread multi-device calls need a
                # host-side group and stay on the eager path)
                C = native()
                self.peers = []
                for i, d in enumerate(self.devices):
                    with torch.cuda.device(d):
                        self.peers.append(C.PeerComm(i, self.n, d.index, 32 << 20, peer_blocks))
                for pc, d in zip(self.peers, self.devices):
                    with torch.cuda.device(d):
                        pc.open_local(self.peers)
            if self.use_graph:
                self._make_reducers(bucket_cap_mb)
        self._sync(self.flats[0].data, [f.data for f in self.flats])
        if self.n > 1:  # raw-pointer write to the replicas' weights: banked conv filters are stale
            from .. import ops

            ops.invalidate_filters()
        if self.buffers and self.buffers[0] is not None:
            self._sync(self.buffers[0], self.buffers)

    def _make_reducers(self, bucket_cap_mb: float):
        """Graph mode: per replica, the DDP bucket reducer (csrc/reducer.cpp) over the peer
        transport -- reverse-order buckets (1 MB first, then bucket_cap_mb) all-reduced on the
        reducer's side stream as the backward fills them, so the exchange overlaps the rest of the
        backward (PyramidNet's 97 MB gradient leaves in 5 buckets instead of one exchange after
        the backward).  The hooks only act while a replica's step is being captured."""
        from .ddp import assign_buckets

        C = native()
        f0 = self.flats[0]
        self.buckets, pb = assign_buckets([p.numel() for p in f0.params], f0.offsets, f0.numel, bucket_cap_mb,
                                          min(1.0, bucket_cap_mb))
        self.reducers = []
        for i, (f, d) in enumerate(zip(self.flats, self.devices)):
            with torch.cuda.device(d):
                r = C.Reducer(None, f.grad.data_ptr(), C.DType.f32, self.buckets, pb, C.RedOp.avg, False)
                r.set_peer(self.peers[i])
                r.comm_stream()  # its side stream exists before the capture that first uses it
            self.reducers.append(r)
            for j, p in enumerate(f.params):
                self._hook_handles.append(p.register_post_accumulate_grad_hook(self._hook(i, j)))

    def _hook(self, i: int, j: int):
        # the hooks live on the parameters (replica 0's are the caller's model): they hold the
        # group only weakly, so the group, its reducers and peer transports can be collected
        ref = weakref.ref(self)

        def hook(p):
            g = ref()
            if g is not None and g._capturing == i:
                # fenced against the capture stream the step's backward kernels run on (the hook
                # runs on an autograd device thread, whose current stream need not be that one)
                g.reducers[i].mark_ready(j, g._cap_stream)
        return hook

    def close(self):
        """Remove the gradient hooks from the replicas' parameters (the caller's model keeps no
        reference to this group afterwards)."""
        for h in self._hook_handles:
            h.remove()
        self._hook_handles = []

    def align(self) -> str:
        """Device-side start line of a timed region (bench.py, config 4): one tiny all-reduce over
        the replicas on every device's current stream, so the devices leave it together; events
        recorded right after it on each device's current stream are a common start.  Returns
        the transport ("peer", "rccl" or "none")."""
        if self.n == 1:
            return "none"
        C = native()
        if self._align_buf is None:
            self._align_buf = [torch.zeros(64, device=d) for d in self.devices]
        if self.peers is not None:
            self._peer_each(self._align_buf, C.RedOp.sum)
            return "peer"
        C.Comm.group_start()
        for i, (c, t) in enumerate(zip(self.comms, self._align_buf)):
            c.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), C.DType.f32, C.RedOp.sum, self._stream(i))
        C.Comm.group_end()
        return "rccl"

    # ------------------------------------------------------------------ collectives
    def _stream(self, i):
        return torch.cuda.current_stream(self.devices[i]).cuda_stream

    def _peer_each(self, tensors, op, zero_others: bool = False):
        """One peer all-reduce per replica, each on its replica's own stream (ordered after the
        device's current stream, and the current stream after it)."""
        C = native()
        for i, (t, d) in enumerate(zip(tensors, self.devices)):
            rs = self._rs[i]
            rs.wait_stream(torch.cuda.current_stream(d))
            with torch.cuda.stream(rs):
                if zero_others and i != 0:
                    t.zero_()
                self.peers[i].all_reduce(t.data_ptr(), t.numel(), C.DType.f32, rs.cuda_stream, op)
        for rs, d in zip(self._rs, self.devices):
            torch.cuda.current_stream(d).wait_stream(rs)

    def _sync(self, src, dsts):
        if self.n == 1:
            return
        C = native()
        if self.comms is None:  # broadcast from replica 0 = peer sum of (replica 0 ? t : 0), exact
            self._peer_each(dsts, C.RedOp.sum, zero_others=True)
            return
        C.Comm.group_start()
        for i, (c, t) in enumerate(zip(self.comms, dsts)):
            c.broadcast(t.data_ptr(), t.data_ptr(), t.numel(), C.DType.f32, 0, self._stream(i))
        C.Comm.group_end()

    def _all_reduce_grads(self):
        if self.n == 1:
            return
        C = native()
        if self.comms is None:
            self._peer_each([f.grad for f in self.flats], C.RedOp.avg)
            return
        C.Comm.group_start()
        for i, (c, f) in enumerate(zip(self.comms, self.flats)):
            c.all_reduce(f.grad.data_ptr(), f.grad.data_ptr(), f.numel, C.DType.f32, C.RedOp.avg, self._stream(i))
        C.Comm.group_end()

    # ------------------------------------------------------------------ training step
    def train(self, mode: bool = True):
        for m in self.replicas:
            m.train(mode)

    def zero_grad(self):
        for f in self.flats:
            f.zero_grad()

    def step(self, x: torch.Tensor, y: torch.Tensor, loss_fn):
        """One synchronous-replica step on a GLOBAL batch.  Loss (per-image sum) and correct
        count accumulate on the devices; read them with read_metrics() (no host sync here)."""
        xs, ys = x.chunk(self.n), y.chunk(self.n)
        if len(xs) != self.n:
            raise ValueError(f"global batch {x.shape[0]} smaller than the number of replicas {self.n}")
        if self.use_graph:
            if self._graphs is None and self._eager_steps >= 2:  # allocator / autograd warmed up
                self._capture(xs, ys, loss_fn)
            if self._graphs is not None and [t.shape for t in xs] == [t.shape for t in self._xs]:
                return self._replay(xs, ys)
            self._eager_steps += 1
        if self.buffers and self.buffers[0] is not None and self.n > 1:
            self._sync(self.buffers[0], self.buffers)
        self.zero_grad()
        losses, corrects = [], []
        for i, (m, d) in enumerate(zip(self.replicas, self.devices)):
            xi = xs[i].to(d, non_blocking=True)
            yi = ys[i].to(d, non_blocking=True)
            loss, correct = loss_fn(m(xi), yi)
            losses.append(loss)
            corrects.append(correct)
        torch.autograd.backward(losses)  # one multi-root call: per-device graphs run concurrently
        self._all_reduce_grads()
        for i, opt in enumerate(self.optimizers):
            opt.step()
            self._accumulate(i, losses[i].detach(), corrects[i], xs[i].shape[0])

    def _accumulate(self, i, loss, correct, n):
        a = self._acc[i]
        a[0].add_(loss * n)
        a[1].add_(correct)

    def read_metrics(self) -> tuple[float, float]:
        """(sum of per-image losses, correct) over all replicas since the last read (host sync)."""
        tot = [0.0, 0.0]
        for i, d in enumerate(self.devices):
            torch.cuda.synchronize(d) if d.type == "cuda" else None
            v = self._acc[i].tolist()
            tot[0] += v[0]
            tot[1] += v[1]
            self._acc[i].zero_()
        self._check_peers()
        return tot[0], tot[1]

    def _check_peers(self):
        for pc in self.peers or []:
            if pc.error():
                raise RuntimeError(f"replica all-reduce: replica {pc.error() - 1} never arrived (timeout)")

    def _graph_step(self, i, loss_fn):
        """Replica i's whole step, as captured: BN-buffer sync from replica 0, zero-grad,
        forward, loss, backward, gradient average, optimizer, metric accumulation."""
        C = native()
        st = self._stream(i)
        if self.n > 1 and self.buffers and self.buffers[i] is not None:
            # broadcast from replica 0 = peer sum of (replica 0 ? buffers : 0): exact in fp32
            if i != 0:
                self.buffers[i].zero_()
            self.peers[i].all_reduce(self.buffers[i].data_ptr(), self.buffers[i].numel(), C.DType.f32, st, C.RedOp.sum)
        self.flats[i].zero_grad()
        loss, correct = loss_fn(self.replicas[i](self._xs[i]), self._ys[i])
        if self.reducers is not None:
            # bucketed: each bucket's average leaves on the reducer's side stream as soon as the
            # backward has filled it; finalize joins them before the optimizer
            r = self.reducers[i]
            r.prepare()
            self._cap_stream = st
            self._capturing = i
            try:
                loss.backward()
            finally:
                self._capturing = None
            r.finalize(st)
        else:
            loss.backward()
        self.optimizers[i].step()
        self._accumulate(i, loss.detach(), correct, self._xs[i].shape[0])

    def _capture(self, xs, ys, loss_fn):
        self._xs = [t.to(d).clone() for t, d in zip(xs, self.devices)]
        self._ys = [t.to(d).clone() for t, d in zip(ys, self.devices)]
        graphs = []
        for i, d in enumerate(self.devices):
            with torch.cuda.device(d):
                from .graphed import capture_stream

                cur = torch.cuda.current_stream(d)
                # replicas sharing a device replay concurrently: a capture stream (and its split-K
                # planes) each
                side = capture_stream(d, i if self.shared else 0)
                side.wait_stream(cur)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=side, capture_error_mode="thread_local"):
                    self._graph_step(i, loss_fn)
                cur.wait_stream(side)
            graphs.append(g)
        self._graphs = graphs

    def _replay(self, xs, ys):
        # EVERY replica's graph is launched before the host waits on any of them, each on its
        # replica's own stream: each graph's gradient exchange waits on the GPUs for the others
        if self.n == 1:
            with torch.cuda.device(self.devices[0]):
                self._xs[0].copy_(xs[0], non_blocking=True)
                self._ys[0].copy_(ys[0], non_blocking=True)
                self.optimizers[0]._sync_lr()
                self._graphs[0].replay()
            return
        for i, d in enumerate(self.devices):
            rs = self._rs[i]
            with torch.cuda.device(d):
                rs.wait_stream(torch.cuda.current_stream(d))
                with torch.cuda.stream(rs):
                    self._xs[i].copy_(xs[i], non_blocking=True)
                    self._ys[i].copy_(ys[i], non_blocking=True)
                    self.optimizers[i]._sync_lr()
                    self._graphs[i].replay()
        for rs, d in zip(self._rs, self.devices):
            torch.cuda.current_stream(d).wait_stream(rs)

    @property
    def module(self) -> nn.Module:
        return self.replicas[0]


class FusedMnistReplicas(FusedReplicas):
    """In-process replica data parallelism for the MNIST CNN on the fused native engine: ONE
    process drives one ``FusedMnistTrainer`` per device (MirroredStrategy / DataParallel /
    ParallelUpdater semantics: the global batch = replicas x per-replica batch, gradients
    averaged every step, replicas stay identical).

    The gradient exchange is the peer transport opened in-process (``PeerComm.open_local``:
    device peer access over xGMI, no IPC), so a replica's whole step -- forward, backward,
    all-reduce, SGD -- stays one hipGraph on its own stream and the host only issues one graph
    launch per replica per group of steps; the replicas synchronise with each other on the GPUs.
    Because a replica's all-reduce waits for every other replica, all replicas' work is always
    LAUNCHED before the host waits on any of them (fused.FusedReplicas).
    """

    def __init__(self, devices, batch: int = 64, lr: float = 0.1, momentum: float = 0.9, weight_decay: float = 1e-4,
                 seed: int = 1, init_model=None, use_graph: bool = True, steps_per_graph: int | None = None,
                 blocks: int = 64):
        from ..engine import FusedMnistTrainer
        from ..models.mnist_cnn import MnistCNN

        if init_model is None:
            torch.manual_seed(seed)
            init_model = MnistCNN()
        self.batch = batch
        super().__init__(devices, lambda d, pc: FusedMnistTrainer(
            batch=batch, device=d, comm=None, peer=pc, seed=seed, lr=lr, momentum=momentum, weight_decay=weight_decay,
            init_model=init_model, use_graph=use_graph, graph_mode=1, steps_per_graph=steps_per_graph),
            blocks=blocks, peer_bytes=32 << 20)
