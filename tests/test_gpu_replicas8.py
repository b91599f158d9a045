"""BASELINE config 4 at the node's width: EIGHT in-process replicas (MirroredStrategy over all
local GPUs, tensorflow2/mnist_mirror_strategy.py:12,68-79; DataParallel / ParallelUpdater) of each
fused engine -- MNIST CNN + SGD, Keras CNN + Keras Adam (exchange co-scheduled with Adam), Chainer
MLP + Chainer Adam -- trained on the eight slices of a global batch == ONE trainer on the whole
batch, eager and captured in hipGraphs.

Here all eight replicas share the one GPU (each on its own stream; the test process gets 32 HIP
hardware queues -- the most gpurun allows -- so no two replicas' streams share a queue and no
replica's exchange kernel waits behind another's; with 8 queues, stream k of the process lands on
queue k mod 8 and replicas 0 and 4 collided), which exercises the
8-way ``open_local`` mesh, per-replica flag sets and the rank-ordered sums exactly as on an 8-GPU
node, minus the links.
"""
import os
import traceback

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N_REP = 8


def _worker(model, graph, q):
    try:
        cuda = torch.device("cuda", 0)
        torch.manual_seed(0)
        b, steps = 16, 3
        devs = [cuda] * N_REP
        if model == "mnist":
            from mxddp.engine import FusedMnistTrainer as T
            from mxddp.models import MnistCNN as M
            from mxddp.parallel.replica import FusedMnistReplicas

            init, lr = M(), 0.05
            rep = FusedMnistReplicas(devs, batch=b, lr=lr, init_model=init, use_graph=graph)
        elif model == "keras":
            from mxddp.keras_engine import FusedKerasReplicas
            from mxddp.keras_engine import FusedKerasTrainer as T
            from mxddp.models import KerasCNN as M

            init, lr = M(), 2e-3
            rep = FusedKerasReplicas(devs, batch=b, lr=lr, init_model=init, use_graph=graph)
        else:
            from mxddp.mlp_engine import FusedMlpReplicas
            from mxddp.mlp_engine import FusedMlpTrainer as T
            from mxddp.models import MLP as M

            init, lr = M(), 2e-3
            rep = FusedMlpReplicas(devs, batch=b, lr=lr, init_model=init, use_graph=graph)
        g = torch.Generator().manual_seed(13)
        batches = [(torch.rand(N_REP * b, 1, 28, 28, generator=g), torch.randint(0, 10, (N_REP * b,), generator=g))
                   for _ in range(steps)]
        for x, y in batches:
            rep.set_batch(x.to(cuda), y.to(cuda))
            rep.step(1)
        rep.synchronize()
        bad = []
        ps = [t.params.cpu() for t in rep.trainers]
        if any(not torch.equal(ps[0], p) for p in ps[1:]):
            bad.append("replicas diverged")
        ref = T(batch=N_REP * b, device=cuda, lr=lr, init_model=init, use_graph=False)
        for x, y in batches:
            ref.set_batch(x.to(cuda), y.to(cuda))
            ref.step(1)
        ref.synchronize()
        p0 = torch.cat([v.reshape(-1) for v in init.state_dict().values()])
        moved = (ref.params.cpu() - p0).norm().item()
        d = ((ref.params.cpu() - ps[0]).norm() / max(moved, 1e-12)).item()
        # relative to how far the steps moved the weights: summation-order noise only
        if not d < (1e-4 if model == "mnist" else 1e-3) or not moved > 1e-4:
            bad.append(("replicas != global batch", d, moved))
        ls, _ = rep.read_metrics()
        lr_, _ = ref.read_metrics()
        if not abs(ls - lr_) < 1e-3 * abs(lr_):
            bad.append(("loss", ls, lr_))
        q.put(bad)
    except Exception:
        q.put(["exception: " + traceback.format_exc()])


@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("model", ["mnist", "keras", "mlp"])
def test_eight_fused_replicas_match_global_batch(cuda, model, graph):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    old = os.environ.get("GPU_MAX_HW_QUEUES")
    os.environ["GPU_MAX_HW_QUEUES"] = "32"
    try:
        p = ctx.Process(target=_worker, args=(model, graph, q))
        p.start()
    finally:
        if old is None:
            del os.environ["GPU_MAX_HW_QUEUES"]
        else:
            os.environ["GPU_MAX_HW_QUEUES"] = old
    try:
        bad = q.get(timeout=200)
    finally:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert bad == [], bad


def _group_worker(graph, q):
    try:
        from mxddp import ops
        from mxddp.models import build_model
        from mxddp.optim import SGD
        from mxddp.parallel.replica import ReplicaGroup

        cuda = torch.device("cuda", 0)
        n, b = 4, 8
        loss_fn = lambda o, t: ops.cross_entropy(o, t, return_correct=True)  # noqa: E731
        g = torch.Generator().manual_seed(17)
        batches = [(torch.rand(n * b, 1, 28, 28, generator=g), torch.randint(0, 10, (n * b,), generator=g))
                   for _ in range(5)]
        res = []
        for devs in ([cuda] * n, [cuda]):
            torch.manual_seed(0)
            grp = ReplicaGroup(build_model("keras_cnn"), devs, lambda f: SGD(f, lr=0.05, momentum=0.9, weight_decay=1e-4),
                               use_graph=graph and len(devs) > 1, bucket_cap_mb=0.05)
            for x, y in batches:
                grp.step(x.to(cuda), y.to(cuda), loss_fn)
            ls, _ = grp.read_metrics()
            res.append((grp, ls))
        (grp, ls), (ref, lr_) = res
        bad = []
        if graph and (grp._graphs is None or len(grp.buckets) < 4):
            bad.append(("not graphed / bucketed", grp._graphs is None, getattr(grp, "buckets", None)))
        ps = [f.data.cpu() for f in grp.flats]
        if any(not torch.equal(ps[0], p) for p in ps[1:]):
            bad.append("replicas diverged")
        d = (ps[0] - ref.flats[0].data.cpu()).abs().max().item()
        if not d < 1e-4:
            bad.append(("replicas != global batch", d))
        if not abs(ls - lr_) < 1e-3 * abs(lr_):
            bad.append(("loss", ls, lr_))
        q.put(bad)
    except Exception:
        q.put(["exception: " + traceback.format_exc()])


@pytest.mark.parametrize("graph", [False, True])
def test_replica_group_shared_gpu_bucketed_exchange(cuda, graph):
    """The layer-path replica group (DataParallel / MirroredStrategy for any model) with 4 replicas
    on the one GPU: eager steps exchange over the in-process peer transport; graph mode captures
    each replica's step with the DDP bucket reducer over the peer transport, so the gradient leaves
    bucket by bucket during the backward (here ~8 buckets of 50 KB) -- both == one replica on the
    global batch."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    old = os.environ.get("GPU_MAX_HW_QUEUES")
    os.environ["GPU_MAX_HW_QUEUES"] = "32"
    try:
        p = ctx.Process(target=_group_worker, args=(graph, q))
        p.start()
    finally:
        if old is None:
            del os.environ["GPU_MAX_HW_QUEUES"]
        else:
            os.environ["GPU_MAX_HW_QUEUES"] = old
    try:
        bad = q.get(timeout=200)
    finally:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert bad == [], bad
