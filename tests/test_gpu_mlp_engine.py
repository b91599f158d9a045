"""Fused native Chainer-MLP step (csrc/mlp_kernels.hip) vs a plain PyTorch fp32 reference of the
same model (models.MLP math on the CPU, Chainer epsilon-hat Adam): same weights, same batches,
several steps -- the loss of every step and the parameters after them.  Plus graph == eager
bit for bit, the RCCL / DDP path (gradients all-reduced, then the flat Adam), training on the
on-device data stream, the state round trip, and in-process replicas (Chainer ParallelUpdater,
chainer/train_mnist_gpu.py:87-93) == one trainer on the global batch.
"""
import os
import traceback

import pytest
import torch
import torch.multiprocessing as mp
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _batches(steps, B, seed=3):
    g = torch.Generator().manual_seed(seed)
    return [(torch.rand(B, 1, 28, 28, generator=g), torch.randint(0, 10, (B,), generator=g)) for _ in range(steps)]


def _ref_run(sd, batches, lr):
    """CPU fp32 reference: the MLP forward in plain torch ops, Chainer's epsilon-hat Adam
    (mxddp.optim.Adam CPU path), softmax cross entropy (L.Classifier)."""
    from mxddp.models import MLP
    from mxddp.optim import Adam as FlatAdam
    from mxddp.parallel.flat import FlatParams

    model = MLP()
    model.load_state_dict(sd)

    def fwd(x):
        h = F.relu(F.linear(x.flatten(1), model.l1.weight, model.l1.bias))
        h = F.relu(F.linear(h, model.l2.weight, model.l2.bias))
        return F.linear(h, model.l3.weight, model.l3.bias)

    flat = FlatParams(model, torch.device("cpu"))
    opt = FlatAdam(flat, lr=lr, eps=1e-8, eps_hat=True)
    losses = []
    for x, y in batches:
        opt.zero_grad()
        loss = F.cross_entropy(fwd(x), y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    return losses, model.state_dict()


def _check(tr, batches, lr, B, init):
    losses = []
    for x, y in batches:
        tr.set_batch(x.to(tr.device), y.to(tr.device))
        tr.step(1)
        ls, _ = tr.read_metrics()
        losses.append(ls / B)
    ref_losses, ref_sd = _ref_run(init, batches, lr)
    for a, b in zip(losses, ref_losses):
        assert abs(a - b) < 1e-4 * max(1.0, abs(b)), (losses, ref_losses)
    assert tr.adam_steps == len(batches)
    sd = tr.state_dict()
    # the parameters relative to how far the 5 steps moved them (the losses above match at 1e-4):
    # Adam divides each update by its own sqrt(v), so a gradient element that is rounding noise in
    # both implementations still moves its weight by ~lr -- an elementwise fp32 tolerance would
    # test that noise, not the step
    for k, v in ref_sd.items():
        step = (v - init[k]).norm()
        assert (sd[k] - v).norm() <= 1e-3 * step, (k, ((sd[k] - v).norm() / step).item())
    moved = max((sd[k] - init[k]).abs().max().item() for k in init)
    assert moved > 1e-4


@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("B", [64, 16, 128, 100, 200, 4, 512])
def test_fused_mlp_matches_reference(cuda, graph, B):
    """Whole 16-row tiles and the reference's own batches: 100 (chainer/train_mnist.py:31) and 200
    per device (ParallelUpdater's 400 over 2 GPUs, chainer/train_mnist_gpu.py:33); 200 and 512 run
    the backward kernels' batch in several LDS passes."""
    from mxddp.mlp_engine import FusedMlpTrainer
    from mxddp.models import MLP

    torch.manual_seed(0)
    m0 = MLP()
    init = {k: v.clone() for k, v in m0.state_dict().items()}
    lr = 2e-3
    tr = FusedMlpTrainer(batch=B, device=cuda, lr=lr, use_graph=graph, init_model=m0)
    _check(tr, _batches(5, B), lr, B, init)


@pytest.mark.parametrize("merged", [False, True])
@pytest.mark.parametrize("graph", [False, True])
def test_fused_mlp_rccl_collectives_ws1(cuda, graph, merged):
    """The DDP path with REAL RCCL all-reduces (1-rank communicator, collectives forced): K4 / K5
    write the gradients, the two buckets (or one merged bucket) are all-reduced, the flat Adam
    updates -- eager and captured in the step graph."""
    from mxddp import native
    from mxddp.mlp_engine import FusedMlpTrainer
    from mxddp.models import MLP

    C = native()
    comm = C.Comm(C.Comm.new_unique_id(), 0, 1, cuda.index or 0)
    torch.manual_seed(0)
    m0 = MLP()
    init = {k: v.clone() for k, v in m0.state_dict().items()}
    lr, B = 2e-3, 32
    tr = FusedMlpTrainer(batch=B, device=cuda, lr=lr, comm=comm, use_graph=graph, graph_mode=1 if graph else 0,
                         init_model=m0, force_collectives=True)
    tr._set_buckets("one" if merged else "ovl")
    assert tr.eng.reducer_active and tr.eng.merged == merged
    _check(tr, _batches(4, B, seed=9), lr, B, init)


def test_fused_mlp_deterministic_and_graph_equals_eager(cuda):
    """Multi-step graphs (8 per graph + remainders) over the on-device data stream == eager steps,
    bit for bit, and two runs are identical (no order-dependent float atomics)."""
    from mxddp.mlp_engine import FusedMlpTrainer

    runs = []
    for graph, spg in ((True, 8), (True, 8), (False, None)):
        t = FusedMlpTrainer(batch=64, device=cuda, lr=1e-3, use_graph=graph, steps_per_graph=spg)
        for n in (1, 13, 3):
            t.step(n)
        runs.append((t.state_dict(), t.read_metrics(), t.adam_steps))
    (sa, ma, na), (sb, mb, nb), (sc, mc, nc) = runs
    assert ma == mb == mc and na == nb == nc == 17
    for k in sa:
        assert torch.equal(sa[k], sb[k]) and torch.equal(sa[k], sc[k]), k


@pytest.mark.parametrize("B", [64, 16, 200, 512])
@pytest.mark.parametrize("graph", [True, False])
def test_w2_update_in_k5_is_bitwise_equal(cuda, graph, B):
    """mlp_set_w2_defer: the dW2 tile + Adam run as extra resident blocks of K5 (K4 keeps the
    dgrad) -- the same operands and MFMA sequence as K4's folded path, so 12 steps train bit for
    bit alike (200 / 512: several LDS passes in both places)."""
    from mxddp import native
    from mxddp.mlp_engine import FusedMlpTrainer

    C = native()
    assert C.mlp_w2_defer() == 0
    runs = []
    try:
        for on in (1, 0):
            C.mlp_set_w2_defer(on)
            t = FusedMlpTrainer(batch=B, device=cuda, lr=1e-3, use_graph=graph)
            t.step(12)
            runs.append((t.state_dict(), t.read_metrics()))
    finally:
        C.mlp_set_w2_defer(0)
    for k, v in runs[0][0].items():
        assert torch.equal(v, runs[1][0][k]), (k, (v - runs[1][0][k]).abs().max().item())
    assert runs[0][1] == runs[1][1]


@pytest.mark.parametrize("merged", [True, False])
def test_w2_gradient_in_k5_with_collectives(cuda, merged):
    """With gradient collectives forced at one rank: the merged bucket lets K5's W2 blocks write
    the l2 gradient (bitwise equal to K4 writing it); the two-bucket strategy keeps it in K4 (its
    bucket is all-reduced while K5 runs)."""
    from mxddp import native
    from mxddp.mlp_engine import FusedMlpTrainer

    C = native()
    comm = C.Comm(C.Comm.new_unique_id(), 0, 1, cuda.index or 0)
    sds = []
    try:
        for on in (1, 0):
            C.mlp_set_w2_defer(on)
            t = FusedMlpTrainer(batch=32, device=cuda, lr=1e-3, comm=comm, force_collectives=True, use_graph=False)
            t._set_buckets("one" if merged else "ovl")
            t.step(8)
            t.synchronize()
            sds.append(t.state_dict())
    finally:
        C.mlp_set_w2_defer(0)
    for k, v in sds[0].items():
        assert torch.equal(v, sds[1][k]), (k, (v - sds[1][k]).abs().max().item())


def test_fused_mlp_trains_on_device_stream(cuda):
    from mxddp.mlp_engine import FusedMlpTrainer

    tr = FusedMlpTrainer(batch=64, device=cuda, lr=1e-3)
    tr.step(5)
    l0, _ = tr.read_metrics()
    tr.step(300)
    tr.read_metrics()
    tr.step(20)
    l1, c1 = tr.read_metrics()
    assert l1 / (20 * 64) < 0.5 * l0 / (5 * 64)
    assert c1 / (20 * 64) > 0.8


def test_fused_mlp_state_roundtrip(cuda):
    from mxddp.mlp_engine import FusedMlpTrainer

    a = FusedMlpTrainer(batch=32, device=cuda, lr=1e-3, use_graph=False)
    a.step(3)
    b = FusedMlpTrainer(batch=32, device=cuda, lr=1e-3, use_graph=False, init_model=a.to_module())
    b.load_optimizer_state(a.optimizer_state())
    b.load_data_state(a.data_state())
    a.step(2)
    b.step(2)
    for k, v in a.state_dict().items():
        assert torch.equal(v, b.state_dict()[k]), k


def _replicas_worker(graph, q):
    try:
        from mxddp.mlp_engine import FusedMlpReplicas, FusedMlpTrainer
        from mxddp.models import MLP

        cuda = torch.device("cuda", 0)
        torch.manual_seed(0)
        init = MLP()
        b, steps = 32, 4
        batches = _batches(steps, 2 * b, seed=11)
        rep = FusedMlpReplicas([cuda, cuda], batch=b, lr=2e-3, init_model=init, use_graph=graph)
        for x, y in batches:
            rep.set_batch(x.to(cuda), y.to(cuda))
            rep.step(1)
        rep.synchronize()
        p0, p1 = rep.trainers[0].params.cpu(), rep.trainers[1].params.cpu()
        bad = []
        if not torch.equal(p0, p1):
            bad.append("replicas diverged")
        ref = FusedMlpTrainer(batch=2 * b, device=cuda, lr=2e-3, init_model=init, use_graph=False)
        for x, y in batches:
            ref.set_batch(x.to(cuda), y.to(cuda))
            ref.step(1)
        ref.synchronize()
        d = (ref.params.cpu() - p0).abs().max().item()
        if not d < 5e-5:
            bad.append(("replicas != global batch", d))
        ls, _ = rep.read_metrics()
        lr_, _ = ref.read_metrics()
        if not abs(ls - lr_) < 1e-3 * abs(lr_):
            bad.append(("loss", ls, lr_))
        q.put(bad)
    except Exception:
        q.put(["exception: " + traceback.format_exc()])


@pytest.mark.parametrize("graph", [False, True])
def test_fused_mlp_replicas_match_global_batch(cuda, graph):
    """ParallelUpdater parity on the fused engine: two in-process replicas (both on the one GPU
    here, 8 HW queues so one replica's all-reduce never sits behind the other's) on the halves of
    a global batch == one trainer on the whole batch."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    old = os.environ.get("GPU_MAX_HW_QUEUES")
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
    try:
        p = ctx.Process(target=_replicas_worker, args=(graph, q))
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
