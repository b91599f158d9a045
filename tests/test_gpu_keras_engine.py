"""Fused native Keras-CNN step (csrc/keras_kernels.hip) vs a plain PyTorch fp32 reference of the
same model (models.KerasCNN on the CPU): same weights, same batches, several Adam steps -- the
loss of every step and the parameters after them.  Plus graph == eager, training on the on-device
data stream, and in-process replicas (MirroredStrategy parity) == one trainer on the global batch.
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


def _ref_run(model, batches, lr, eps_hat):
    """CPU fp32 reference: torch.optim.Adam (eps_hat=False) or the Keras epsilon-hat Adam."""
    from mxddp.optim import Adam as FlatAdam
    from mxddp.parallel.flat import FlatParams

    if eps_hat:
        flat = FlatParams(model, torch.device("cpu"))
        opt = FlatAdam(flat, lr=lr, eps=1e-7, eps_hat=True)
    else:
        opt = torch.optim.Adam(model.parameters(), lr=lr, eps=1e-7)
    losses = []
    for x, y in batches:
        opt.zero_grad()
        loss = F.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    return losses


@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("eps_hat", [False, True])
@pytest.mark.parametrize("B", [64, 24])
def test_fused_keras_matches_reference(cuda, graph, eps_hat, B):
    from mxddp.keras_engine import FusedKerasTrainer
    from mxddp.models import KerasCNN

    torch.manual_seed(0)
    ref = KerasCNN()
    init = {k: v.clone() for k, v in ref.state_dict().items()}
    steps, lr = 5, 2e-3
    batches = _batches(steps, B)
    m0 = KerasCNN()
    m0.load_state_dict(init)
    tr = FusedKerasTrainer(batch=B, device=cuda, lr=lr, eps=1e-7, eps_hat=eps_hat, use_graph=graph, init_model=m0)
    losses = []
    for x, y in batches:
        tr.set_batch(x.to(cuda), y.to(cuda))
        tr.step(1)
        ls, _ = tr.read_metrics()
        losses.append(ls / B)
    ref_losses = _ref_run(ref, batches, lr, eps_hat)
    for a, b in zip(losses, ref_losses):
        assert abs(a - b) < 1e-4 * max(1.0, abs(b)), (losses, ref_losses)
    assert tr.adam_steps == steps
    sd = tr.state_dict()
    for k, v in ref.state_dict().items():
        assert torch.allclose(sd[k], v, rtol=1e-3, atol=2e-5), (k, (sd[k] - v).abs().max())
    moved = max((sd[k] - init[k]).abs().max().item() for k in init)
    assert moved > 1e-3


@pytest.mark.parametrize("graph", [False, True])
def test_fused_keras_rccl_collectives_ws1(cuda, graph):
    """The DDP path of the fused Keras step with REAL RCCL all-reduces (1-rank communicator,
    collectives forced): finalize into g, the 373 KB bucket all-reduced, Adam from g -- eager and
    captured in the step graph -- against the CPU Adam reference."""
    from mxddp import native
    from mxddp.keras_engine import FusedKerasTrainer
    from mxddp.models import KerasCNN

    C = native()
    comm = C.Comm(C.Comm.new_unique_id(), 0, 1, cuda.index or 0)
    torch.manual_seed(0)
    ref = KerasCNN()
    init = {k: v.clone() for k, v in ref.state_dict().items()}
    steps, lr, B = 4, 2e-3, 32
    batches = _batches(steps, B, seed=5)
    m0 = KerasCNN()
    m0.load_state_dict(init)
    tr = FusedKerasTrainer(batch=B, device=cuda, lr=lr, eps=1e-7, comm=comm, force_collectives=True,
                           use_graph=graph, graph_mode=1 if graph else 0, init_model=m0)
    assert tr.eng.reducer_active and tr.active_transport == "rccl:default"
    losses = []
    for x, y in batches:
        tr.set_batch(x.to(cuda), y.to(cuda))
        tr.step(1)
        losses.append(tr.read_metrics()[0] / B)
    assert tr.eng.captured == graph
    ref_losses = _ref_run(ref, batches, lr, True)
    for a, b in zip(losses, ref_losses):
        assert abs(a - b) < 1e-4 * max(1.0, abs(b)), (losses, ref_losses)
    sd = tr.state_dict()
    for k, v in ref.state_dict().items():
        assert torch.allclose(sd[k], v, rtol=1e-3, atol=2e-5), (k, (sd[k] - v).abs().max())


def test_fused_keras_autotune_ws1(cuda):
    """autotune() of the Keras engine (RCCL variants x eager / graph, collectives forced at one
    rank) only changes how the step is launched: the trained weights equal an untuned engine's."""
    from mxddp import native
    from mxddp.keras_engine import FusedKerasTrainer

    C = native()
    comm = C.Comm(C.Comm.new_unique_id(), 0, 1, cuda.index or 0)
    a = FusedKerasTrainer(batch=64, device=cuda, lr=1e-3, comm=comm, force_collectives=True)
    b = FusedKerasTrainer(batch=64, device=cuda, lr=1e-3)
    a.step(1)
    res = a.autotune(trial_steps=3, include_graphs=True)
    assert len(res) == 2 and a.tuned["buckets"] == "one"  # {eager, graph} x {one}
    assert a.steps == 1  # the trial steps are scratch (restored)
    a.step(5)
    b.step(1 + 5)
    assert a.steps == b.steps and a.adam_steps == b.adam_steps
    for k, v in a.state_dict().items():
        assert torch.equal(v, b.state_dict()[k]), k


def test_fused_keras_trains_on_device_stream(cuda):
    from mxddp.keras_engine import FusedKerasTrainer

    tr = FusedKerasTrainer(batch=64, device=cuda, lr=1e-3)
    tr.step(5)
    l0, _ = tr.read_metrics()
    tr.step(300)
    tr.read_metrics()
    tr.step(20)
    l1, c1 = tr.read_metrics()
    assert l1 / (20 * 64) < 0.5 * l0 / (5 * 64)
    assert c1 / (20 * 64) > 0.8


def test_fused_keras_graph_equals_eager_synthetic(cuda):
    """Multi-step graphs (8 per graph + remainders) over the on-device data stream == eager steps."""
    from mxddp.keras_engine import FusedKerasTrainer

    a = FusedKerasTrainer(batch=64, device=cuda, lr=1e-3, steps_per_graph=8)
    b = FusedKerasTrainer(batch=64, device=cuda, lr=1e-3, use_graph=False)
    for n in (1, 13, 3):
        a.step(n)
        b.step(n)
    la, ca = a.read_metrics()
    lb, cb = b.read_metrics()
    assert abs(la - lb) < 1e-4 * abs(lb) and ca == cb
    for k, v in a.state_dict().items():
        assert torch.equal(v, b.state_dict()[k]), k  # deterministic kernels: bit-identical


def test_fused_keras_state_roundtrip(cuda):
    from mxddp.keras_engine import FusedKerasTrainer

    a = FusedKerasTrainer(batch=32, device=cuda, lr=1e-3, use_graph=False)
    a.step(3)
    m = a.to_module()
    b = FusedKerasTrainer(batch=32, device=cuda, lr=1e-3, use_graph=False, init_model=m)
    b.load_optimizer_state(a.optimizer_state())
    b.load_data_state(a.data_state())
    a.step(2)
    b.step(2)
    for k, v in a.state_dict().items():
        assert torch.equal(v, b.state_dict()[k]), k


def _replicas_worker(graph, q):
    try:
        from mxddp.keras_engine import FusedKerasReplicas, FusedKerasTrainer
        from mxddp.models import KerasCNN

        cuda = torch.device("cuda", 0)
        torch.manual_seed(0)
        init = KerasCNN()
        b, steps = 32, 4
        batches = _batches(steps, 2 * b, seed=11)
        rep = FusedKerasReplicas([cuda, cuda], batch=b, lr=2e-3, init_model=init, use_graph=graph)
        for x, y in batches:
            rep.set_batch(x.to(cuda), y.to(cuda))
            rep.step(1)
        rep.synchronize()
        p0, p1 = rep.trainers[0].params.cpu(), rep.trainers[1].params.cpu()
        bad = []
        if not torch.equal(p0, p1):
            bad.append("replicas diverged")
        ref = FusedKerasTrainer(batch=2 * b, device=cuda, lr=2e-3, init_model=init, use_graph=False)
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
def test_fused_keras_replicas_match_global_batch(cuda, graph):
    """MirroredStrategy parity on the fused engine: two in-process replicas (both on the one GPU
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


def test_tensorboard_profile_batch_has_device_kernels(cuda, tmp_path):
    """TF2 TensorBoard profile_batch parity on the GPU path: the trace of batch 2 holds the fused
    engine's HIP kernels (device activity from the ROCm tracer), not only host events."""
    import glob
    import gzip
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    td = tmp_path / "tb"
    r = subprocess.run([sys.executable, "-m", "mxddp.train", "--model", "keras_cnn", "-e", "1", "--steps-per-epoch", "6",
                        "--log-interval", "1", "-b", "32", "--tensorboard-dir", str(td)],
                       cwd=root, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    traces = glob.glob(str(td / "plugins" / "profile" / "*" / "*.trace.json.gz"))
    assert len(traces) == 1, traces
    ev = json.loads(gzip.open(traces[0]).read())["traceEvents"]
    kernels = [e.get("name", "") for e in ev if e.get("cat") == "kernel"]
    assert any("keras" in k for k in kernels), sorted(set(kernels))[:20]
