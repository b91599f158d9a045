"""T3: GPU paths of the parallel layer at world_size 1 on one MI355X: mxddp DDP (RCCL reducer
with its side stream and event fences, no peers), replica group on one device, and the
layer-by-layer trainer vs a plain torch fp32 reference."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def test_ddp_reducer_ws1_matches_torch(cuda):
    from mxddp import ops
    from mxddp.models import build_model
    from mxddp.optim import SGD
    from mxddp.parallel import comm
    from mxddp.parallel.ddp import DistributedDataParallel as DDP

    comm.init_distributed(use_gpu=True)
    torch.manual_seed(0)
    ref = build_model("mlp")
    m = build_model("mlp")
    m.load_state_dict(ref.state_dict())
    ddp = DDP(m.to(cuda), timing=True)
    opt = SGD(ddp.flat, lr=0.05, momentum=0.9, weight_decay=1e-4)
    ropt = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    g = torch.Generator().manual_seed(1)
    for _ in range(3):
        x, y = torch.rand(32, 1, 28, 28, generator=g), torch.randint(0, 10, (32,), generator=g)
        opt.zero_grad()
        ops.cross_entropy(ddp(x.to(cuda)), y.to(cuda)).backward()
        opt.step()
        ropt.zero_grad()
        F.cross_entropy(ref(x), y).backward()
        ropt.step()
    torch.cuda.synchronize()
    assert ddp.reducer.launched == ddp.reducer.num_buckets  # every bucket went through the reducer
    for (k, a), b in zip(m.state_dict().items(), ref.state_dict().values()):
        assert torch.allclose(a.cpu(), b, rtol=1e-4, atol=1e-5), k


def test_replica_group_single_device(cuda):
    from mxddp import ops
    from mxddp.models import build_model
    from mxddp.optim import Adam
    from mxddp.parallel.replica import ReplicaGroup

    torch.manual_seed(0)
    grp = ReplicaGroup(build_model("keras_cnn"), [cuda], lambda f: Adam(f, lr=1e-3, eps=1e-7, eps_hat=True))
    x = torch.rand(16, 1, 28, 28, device=cuda)
    y = torch.randint(0, 10, (16,), device=cuda)
    grp.step(x, y, lambda o, t: ops.cross_entropy(o, t, return_correct=True))
    l0, _ = grp.read_metrics()
    for _ in range(20):
        grp.step(x, y, lambda o, t: ops.cross_entropy(o, t, return_correct=True))
        ls, c = grp.read_metrics()
    assert ls < l0 and 0 <= c <= 16


@pytest.mark.parametrize("model", ["keras_cnn", "mlp"])
def test_replica_group_graph_matches_eager(cuda, model):
    """use_graph=True (per-device hipGraph of the whole step -- zero-grad, forward, backward,
    Adam with its on-device step count, metric accumulation -- after two eager steps, fresh
    batches copied into static inputs) trains exactly like the eager replica step."""
    from mxddp import ops
    from mxddp.models import build_model
    from mxddp.optim import Adam
    from mxddp.parallel.replica import ReplicaGroup

    loss_fn = lambda o, t: ops.cross_entropy(o, t, return_correct=True)  # noqa: E731
    g = torch.Generator().manual_seed(3)
    batches = [(torch.rand(32, 1, 28, 28, generator=g), torch.randint(0, 10, (32,), generator=g)) for _ in range(6)]
    res = []
    for graph in (False, True):
        torch.manual_seed(0)
        grp = ReplicaGroup(build_model(model), [cuda], lambda f: Adam(f, lr=1e-3, eps=1e-7, eps_hat=True),
                           use_graph=graph)
        losses = []
        for x, y in batches:
            grp.step(x.to(cuda), y.to(cuda), loss_fn)
            losses.append(grp.read_metrics()[0])
        assert (grp._graphs is not None) == graph
        res.append((losses, grp.flats[0].data.cpu()))
    (la, pa), (lb, pb) = res
    assert max(abs(a - b) for a, b in zip(la, lb)) < 1e-4 * max(abs(a) for a in la)
    assert torch.allclose(pa, pb, rtol=1e-4, atol=1e-6)
    assert grp.optimizers[0].steps == len(batches)  # the device step count advanced in the graph


@pytest.mark.parametrize("name", ["pyramidnet110", "resnet50"])
def test_model_forward_backward_vs_torch(cuda, name):
    """Full-model numerics: mxddp HIP path (fp32) vs a float64 CPU reference on the same weights
    and batch, judged against stock PyTorch-ROCm's own fp32 GPU error on the same problem."""
    import copy

    from mxddp import ops
    from mxddp.models import build_model

    torch.manual_seed(0)
    m = build_model(name)
    # batch 8: BN backward at tiny batch is a catastrophic cancellation of three nearly equal
    # terms, which amplifies summation-order noise in ANY fp32 implementation
    shape = (8, 3, 32, 32) if name == "pyramidnet110" else (8, 3, 64, 64)
    x = torch.randn(shape)
    y = torch.randint(0, 10, (8,))
    m64 = copy.deepcopy(m).double()
    ref_loss = F.cross_entropy(m64(x.double()), y)
    ref_loss.backward()
    ref = torch.cat([p.grad.reshape(-1).float().clone() for p in m64.parameters()])
    mg = m.to(cuda)

    def grads(reference_mode):
        mg.zero_grad()
        if reference_mode:  # stock PyTorch-ROCm (MIOpen/hipBLASLt) on the same GPU
            with ops.torch_reference_mode():
                loss = F.cross_entropy(mg(x.to(cuda)), y.to(cuda))
                loss.backward()
        else:
            loss = ops.cross_entropy(mg(x.to(cuda)), y.to(cuda))
            loss.backward()
        torch.cuda.synchronize()
        return loss.item(), torch.cat([p.grad.reshape(-1).cpu() for p in mg.parameters()])

    loss, got = grads(False)
    tloss, tgpu = grads(True)
    ref_l = ref_loss.item()
    assert abs(loss - ref_l) < max(1e-3 * max(1.0, abs(ref_l)), 3 * abs(tloss - ref_l)), (loss, tloss, ref_l)
    rel = ((got - ref).norm() / ref.norm()).item()  # whole-model gradient, relative L2
    # deep nets amplify fp32 summation-order noise; the bar is "no worse than stock
    # PyTorch-ROCm's own GPU kernels are vs the CPU" (with a floor)
    rel_torch = ((tgpu - ref).norm() / ref.norm()).item()
    assert rel < max(2e-3, 3 * rel_torch), (rel, rel_torch)
    cos = torch.nn.functional.cosine_similarity(got, ref, dim=0).item()
    assert cos > 0.9995, cos


@pytest.mark.parametrize("model,extra", [("mnist_cnn", ["--per-rank-batch", "64"]),
                                         ("keras_cnn", ["--per-rank-batch", "32"]),
                                         ("mlp", ["--per-rank-batch", "32"])])
def test_train_cli_two_ranks_share_gpu(cuda, tmp_path, model, extra):
    """The reference DDP launch (one process per rank, reference flags) with two ranks on the one
    GPU: RCCL cannot span them, so the DDP gradient exchange is the peer transport -- each model
    on its fused engine (train.py routes mnist_cnn, keras_cnn and mlp there) with the autotuned
    DDP step.  Both ranks' reference-layout checkpoints must be identical (the global-batch
    equivalence of the fused DDP steps is checked in test_gpu_peer.py / test_gpu_keras_engine.py)."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root)
    cmd = [sys.executable, "-m", "mxddp.train", "--model", model, "--nproc-per-node", "2", "-e", "1",
           "--steps-per-epoch", "20", "--log-interval", "10", "-td", str(tmp_path), "-sm"] + extra
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    a = torch.load(tmp_path / "distributed_data_parallel_0.pth", weights_only=True)
    b = torch.load(tmp_path / "distributed_data_parallel_1.pth", weights_only=True)
    for k in a:
        assert torch.equal(a[k], b[k]), k
    assert "From Rank: 1, Training time" in p.stdout


@pytest.mark.parametrize("script,argv,expect", [
    ("chainer/train_mnist.py", ["--gpu", "0", "-e", "1"], "engine fused"),
    ("chainer/train_mnist_gpu.py", ["--gpu", "-e", "1"], "replica mode (fused mlp engine)"),
])
def test_chainer_examples_run_fused_engine_at_reference_batch(cuda, tmp_path, script, argv, expect):
    """The reference's Chainer launch lines with their DEFAULT batch sizes (100 for
    train_mnist.py, 400 on --gpu_number 1 for train_mnist_gpu.py) run the native fused MLP step,
    not the generic layer path (the engine pads the partial last 16-row tile)."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root)
    cmd = [sys.executable, os.path.join(root, "examples", script)] + argv + ["-o", str(tmp_path / "out")]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=tmp_path)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert expect in p.stdout, p.stdout[-3000:]
