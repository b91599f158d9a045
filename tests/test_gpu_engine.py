"""Fused native MNIST step vs the layer-by-layer PyTorch fp32 reference (same weights,
same batch): loss, gradients and updated parameters after several SGD steps."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref_steps(model, xs, ys, steps, lr=0.1, mom=0.9, wd=1e-4):
    opt = torch.optim.SGD(model.parameters(), lr=lr, momentum=mom, weight_decay=wd)
    losses = []
    for i in range(steps):
        opt.zero_grad()
        loss = F.cross_entropy(model(xs[i]), ys[i])
        loss.backward()
        opt.step()
        losses.append(loss.item())
    return losses


@pytest.mark.parametrize("variant", [0, 1])
@pytest.mark.parametrize("graph", [0, 1, 2])
def test_fused_engine_matches_reference(cuda, variant, graph):
    from mxddp.engine import FusedMnistTrainer
    from mxddp.models import MnistCNN

    torch.manual_seed(0)
    ref = MnistCNN()  # CPU, torch ops
    B, steps = 32, 4
    tr = FusedMnistTrainer(batch=B, device=cuda, comm=None, init_model=ref, variant=variant, use_graph=graph > 0,
                           graph_mode=graph if graph else None)
    xs = [torch.rand(B, 1, 28, 28) for _ in range(steps)]
    ys = [torch.randint(0, 10, (B,)) for _ in range(steps)]
    losses = []
    for i in range(steps):
        tr.set_batch(xs[i].to(cuda), ys[i].to(cuda))
        tr.step(1)
        ls, _ = tr.read_metrics()
        losses.append(ls / B)
    ref_losses = _ref_steps(ref, xs, ys, steps)
    for a, b in zip(losses, ref_losses):
        assert abs(a - b) < 1e-4 * max(1.0, abs(b)), (losses, ref_losses)
    sd = tr.state_dict()
    for k, v in ref.state_dict().items():
        err = (sd[k] - v).abs().max().item() / (v.abs().max().item() + 1e-6)
        assert err < 1e-4, (k, err)


@pytest.mark.parametrize("B", [16, 48, 64, 128, 8, 1, 100, 37])
def test_fused_engine_batch_sizes_match_reference(cuda, B):
    """Batches the fused engine accepts (1..128) against the fp32 reference: whole 16-row tiles,
    and partial last tiles whose pad rows must add nothing (8 = the reference DDP CLI's -b 64
    over 8 local ranks, pytorch/distributed_data_parallel.py:71)."""
    from mxddp.engine import FusedMnistTrainer
    from mxddp.models import MnistCNN

    torch.manual_seed(0)
    ref = MnistCNN()
    steps = 3
    tr = FusedMnistTrainer(batch=B, device=cuda, comm=None, init_model=ref, use_graph=False)
    g = torch.Generator().manual_seed(B)
    xs = [torch.rand(B, 1, 28, 28, generator=g) for _ in range(steps)]
    ys = [torch.randint(0, 10, (B,), generator=g) for _ in range(steps)]
    losses = []
    for i in range(steps):
        tr.set_batch(xs[i].to(cuda), ys[i].to(cuda))
        tr.step(1)
        losses.append(tr.read_metrics()[0] / B)
    ref_losses = _ref_steps(ref, xs, ys, steps)
    for a, b in zip(losses, ref_losses):
        assert abs(a - b) < 1e-4 * max(1.0, abs(b)), (B, losses, ref_losses)
    sd = tr.state_dict()
    for k, v in ref.state_dict().items():
        err = (sd[k] - v).abs().max().item() / (v.abs().max().item() + 1e-6)
        assert err < 1e-4, (B, k, err)


@pytest.mark.parametrize("B,wt", [(64, 0), (64, 1), (32, 7)])  # default 6: every other test
def test_fused_engine_write_through_stores_match_reference(cuda, B, wt):
    """Plain and agent-scope (L2 write-through) stores of F5 / F2 / F6W's bulk outputs vs the reference."""
    from mxddp import native
    from mxddp.engine import FusedMnistTrainer
    from mxddp.models import MnistCNN

    torch.manual_seed(0)
    ref = MnistCNN()
    steps = 3
    old = native().mnist_wt_stores()
    native().mnist_set_wt_stores(wt)
    try:
        tr = FusedMnistTrainer(batch=B, device=cuda, comm=None, init_model=ref, use_graph=True)
        g = torch.Generator().manual_seed(B + 1)
        xs = [torch.rand(B, 1, 28, 28, generator=g) for _ in range(steps)]
        ys = [torch.randint(0, 10, (B,), generator=g) for _ in range(steps)]
        losses = []
        for i in range(steps):
            tr.set_batch(xs[i].to(cuda), ys[i].to(cuda))
            tr.step(1)
            losses.append(tr.read_metrics()[0] / B)
    finally:
        native().mnist_set_wt_stores(old)
    ref_losses = _ref_steps(ref, xs, ys, steps)
    for a, b in zip(losses, ref_losses):
        assert abs(a - b) < 1e-4 * max(1.0, abs(b)), (B, losses, ref_losses)
    sd = tr.state_dict()
    for k, v in ref.state_dict().items():
        err = (sd[k] - v).abs().max().item() / (v.abs().max().item() + 1e-6)
        assert err < 1e-4, (B, k, err)


@pytest.mark.parametrize("merged", [False, True])
@pytest.mark.parametrize("graph", [0, 1, 2])
def test_fused_engine_rccl_collectives_ws1(cuda, graph, merged):
    """The DDP path with REAL RCCL all-reduces (1-rank communicator, collectives forced):
    eager, captured inside the step graph (mode 1) and issued between compute graphs (mode 2);
    two buckets, or one all-reduce over the whole gradient (merged)."""
    from mxddp import native
    from mxddp.engine import FusedMnistTrainer
    from mxddp.models import MnistCNN

    C = native()
    comm = C.Comm(C.Comm.new_unique_id(), 0, 1, cuda.index or 0)
    torch.manual_seed(0)
    ref = MnistCNN()
    B, steps = 32, 5
    tr = FusedMnistTrainer(batch=B, device=cuda, comm=comm, init_model=ref, use_graph=graph > 0,
                           graph_mode=graph if graph else None, force_collectives=True)
    tr.eng.set_merged(merged)
    assert tr.eng.merged == merged
    xs = [torch.rand(B, 1, 28, 28) for _ in range(steps)]
    ys = [torch.randint(0, 10, (B,)) for _ in range(steps)]
    losses = []
    for i in range(steps):
        tr.set_batch(xs[i].to(cuda), ys[i].to(cuda))
        tr.step(1)
        losses.append(tr.read_metrics()[0] / B)
    ref_losses = _ref_steps(ref, xs, ys, steps)
    for a, b in zip(losses, ref_losses):
        assert abs(a - b) < 1e-4 * max(1.0, abs(b)), (losses, ref_losses)


def test_fused_engine_multi_step_graph(cuda):
    """8 steps unrolled per graph (+ 4/2/1-step remainder graphs) == single steps (same
    device-side data stream)."""
    from mxddp.engine import FusedMnistTrainer

    a = FusedMnistTrainer(batch=64, device=cuda, lr=0.01, steps_per_graph=8)
    b = FusedMnistTrainer(batch=64, device=cuda, lr=0.01, steps_per_graph=1)
    for n in (1, 13, 3, 7):  # remainders run from the 4 / 2 / 1-step graphs
        a.step(n)
        b.step(n)
    la, ca = a.read_metrics()
    lb, cb = b.read_metrics()
    assert abs(la - lb) < 1e-3 * abs(lb) and ca == cb
    for k, v in a.state_dict().items():
        assert torch.allclose(v, b.state_dict()[k], rtol=1e-4, atol=1e-6), k


def test_fused_engine_warm_graphs_are_training_steps(cuda):
    """warm_graphs() launches every captured graph once (8 + 4 + 2 + 1 steps) and counts them:
    the same state and metrics as that many single steps, and small-first replay ordering runs
    the same steps."""
    from mxddp.engine import FusedMnistTrainer

    a = FusedMnistTrainer(batch=64, device=cuda, lr=0.01, steps_per_graph=8)
    b = FusedMnistTrainer(batch=64, device=cuda, lr=0.01, steps_per_graph=1)
    a.step(1)
    n = a.warm_graphs()
    assert n == 8 + 4 + 2 + 1 and a.steps == 1 + n
    b.step(1 + n)
    a.eng.set_small_first(True)
    a.step(13)  # 8 + 4 + 1, remainders first
    b.step(13)
    la, ca = a.read_metrics()
    lb, cb = b.read_metrics()
    assert a.steps_at_reset == a.steps == b.steps
    assert abs(la - lb) < 1e-3 * abs(lb) and ca == cb
    for k, v in a.state_dict().items():
        assert torch.allclose(v, b.state_dict()[k], rtol=1e-4, atol=1e-6), k


def test_fused_engine_trains(cuda):
    from mxddp.engine import FusedMnistTrainer

    tr = FusedMnistTrainer(batch=64, device=cuda, lr=0.01)
    tr.step(5)
    l0, _ = tr.read_metrics()
    tr.step(200)
    tr.read_metrics()
    tr.step(20)
    l1, c1 = tr.read_metrics()
    assert l1 / (20 * 64) < 0.5 * l0 / (5 * 64)
    assert c1 / (20 * 64) > 0.8


def test_fused_engine_autotune_keeps_training_exact(cuda):
    """Strategy autotuning (eager/graph x overlapped/in-order collectives) only changes HOW the
    step is launched: the trained weights equal an untuned engine's after the same step count."""
    from mxddp import native
    from mxddp.engine import FusedMnistTrainer

    C = native()
    comm = C.Comm(C.Comm.new_unique_id(), 0, 1, cuda.index or 0)
    a = FusedMnistTrainer(batch=64, device=cuda, lr=0.01, comm=comm, force_collectives=True)
    b = FusedMnistTrainer(batch=64, device=cuda, lr=0.01)
    a.step(1)
    res = a.autotune(trial_steps=4, include_graphs=True)
    assert len(res) == 6 and a.tuned is not None  # {eager, graph} x {ovl, inl, one}
    assert a.steps == 1 and a.discarded_steps == 6 * (2 + 4)  # the trial steps are scratch
    a.step(10)
    b.step(1 + 10)
    assert a.steps == b.steps
    # same device-side data stream and update rule, every cross-block sum order-independent
    # (int64 fixed point) or in a fixed order: the two launch paths train bit for bit alike
    for k, v in a.state_dict().items():
        assert torch.equal(v, b.state_dict()[k]), (k, ((v - b.state_dict()[k]).norm() / v.norm()).item())


def test_bench_json_reports_per_image_metrics(cuda):
    """The driver-visible bench line: train_acc is a fraction in [0, 1] and train_loss_avg a
    per-image average (round 2 divided the sums by 1 after a premature reset)."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "20", "--warmup", "5"],
                       capture_output=True, text=True, timeout=240, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    assert 0.0 <= out["train_acc"] <= 1.0, out
    assert 0.0 < out["train_loss_avg"] < 3.0, out
    assert out["train_images"] >= 25 * 64, out


@pytest.mark.parametrize("args", [["--model", "resnet50", "--dtype", "bf16", "--batch", "8"],
                                  ["--model", "mlp", "--impl", "layers"]])
def test_bench_json_layer_path(cuda, args):
    """bench.py on the layer path (no fused engine): one JSON line with the graph flag (round 3
    broke this for every non-fused model)."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "3", "--warmup", "2", *args],
                       capture_output=True, text=True, timeout=240, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["value"] > 0 and out["config"]["model"] == args[1], out
    assert "graph" in out["config"], out


@pytest.mark.parametrize("variant", ["default", "Ring:c7", "Ring:c28", "Ring/Simple:c14"])
def test_fused_engine_rccl_variants_ws1(cuda, variant):
    """Every xGMI-sized RCCL communicator variant (ncclCommInitRankConfig with pinned CTA counts,
    NCCL_ALGO / NCCL_PROTO pinned for its init) carries the forced DDP all-reduces of the fused
    step -- the padded fc bucket included -- and trains exactly like the reference."""
    from mxddp import native
    from mxddp.engine import FusedMnistTrainer
    from mxddp.models import MnistCNN
    from mxddp.parallel.comm import parse_variant

    C = native()
    comm = C.Comm(C.Comm.new_unique_id(), 0, 1, cuda.index or 0, **parse_variant(variant))
    assert comm.variant == variant
    torch.manual_seed(0)
    ref = MnistCNN()
    B, steps = 32, 4
    tr = FusedMnistTrainer(batch=B, device=cuda, comm=comm, init_model=ref, use_graph=False, force_collectives=True)
    assert tr.active_transport == f"rccl:{variant}"
    xs = [torch.rand(B, 1, 28, 28) for _ in range(steps)]
    ys = [torch.randint(0, 10, (B,)) for _ in range(steps)]
    losses = []
    for i in range(steps):
        tr.set_batch(xs[i].to(cuda), ys[i].to(cuda))
        tr.step(1)
        losses.append(tr.read_metrics()[0] / B)
    ref_losses = _ref_steps(ref, xs, ys, steps)
    for a, b in zip(losses, ref_losses):
        assert abs(a - b) < 1e-4 * max(1.0, abs(b)), (losses, ref_losses)
    assert tr._grad_store[tr.params.numel():].abs().max().item() == 0.0  # padding slack stays zero


@pytest.mark.parametrize("graphs", [False, None])
def test_fused_autotune_lists_rccl_variants(cuda, monkeypatch, graphs):
    """autotune() times every configured RCCL variant (here at world size 1, collectives
    forced) and reports them in its JSON; the trained weights stay exact under restore=True.
    graphs=None: the default (MXDDP_AUTOTUNE_GRAPHS=1), every variant also captured in the step
    graph."""
    from mxddp.engine import FusedMnistTrainer
    from mxddp.parallel import comm as pc

    monkeypatch.setenv("MXDDP_RCCL_VARIANTS", "default,Ring:c7,Ring:c28")
    pc.init_distributed(use_gpu=True)
    comm = pc.rccl_comm(force=True)
    a = FusedMnistTrainer(batch=64, device=cuda, lr=0.01, comm=comm, force_collectives=True)
    b = FusedMnistTrainer(batch=64, device=cuda, lr=0.01)
    a.step(1)
    b.step(1)
    monkeypatch.delenv("MXDDP_AUTOTUNE_GRAPHS", raising=False)
    res = a.autotune(trial_steps=3, restore=True, include_graphs=graphs)
    names = {k.split("/")[0] for k in a.tuned["trials_ms"]}
    assert names == {"rccl:default", "rccl:Ring:c7", "rccl:Ring:c28"}, a.tuned
    assert len(res) == (9 if graphs is False else 18) and a.steps == 1
    a.step(10)
    b.step(10)
    for k, v in a.state_dict().items():
        assert torch.equal(v, b.state_dict()[k]), (k, ((v - b.state_dict()[k]).norm() / v.norm()).item())


def test_fused_engine_is_deterministic(cuda):
    """Two engines from the same seed train bit-identically over 60 steps (graph replays and
    eager steps alike): F3's split-K partials, the conv1 / conv2-bias gradients and the loss are
    summed as int64 fixed point or in a fixed order, never with order-dependent float atomics."""
    from mxddp.engine import FusedMnistTrainer

    runs = []
    for graph in (True, True, False):
        tr = FusedMnistTrainer(batch=64, device=cuda, lr=0.05, use_graph=graph)
        tr.step(60)
        runs.append((tr.state_dict(), tr.read_metrics()))
    (sa, ma), (sb, mb), (sc, mc) = runs
    assert ma == mb == mc
    for k in sa:
        assert torch.equal(sa[k], sb[k]) and torch.equal(sa[k], sc[k]), k


def test_fused_engine_divergence_stays_visible(cuda):
    """A NaN reaching one of the step's int64 fixed-point sums (F3's fc1 pre-activation, the conv
    gradient slabs) must not be saturated into finite garbage: the loss and the updated weights
    come out NaN (the sticky flag of mnist_common.h fix_add)."""
    from mxddp.engine import FusedMnistTrainer
    from mxddp.models import MnistCNN

    torch.manual_seed(0)
    m = MnistCNN()
    with torch.no_grad():
        m.fc1.weight[7, 100] = float("nan")  # F3's fc1 partial of output column 7 becomes NaN
    tr = FusedMnistTrainer(batch=16, device=cuda, comm=None, init_model=m, use_graph=False)
    tr.step(1)
    loss, _ = tr.read_metrics()
    assert loss != loss, loss
    sd = tr.state_dict()
    assert torch.isnan(sd["fc2.weight"]).any() and torch.isnan(sd["conv1.weight"]).any()



@pytest.mark.parametrize("batch,graph,mode", [(64, True, 1), (64, False, 1), (37, True, 1), (96, True, 1),
                                              (128, True, 1), (64, True, 2), (48, False, 2), (96, True, 2)])
def test_deferred_fc1_update_is_bitwise_equal(cuda, batch, graph, mode):
    """mnist_set_fc1_defer: F5 publishes dh and the fc1 weight gradient + SGD run in the last
    blocks of the conv-backward launch -- the same operands, MFMA order and update as F5's folded
    path, so 30 steps train bit for bit alike (batch 128: the deferral is declined, LDS)."""
    from mxddp import native
    from mxddp.engine import FusedMnistTrainer

    C = native()
    sds = []
    try:
        for defer in (mode, 0):
            C.mnist_set_fc1_defer(defer)
            tr = FusedMnistTrainer(batch=batch, device=cuda, lr=0.05, use_graph=graph)
            tr.step(30)
            tr.synchronize()
            sds.append((tr.state_dict(), tr.read_metrics()))
    finally:
        C.mnist_set_fc1_defer(2)
    for k, v in sds[0][0].items():
        assert torch.equal(v, sds[1][0][k]), (k, (v - sds[1][0][k]).abs().max().item())
    assert sds[0][1] == sds[1][1]


@pytest.mark.parametrize("graph", [True, False])
def test_deferred_fc1_gradient_with_merged_allreduce(cuda, graph):
    """With gradient collectives (forced at one rank) and the merged bucket strategy, F67's fc1
    blocks write the fc1 weight gradient to g (the SGD launch updates): bitwise equal to F5
    writing it, over 20 steps."""
    from mxddp import native
    from mxddp.engine import FusedMnistTrainer

    C = native()
    comm = C.Comm(C.Comm.new_unique_id(), 0, 1, cuda.index or 0)
    sds = []
    try:
        for defer in (2, 0):
            C.mnist_set_fc1_defer(defer)
            tr = FusedMnistTrainer(batch=64, device=cuda, lr=0.05, comm=comm, force_collectives=True,
                                   use_graph=graph, graph_mode=1 if graph else 0)
            tr._set_buckets("one")
            tr.step(20)
            tr.synchronize()
            sds.append(tr.state_dict())
    finally:
        C.mnist_set_fc1_defer(2)
    for k, v in sds[0].items():
        assert torch.equal(v, sds[1][k]), (k, (v - sds[1][k]).abs().max().item())
