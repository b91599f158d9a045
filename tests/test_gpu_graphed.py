"""Whole-step hipGraph (parallel/graphed.py) and learning-rate changes.

A StepLR change of the learning rate between the eager warm-up steps and the capture, and again
after the capture, must reach every replay: the captured step must not record the lr fill of
``opt.step()`` (it would write the capture-time lr back on every replay).  The graph run is
compared with the same schedule run eagerly; the SGD step count (on the device) must count the
replays too.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(use_graph: bool, schedule):
    from mxddp import ops
    from mxddp.models import build_model
    from mxddp.optim import SGD
    from mxddp.parallel.flat import FlatParams
    from mxddp.parallel.graphed import GraphedStep

    dev = torch.device("cuda", 0)
    torch.manual_seed(3)
    model = build_model("mlp").to(dev)
    flat = FlatParams(model, dev)
    opt = SGD(flat, lr=schedule[0], momentum=0.9, weight_decay=1e-4)
    g = torch.Generator().manual_seed(5)
    batches = [(torch.rand(32, 1, 28, 28, generator=g), torch.randint(0, 10, (32,), generator=g))
               for _ in schedule]

    def step(x, y):
        opt.zero_grad()
        loss = ops.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        return (loss.detach(),)

    run = GraphedStep(step, dev, warmup=2, before_replay=opt._sync_lr, enabled=use_graph)
    for lr, (x, y) in zip(schedule, batches):
        opt.param_groups[0]["lr"] = lr
        run(x.to(dev), y.to(dev))
    torch.cuda.synchronize()
    return flat.data.cpu().clone(), run, opt


def test_graphed_step_follows_lr_changes_across_capture():
    # calls 1-2 eager (lr 0.1), call 3 captures with a NEW lr (0.05), replays at 0.05, then 0.01
    schedule = [0.1, 0.1, 0.05, 0.05, 0.05, 0.01, 0.01]
    pe, _, oe = _run(False, schedule)
    pg, run, og = _run(True, schedule)
    assert run.captured and run.replays == 5
    rel = ((pe - pg).abs().max() / pe.abs().max()).item()
    assert rel < 1e-5, rel
    # a graph that kept replaying the capture-time lr would differ by far more than rounding
    pc, _, _ = _run(True, [0.1, 0.1, 0.05, 0.05, 0.05, 0.05, 0.05])
    assert ((pc - pg).abs().max() / pe.abs().max()).item() > 1e-4
    assert oe.steps == len(schedule) and og.steps == len(schedule)
