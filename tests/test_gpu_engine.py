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
