"""Deferred weight-gradient reductions (csrc/wgrad_defer.h, ops.set_wgrad_defer): the convs'
split-K partial planes are summed by the optimizer's batched flush instead of one reduce launch
per conv.  Same per-element arithmetic, so training is bitwise identical to the per-conv
reductions -- PyramidNet-110 (fp32 Winograd weight gradients) and ResNet-50 (bf16 channels-last
weight gradients), eager steps and one captured hipGraph step.  Where the model's own training is
not bitwise reproducible (PyramidNet's fc split-K and average-pool backward use float atomics),
the deferred run must stay within the run-to-run spread of two plain runs."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _batches(cuda, nc, shape, B, n, seed=5):
    from mxddp import native

    Cn = native()
    D = 1
    for s in shape:
        D *= s
    tmpl = torch.empty(nc * D, device=cuda)
    ctr = torch.zeros(4, dtype=torch.int32, device=cuda)
    st = torch.cuda.current_stream(cuda).cuda_stream
    Cn.synth_templates(tmpl.data_ptr(), nc, D, seed, st)
    out = []
    for _ in range(n):
        x = torch.empty((B,) + tuple(shape), device=cuda)
        y = torch.empty(B, dtype=torch.int32, device=cuda)
        Cn.synth_batch(x.data_ptr(), y.data_ptr(), tmpl.data_ptr(), B, D, nc, seed, ctr.data_ptr(), st)
        out.append((x, y))
    return out


def _train(m0, batches, cuda, defer, dtype, graph=False, flush_mb=0):
    from mxddp import native, ops
    from mxddp.optim import SGD
    from mxddp.parallel.flat import FlatParams

    m = copy.deepcopy(m0)
    flat = FlatParams(m, cuda)
    opt = SGD(flat, lr=0.01, momentum=0.9, weight_decay=1e-4)
    ops.set_compute_dtype(dtype)
    ops.set_wgrad_defer(defer)
    ops.set_wgrad_flush_mb(flush_mb)  # 0: everything waits for the step (the counts below)
    pend = []
    try:
        def step(x, y):
            opt.zero_grad()
            flat.attach_grads()
            ops.cross_entropy(m(x), y).backward()
            pend.append(native().wgrad_defer_pending())
            opt.step()

        for x, y in batches[:2]:
            step(x, y)
        if graph:  # the rest as replays of one captured step (flush recorded inside it)
            sx, sy = batches[2][0].clone(), batches[2][1].clone()
            s = torch.cuda.Stream(cuda)
            s.wait_stream(torch.cuda.current_stream(cuda))
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                step(sx, sy)
            for x, y in batches[2:]:
                sx.copy_(x)
                sy.copy_(y)
                g.replay()
        else:
            for x, y in batches[2:]:
                step(x, y)
        torch.cuda.synchronize()
    finally:
        ops.set_wgrad_defer(False)
        ops.set_wgrad_flush_mb(64)
        ops.set_compute_dtype("fp32")
    assert native().wgrad_defer_pending() == 0
    return flat.data.clone(), pend


def _same_within_spread(a, b, c):
    """a (deferred) == b (plain) bitwise when two plain runs agree bitwise; else within their spread."""
    spread = (b - c).abs().max().item()
    d = (a - b).abs().max().item()
    if spread == 0.0:
        assert d == 0.0, d
    else:
        assert d <= 4 * spread + 1e-7, (d, spread)


@pytest.mark.parametrize("graph", [False, True])
def test_pyramidnet_deferred_wgrad_bitwise(cuda, graph):
    from mxddp.models import build_model

    torch.manual_seed(3)
    m0 = build_model("pyramidnet110").to(cuda)
    batches = _batches(cuda, 10, (3, 32, 32), 8, 4)
    a, pa = _train(m0, batches, cuda, True, "fp32", graph)
    b, pb = _train(m0, batches, cuda, False, "fp32", graph)
    c, _ = _train(m0, batches, cuda, False, "fp32", graph)
    assert pa[0] > 50 and pb[0] == 0, (pa, pb)  # ~100 Winograd convs deferred their reductions
    _same_within_spread(a, b, c)
    # early flushes inside the backward (every ~2 MB of pending planes) give the same sums
    e, pe = _train(m0, batches, cuda, True, "fp32", graph, flush_mb=2)
    assert pe[0] < pa[0], (pe, pa)
    _same_within_spread(e, b, c)


@pytest.mark.parametrize("graph", [False, True])
def test_resnet50_bf16_deferred_wgrad_bitwise(cuda, graph):
    from mxddp.models import resnet50

    torch.manual_seed(4)
    m0 = resnet50(num_classes=10).to(cuda)
    batches = _batches(cuda, 10, (3, 64, 64), 4, 4)
    a, pa = _train(m0, batches, cuda, True, "bf16", graph)
    b, pb = _train(m0, batches, cuda, False, "bf16", graph)
    c, _ = _train(m0, batches, cuda, False, "bf16", graph)
    assert pa[0] > 20 and pb[0] == 0, (pa, pb)
    _same_within_spread(a, b, c)
    e, pe = _train(m0, batches, cuda, True, "bf16", graph, flush_mb=2)
    assert pe[0] < pa[0], (pe, pa)
    _same_within_spread(e, b, c)
