"""Numerics of every HIP kernel vs a plain PyTorch fp32 reference of the same op (CPU).

Asymmetric random operands everywhere (a symmetric operand hides a row/col swap,
cdna_hip_programming.md §3), and shapes that are not tile multiples.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from mxddp import ops  # noqa: E402

CONV_CASES = [
    # N, C, H, W, K, R, S, stride, pad
    (4, 1, 28, 28, 32, 3, 3, 1, 0),      # mnist conv1
    (3, 32, 26, 26, 64, 3, 3, 1, 0),     # mnist conv2
    (2, 21, 16, 16, 26, 3, 3, 1, 1),     # pyramidnet-like odd channels
    (2, 101, 32, 32, 106, 3, 3, 2, 1),   # pyramidnet stride-2 entry (dgrad: zero-insert + Winograd)
    (3, 186, 16, 16, 191, 3, 3, 2, 1),   # pyramidnet stride-2 entry of stage 3
    (2, 3, 33, 31, 17, 7, 7, 2, 3),      # resnet stem-like, odd spatial
    (2, 64, 14, 14, 40, 1, 1, 1, 0),     # 1x1
    # direct-LDS 3x3 s1 p1 path (conv3x3.hip): every supported width, C not a multiple of 8,
    # K not a multiple of 64, partial row tiles (H not a multiple of 64/W)
    (2, 13, 32, 32, 70, 3, 3, 1, 1),
    (3, 40, 8, 8, 130, 3, 3, 1, 1),
    (2, 9, 7, 7, 20, 3, 3, 1, 1),
    (2, 17, 14, 14, 33, 3, 3, 1, 1),
    (1, 12, 28, 27 + 1, 65, 3, 3, 1, 1),
    (1, 8, 56, 56, 24, 3, 3, 1, 1),
    (2, 5, 13, 16, 7, 3, 3, 1, 1),
    # Winograd F(2x2,3x3) path (winograd.hip): split-C grid (8x8, many channels), partial tile blocks
    (16, 191, 8, 8, 196, 3, 3, 1, 1),
    (4, 101, 16, 16, 106, 3, 3, 1, 1),
    # few output tiles over a long reduction: split-K into partial planes + finish pass
    # (forward and the flipped-filter data gradient), small-tile weight-gradient splits
    (64, 64, 5, 5, 64, 3, 3, 1, 0),      # keras conv3
    (16, 32, 13, 13, 64, 3, 3, 1, 0),    # keras conv2
]


def _rel(a, b):
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("relu", [False, True])
def test_conv2d_fwd_bwd(cuda, case, relu):
    N, C, H, W, K, R, S, st, pd = case
    torch.manual_seed(0)
    x = torch.randn(N, C, H, W)
    w = torch.randn(K, C, R, S) * 0.1
    b = torch.randn(K)
    xg, wg, bg = (t.to(cuda).requires_grad_() for t in (x, w, b))
    y = ops.conv2d(xg, wg, bg, st, pd, relu=relu)
    xr, wr, br = (t.clone().requires_grad_() for t in (x, w, b))
    yr = F.conv2d(xr, wr, br, st, pd)
    if relu:
        # the reference takes the kernel's ReLU mask: an output within rounding of 0 may go either
        # way, and a flipped mask element would move dx / dw by a whole gradient term
        assert _rel(y.detach().cpu(), F.relu(yr.detach())) < 1e-4
        yr = yr * (y.detach().cpu() > 0)
    gy = torch.randn_like(yr)
    yr.backward(gy)
    y.backward(gy.to(cuda))
    torch.cuda.synchronize()
    assert _rel(y.cpu(), yr.detach()) < 1e-4
    assert _rel(xg.grad.cpu(), xr.grad) < 1e-4
    assert _rel(wg.grad.cpu(), wr.grad) < 1e-4
    assert _rel(bg.grad.cpu(), br.grad) < 1e-4


WINO_CASES = [
    # N, C, W, K  (3x3 s1 p1, square)
    (2, 16, 32, 21),
    (3, 37, 16, 45),
    (5, 191, 8, 196),
    (64, 271, 8, 10),
    (1, 8, 8, 8),
]


@pytest.mark.parametrize("case", WINO_CASES)
def test_winograd_vs_direct_fp64(cuda, case):
    """Winograd and direct-LDS 3x3 paths against an fp64 oracle: Winograd's extra rounding
    (transforms) must stay within a small factor of the direct path's fp32 error."""
    import mxddp

    C_ = mxddp.native()
    N, C, W, K = case
    torch.manual_seed(1)
    x = torch.randn(N, C, W, W)
    w = torch.randn(K, C, 3, 3) / (3 * C ** 0.5)
    gy = torch.randn(N, K, W, W)
    xr, wr = x.double().requires_grad_(), w.double().requires_grad_()
    yr = F.conv2d(xr, wr, None, 1, 1)
    yr.backward(gy.double())
    errs = {}
    prev = C_.conv_algo()
    try:
        for algo in (0, 1):
            C_.set_conv_algo(algo)
            xg, wg = x.to(cuda).requires_grad_(), w.to(cuda).requires_grad_()
            y = ops.conv2d(xg, wg, None, 1, 1)
            y.backward(gy.to(cuda))
            torch.cuda.synchronize()
            errs[algo] = [_rel(y.cpu().double(), yr.detach()), _rel(xg.grad.cpu().double(), xr.grad),
                          _rel(wg.grad.cpu().double(), wr.grad)]
    finally:
        C_.set_conv_algo(prev)
    for e_w, e_d in zip(errs[0], errs[1]):
        assert e_w < 2e-5 and e_w < 8 * e_d + 1e-6, errs


@pytest.mark.parametrize("M,N,K", [(64, 128, 9216), (64, 10, 128), (100, 1000, 784), (7, 33, 65), (64, 64, 576),
                                   (64, 1000, 1000)])
def test_linear_fwd_bwd(cuda, M, N, K):
    torch.manual_seed(1)
    x, w, b = torch.randn(M, K), torch.randn(N, K) * 0.05, torch.randn(N)
    xr, wr, br = (t.clone().requires_grad_() for t in (x, w, b))
    yr = F.relu(F.linear(xr, wr, br))
    gy = torch.randn_like(yr)
    yr.backward(gy)
    xg, wg, bg = (t.to(cuda).requires_grad_() for t in (x, w, b))
    y = ops.linear(xg, wg, bg, relu=True)
    y.backward(gy.to(cuda))
    torch.cuda.synchronize()
    assert _rel(y.cpu(), yr.detach()) < 1e-4
    assert _rel(xg.grad.cpu(), xr.grad) < 1e-4
    assert _rel(wg.grad.cpu(), wr.grad) < 1e-4
    assert _rel(bg.grad.cpu(), br.grad) < 1e-4


@pytest.mark.parametrize("M,N,K", [(64, 1000, 1000), (64, 128, 9216), (5, 70, 300)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_linear_dgrad_mask_accumulate(cuda, M, N, K, accumulate):
    """dx (+)= (dy @ w) * (mask > 0): split-K partial planes finish with mask and accumulate."""
    from mxddp import native

    torch.manual_seed(3)
    dy, w = torch.randn(M, N), torch.randn(N, K) * 0.05
    mask = torch.randn(M, K).clamp_min(0)  # ~half the entries masked
    dx0 = torch.randn(M, K)
    ref = (dy @ w) * (mask > 0) + (dx0 if accumulate else 0)
    dyg, wg, mg = dy.to(cuda), w.to(cuda), mask.to(cuda)
    dx = dx0.to(cuda) if accumulate else torch.full((M, K), float("nan"), device=cuda)
    st = torch.cuda.current_stream(cuda).cuda_stream
    native().linear_dgrad(dyg.data_ptr(), wg.data_ptr(), dx.data_ptr(), M, N, K, mg.data_ptr(), accumulate, st)
    torch.cuda.synchronize()
    assert _rel(dx.cpu(), ref) < 1e-4


@pytest.mark.parametrize("M,N,K", [(64, 1000, 1000), (100, 130, 70)])
def test_linear_backward_dy_mask(cuda, M, N, K):
    """linear_dgrad / linear_wgrad / bias_grad with dy masked on load == the same kernels on the
    masked copy of dy."""
    from mxddp import native

    C_ = native()
    torch.manual_seed(4)
    dy, w, x = torch.randn(M, N), torch.randn(N, K) * 0.05, torch.randn(M, K)
    y = torch.randn(M, N).clamp_min(0)
    g = dy * (y > 0)
    dyg, wg, xg, yg = (t.to(cuda) for t in (dy, w, x, y))
    dx = torch.empty(M, K, device=cuda)
    dw = torch.empty(N, K, device=cuda)
    db = torch.empty(N, device=cuda)
    st = torch.cuda.current_stream(cuda).cuda_stream
    C_.linear_dgrad(dyg.data_ptr(), wg.data_ptr(), dx.data_ptr(), M, N, K, 0, False, st, yg.data_ptr())
    C_.linear_wgrad(dyg.data_ptr(), xg.data_ptr(), dw.data_ptr(), M, N, K, False, st, yg.data_ptr())
    C_.bias_grad(dyg.data_ptr(), db.data_ptr(), M, N, 1, False, st, yg.data_ptr())
    torch.cuda.synchronize()
    assert _rel(dx.cpu(), g @ w) < 1e-4
    assert _rel(dw.cpu(), g.t() @ x) < 1e-4
    assert _rel(db.cpu(), g.sum(0)) < 1e-4


@pytest.mark.parametrize("k,s,p,ceil", [(2, 2, 0, False), (3, 2, 1, False), (2, 2, 0, True)])
def test_pools(cuda, k, s, p, ceil):
    torch.manual_seed(2)
    x = torch.randn(2, 5, 13, 11)
    for fn_ref, fn in ((F.max_pool2d, ops.max_pool2d), (F.avg_pool2d, ops.avg_pool2d)):
        xr = x.clone().requires_grad_()
        yr = fn_ref(xr, k, s, p, ceil_mode=ceil)
        gy = torch.randn_like(yr)
        yr.backward(gy)
        xg = x.to(cuda).requires_grad_()
        y = fn(xg, k, s, p, ceil_mode=ceil)
        y.backward(gy.to(cuda))
        assert _rel(y.detach().cpu(), yr.detach()) < 1e-5
        assert _rel(xg.grad.cpu(), xr.grad) < 1e-5


def test_cross_entropy(cuda):
    torch.manual_seed(3)
    logits = torch.randn(64, 10) * 3
    y = torch.randint(0, 10, (64,))
    lr = logits.clone().requires_grad_()
    ref = F.cross_entropy(lr, y)
    ref.backward()
    lg = logits.to(cuda).requires_grad_()
    loss, correct = ops.cross_entropy(lg, y.to(cuda), return_correct=True)
    loss.backward()
    assert abs(loss.item() - ref.item()) < 1e-5
    assert correct.item() == (logits.argmax(1) == y).sum().item()
    assert _rel(lg.grad.cpu(), lr.grad) < 1e-5


@pytest.mark.parametrize("shape,offset", [((8, 21, 9, 7), 0.5), ((64, 16, 32, 32), 3.0), ((64, 271, 8, 8), -20.0),
                                          ((3, 5, 7, 7), 0.0), ((32, 64, 56, 56), 1.0),
                                          ((64, 106, 16, 16), 7.0), ((16, 64, 6, 6), 0.0),
                                          ((32, 80, 16, 16), -3.0), ((2, 8, 128, 128), 2.0)])
@pytest.mark.parametrize("relu", [False, True])
def test_batchnorm(cuda, relu, shape, offset):
    """Split-reduction BN (vector and scalar paths, 1..64 splits, large mean offset) and the
    register-resident one-block-per-channel kernels (1, 2, 4 and 8 float4s per thread) vs torch
    fp32."""
    torch.manual_seed(4)
    C = shape[1]
    x = torch.randn(*shape) * 2 + offset
    g, b = torch.rand(C) + 0.5, torch.randn(C)
    rm, rv = torch.zeros(C), torch.ones(C)
    xr, gr, br = (t.clone().requires_grad_() for t in (x, g, b))
    yr = F.batch_norm(xr, rm, rv, gr, br, True, 0.1, 1e-5)
    if relu:
        yr = F.relu(yr)
    gy = torch.randn_like(yr)
    yr.backward(gy)
    rmg, rvg = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    xg, gg, bg = (t.to(cuda).requires_grad_() for t in (x, g, b))
    y = ops.batch_norm(xg, gg, bg, rmg, rvg, True, 0.1, 1e-5, relu=relu)
    y.backward(gy.to(cuda))
    assert _rel(y.detach().cpu(), yr.detach()) < 1e-4
    # With the fused ReLU, an element whose normalised value rounds to ~0 can fall on different
    # sides of the threshold in two fp32 implementations; its dx then differs by the whole
    # gamma*invstd*dy term.  Compare dx where the two masks agree (a handful of elements in 6M).
    agree = ((y.detach().cpu() > 0) == (yr.detach() > 0)) if relu else torch.ones_like(yr, dtype=torch.bool)
    assert agree.float().mean().item() > 1 - 1e-5
    assert _rel(xg.grad.cpu() * agree, xr.grad * agree) < 1e-4
    # dgamma / dbeta sum dy over the ReLU mask: a threshold disagreement (atomic reduction order
    # moves the batch mean by an ulp) shifts them by that element's dy
    assert _rel(gg.grad.cpu(), gr.grad) < (2e-3 if relu else 1e-4)
    assert _rel(bg.grad.cpu(), br.grad) < (2e-3 if relu else 1e-4)
    assert _rel(rmg.cpu(), rm) < 1e-5 and _rel(rvg.cpu(), rv) < 1e-5
    # a second call reuses the self-resetting ticket counters
    y2 = ops.batch_norm(xg.detach(), gg, bg, rmg, rvg, True, 0.1, 1e-5, relu=relu)
    assert _rel(y2.cpu(), yr.detach()) < 1e-4


@pytest.mark.parametrize("stride", [1, 2])
def test_shortcut(cuda, stride):
    torch.manual_seed(5)
    x = torch.randn(2, 21, 9, 9)
    P = 9 if stride == 1 else 5
    out = torch.randn(2, 26, P, P)
    xr, orr = x.clone().requires_grad_(), out.clone().requires_grad_()
    yr = ops.shortcut_pad_add(orr, xr, stride)  # CPU reference path = F.pad + avg_pool
    gy = torch.randn_like(yr)
    yr.backward(gy)
    xg, og = x.to(cuda).requires_grad_(), out.to(cuda).requires_grad_()
    y = ops.shortcut_pad_add(og, xg, stride)
    y.backward(gy.to(cuda))
    assert _rel(y.detach().cpu(), yr.detach()) < 1e-5
    assert _rel(xg.grad.cpu(), xr.grad) < 1e-5
    assert _rel(og.grad.cpu(), orr.grad) < 1e-5


@pytest.mark.parametrize("shape", [(4, 21, 26, 16, 16), (8, 186, 186, 8, 8), (2, 5, 9, 7, 7), (32, 100, 105, 16, 16)])
def test_batchnorm_residual_tap(cuda, shape):
    """PyramidNet identity-shortcut fusion: bn1 with a tap output (its gradient is summed into dx
    by the BN kernel, read in place from the channel slice of the block-output gradient) and bn3
    with the zero-padded residual added in its normalise pass, vs plain torch fp32."""
    torch.manual_seed(7)
    N, Cin, C, H, W = shape
    x = torch.randn(N, Cin, H, W) * 1.5 + 0.3
    z = torch.randn(N, C, H, W) - 0.7
    g1, b1, g3, b3 = torch.rand(Cin) + 0.5, torch.randn(Cin), torch.rand(C) + 0.5, torch.randn(C)
    gh, go = torch.randn(N, Cin, H, W), torch.randn(N, C, H, W)
    leaves = [x, z, g1, b1, g3, b3]
    ref = [t.clone().requires_grad_() for t in leaves]
    xr, zr, g1r, b1r, g3r, b3r = ref
    hr = F.batch_norm(xr, torch.zeros(Cin), torch.ones(Cin), g1r, b1r, True, 0.1, 1e-5)
    outr = F.batch_norm(zr, torch.zeros(C), torch.ones(C), g3r, b3r, True, 0.1, 1e-5) + F.pad(
        xr, (0, 0, 0, 0, 0, C - Cin))
    ((hr * gh).sum() + (outr * go).sum()).backward()
    dev = [t.to(cuda).requires_grad_() for t in leaves]
    xg, zg, g1g, b1g, g3g, b3g = dev
    h, xs = ops.batch_norm(xg, g1g, b1g, torch.zeros(Cin, device=cuda), torch.ones(Cin, device=cuda), True,
                           tap=True)
    out = ops.batch_norm(zg, g3g, b3g, torch.zeros(C, device=cuda), torch.ones(C, device=cuda), True, residual=xs)
    ((h * gh.to(cuda)).sum() + (out * go.to(cuda)).sum()).backward()
    torch.cuda.synchronize()
    assert _rel(h.detach().cpu(), hr.detach()) < 1e-4
    assert _rel(out.detach().cpu(), outr.detach()) < 1e-4
    for a, b in zip(dev, ref):
        assert _rel(a.grad.cpu(), b.grad) < 2e-4


def test_sgd_adam_flat(cuda):
    import torch.nn as nn

    from mxddp.optim import SGD, Adam
    from mxddp.parallel.flat import FlatParams

    for Opt, ref_cls, kw in ((SGD, torch.optim.SGD, dict(lr=0.1, momentum=0.9, weight_decay=1e-4)),
                             (Adam, torch.optim.Adam, dict(lr=1e-3, weight_decay=0.0))):
        torch.manual_seed(6)
        m_ref = nn.Linear(37, 19)
        m = nn.Linear(37, 19)
        m.load_state_dict(m_ref.state_dict())
        m = m.to(cuda)
        flat = FlatParams(m)
        opt = Opt(flat, **kw)
        ref = ref_cls(m_ref.parameters(), **kw)
        for step in range(3):
            gs = [torch.randn_like(p) for p in m_ref.parameters()]
            for p, g in zip(m_ref.parameters(), gs):
                p.grad = g.clone()
            for p, g in zip(m.parameters(), gs):
                p.grad.copy_(g)
            ref.step()
            opt.step()
        torch.cuda.synchronize()
        for p, q in zip(m.parameters(), m_ref.parameters()):
            assert _rel(p.detach().cpu(), q.detach()) < 1e-5, Opt.__name__


@pytest.mark.parametrize("shape", [(64, 21, 32, 21), (64, 61, 32, 66), (64, 191, 8, 196), (4, 13, 16, 7)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_winograd_wgrad_partial_planes(cuda, shape, accumulate):
    """Winograd weight gradient with its split reduction: up to 256 partial planes summed by the
    grouped reduce (plane groups + LDS tree), odd plane sizes (the float tail), accumulate mode;
    vs an fp64 CPU reference."""
    import mxddp

    C_ = mxddp.native()
    N, C, W, K = shape
    torch.manual_seed(11)
    x = torch.randn(N, C, W, W)
    dy = torch.randn(N, K, W, W)
    ref = torch.nn.grad.conv2d_weight(x.double(), (K, C, 3, 3), dy.double(), 1, 1)
    base = torch.randn(K, C, 3, 3) if accumulate else torch.zeros(K, C, 3, 3)
    geo = (N, C, W, W, K, 3, 3, 1, 1, 1, 1, 1, 1)
    xg, dyg, dw = x.to(cuda), dy.to(cuda), base.to(cuda)
    ws = torch.empty(max(1, C_.conv_wgrad_scratch_floats(*geo)), device=cuda)
    C_.conv2d_wgrad(dyg.data_ptr(), xg.data_ptr(), dw.data_ptr(), *geo, accumulate,
                    torch.cuda.current_stream().cuda_stream, ws.data_ptr())
    torch.cuda.synchronize()
    want = ref + base.double()
    err = ((dw.cpu().double() - want).abs().max() / want.abs().max()).item()
    assert err < 2e-5, err


def test_winograd_filter_bank_matches_per_conv_transforms(cuda):
    """Banked Winograd filters (one refresh launch after each optimizer step) give bit-identical
    training to per-conv transforms, and a torch-level weight write (load_state_dict) is
    detected as stale."""
    import torch.nn as nn

    from mxddp import ops as O
    from mxddp.models.layers import BatchNorm2d, Conv2d
    from mxddp.optim import SGD
    from mxddp.parallel.flat import FlatParams

    def run(bank_on):
        prev, O._BANK_ON = O._BANK_ON, bank_on
        try:
            torch.manual_seed(21)
            m = nn.Sequential(Conv2d(8, 12, 3, 1, 1, bias=False), BatchNorm2d(12, fuse_relu=True),
                              Conv2d(12, 13, 3, 1, 1, bias=False), BatchNorm2d(13)).to(cuda)
            flat = FlatParams(m)
            opt = SGD(flat, lr=0.05, momentum=0.9, weight_decay=1e-4)
            x = torch.randn(6, 8, 16, 16, device=cuda)
            for _ in range(3):
                opt.zero_grad()
                m(x).square().mean().backward()
                opt.step()
            y = m(x).detach().clone()
            # torch-level write: the banked filters must be recomputed, not reused
            sd = {k: v * 0.5 if v.is_floating_point() else v for k, v in m.state_dict().items()}
            m.load_state_dict(sd)
            y2 = m(x).detach().clone()
            return flat.data.clone(), y, y2
        finally:
            O._BANK_ON = prev

    a, b = run(True), run(False)
    for u, v in zip(a, b):
        assert torch.equal(u, v)


def test_scratch_is_stream_owned_two_streams(cuda):
    """Split-K partial planes (linear forward / data gradient) and BN partial sums issued on two
    streams AT ONCE: each stream owns its scratch, so neither result is corrupted by the other
    (round 2 shared one per-device buffer across streams: the side-stream experiment's fault)."""
    torch.manual_seed(11)
    cases = []
    for s in range(2):
        x, w = torch.randn(64, 9216 - 7 * s), torch.randn(128 + s, 9216 - 7 * s) * 0.02
        xb = torch.randn(32, 64 + 5 * s, 11, 11) + s
        cases.append((x, w, xb, F.linear(x, w), F.batch_norm(xb, None, None, training=True)))
    streams = [torch.cuda.Stream(cuda) for _ in range(2)]
    dev_in = [(x.to(cuda), w.to(cuda), xb.to(cuda)) for x, w, xb, _, _ in cases]
    torch.cuda.synchronize()
    outs = [[], []]
    for rep in range(12):  # interleave launches so both streams' kernels overlap on the device
        for s in range(2):
            with torch.cuda.stream(streams[s]):
                x, w, xb = dev_in[s]
                C = xb.shape[1]
                y = ops.linear(x, w, None)
                z = ops.batch_norm(xb, None, None, torch.zeros(C, device=cuda), torch.ones(C, device=cuda), True)
                outs[s].append((y, z))
    torch.cuda.synchronize()
    for s in range(2):
        for y, z in outs[s]:
            assert _rel(y.cpu(), cases[s][3]) < 1e-4
            assert _rel(z.cpu(), cases[s][4]) < 1e-4
