"""CPU checks of the NHWC ops' host-side pieces (no kernels): the ReLU-mask-bit layout of the
lazy identity-shortcut join and the fork's fallback when the join was not consumed."""
import torch

from mxddp.ops import nhwc


def test_mask_bits_layout():
    """bit e of byte i masks element 8 i + e (the layout of the BN forward's pos_bits8)."""
    g = torch.arange(1, 33, dtype=torch.float32).view(1, 2, 2, 8)
    mask = torch.tensor([0b00000001, 0b10000000, 0xFF, 0], dtype=torch.uint8)
    out = nhwc._mask_bits(g, mask).view(4, 8)
    ref = g.view(4, 8).clone()
    keep = torch.tensor([[(m >> e) & 1 for e in range(8)] for m in mask.tolist()], dtype=torch.bool)
    ref[~keep] = 0
    assert torch.equal(out, ref)


def test_fork_lazy_join_fallback():
    """A lazy join left in GradJoin (dy + mask bits) but never consumed by a conv epilogue: the
    fork adds the masked gradient itself; consumed: g_main passes through."""
    join = nhwc.GradJoin()
    x = torch.randn(1, 2, 2, 8, requires_grad=True)
    main, short = nhwc.fork(x, join)
    dy = torch.randn(1, 2, 2, 8)
    mask = torch.randint(0, 256, (4,), dtype=torch.uint8)
    join.dres, join.amask = dy, mask
    g_main = torch.randn(1, 2, 2, 8)
    main.backward(g_main)  # short gets no gradient: the fork must add the lazy one
    assert torch.allclose(x.grad, g_main + nhwc._mask_bits(dy, mask))
    assert join.dres is None and join.amask is None and not join.consumed

    x.grad = None
    main, short = nhwc.fork(x, join)
    join.dres, join.amask, join.consumed = dy, mask, True
    main.backward(g_main)
    assert torch.equal(x.grad, g_main)


def test_fork_half_resolution_join_fallback():
    """A stride-2 projection's half-resolution input gradient (GradJoin.sub2; the projection conv
    returns no gradient of its own) that no conv epilogue consumed: the fork adds it at the even
    (h, w) positions and clears the join."""
    join = nhwc.GradJoin()
    x = torch.randn(2, 6, 4, 8, requires_grad=True)
    main, short = nhwc.fork(x, join)
    dres = torch.randn(2, 3, 2, 8)
    join.dres, join.sub2 = dres, True
    g_main = torch.randn(2, 6, 4, 8)
    main.backward(g_main)  # short gets no gradient, as behind the projection conv
    want = g_main.clone()
    want[:, ::2, ::2, :] += dres
    assert torch.allclose(x.grad, want)
    assert join.dres is None and not join.sub2
