"""Channels-last bf16 ops (``mxddp/csrc/nhwc_bf16.hip``): the ResNet-50 mixed-precision path
(BASELINE.json config 5: "ResNet-50 synthetic-ImageNet DDP bf16").

Activations are bf16 tensors of logical shape ``[N, H, W, C]`` (contiguous, C a multiple of 8;
the 3-channel image is zero-padded to 8).  Parameters stay fp32 torch-layout ``nn.Conv2d`` /
``nn.BatchNorm2d`` tensors (same ``state_dict`` as the NCHW model); each convolution repacks its
fp32 weights into the bf16 GEMM layout it needs (a few MB, once per call) and weight gradients
are accumulated in fp32 straight into the flat DDP gradient buffer when one is attached
(``mxddp.ops._grad_sink``).  Batch-norm statistics, accumulation and the optimizer are fp32.

GPU only: there is no CPU twin of these kernels (the CPU path of ResNet-50 is the NCHW fp32
model in ``mxddp.models.resnet``, which is also the oracle of ``tests/test_gpu_nhwc.py``).
"""
from __future__ import annotations

import os

import torch

from .. import native
from . import _grad_sink, _p, stream_of
from .. import ops as _ops

BF16 = torch.bfloat16


def _out(H, k, s, p):
    return (H + 2 * p - k) // s + 1


class _ToNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cp):
        x = x.contiguous()
        N, C, H, W = x.shape
        y = torch.empty((N, H, W, cp), device=x.device, dtype=BF16)
        native().nhwc_from_nchw(x.data_ptr(), y.data_ptr(), N, C, H, W, cp, stream_of(x))
        return y

    @staticmethod
    def backward(ctx, dy):
        return None, None  # network input: no gradient


def to_nhwc(x: torch.Tensor, cp: int | None = None) -> torch.Tensor:
    """fp32 NCHW -> bf16 NHWC with channels zero-padded to ``cp`` (default: next multiple of 8)."""
    C = x.shape[1]
    return _ToNHWC.apply(x, cp or (C + 7) // 8 * 8)


def _splitk_scratch(M, Ng, Kg, device):
    n = native().nhwc_conv_scratch_floats(M, Ng, Kg)
    return torch.empty((n,), device=device, dtype=torch.float32) if n else None


class WeightPack:
    """Every convolution weight of a model repacked to its bf16 GEMM layouts in ONE launch per
    forward (``refresh()``), instead of one repack launch per convolution.

    ``specs``: (weight, Cp, need_dgrad) per convolution; the forward layout [K][R][S][Cp] and,
    when ``need_dgrad``, the data-gradient layout [C][R][S][K] live in one bf16 buffer.  The
    descriptor table (device int64, one row per convolution) is built once; the pack stays valid
    while the weights keep their storage (``matches()``), e.g. views into a FlatParams buffer."""

    def __init__(self, specs):
        Cn = native()
        dev = specs[0][0].device
        rows, self._views, off, blk = [], {}, 0, 0
        layout = []
        for w, cp, nd in specs:
            K, C, R, S = w.shape
            nf, ndg = K * R * S * cp, (C * R * S * K if nd else 0)
            layout.append((off, nf, off + (nf + 63) // 64 * 64 if nd else -1, ndg))
            off += (nf + 63) // 64 * 64 + (ndg + 63) // 64 * 64
        self.buf = torch.empty((max(off, 1),), device=dev, dtype=BF16)
        for (w, cp, nd), (of, nf, od, ndg) in zip(specs, layout):
            K, C, R, S = w.shape
            wt = self.buf[of:of + nf]
            wtd = self.buf[od:od + ndg] if nd else None
            self._views[id(w)] = (wt, wtd)
            rows.append([w.data_ptr(), wt.data_ptr(), _p(wtd), K, C, R * S, cp, blk])
            blk += Cn.nhwc_repack_blocks(K, C, R, S, cp, True, bool(nd))
        self.blocks = blk
        self.desc = torch.tensor(rows, dtype=torch.int64).to(dev)
        self._key = tuple((id(w), w.data_ptr()) for w, _, _ in specs)
        self._specs = [(w, cp, nd) for w, cp, nd in specs]

    def matches(self, specs) -> bool:
        return len(specs) == len(self._key) and all(
            (id(w), w.data_ptr()) == k and (cp, nd) == (c2, n2)
            for (w, cp, nd), k, (_, c2, n2) in zip(specs, self._key, self._specs))

    def refresh(self, stream=None):
        st = stream if stream is not None else torch.cuda.current_stream(self.buf.device).cuda_stream
        native().nhwc_repack_many(self.desc.data_ptr(), self.desc.shape[0], self.blocks, st)

    def get(self, w):
        return self._views.get(id(w))


class _BnLink:
    """What the data gradient of a convolution needs to compute the backward statistics of the
    training BatchNorm whose output it consumes (csrc/nhwc_bf16.hip ConvNArgs::bx): the BN's
    input, batch mean and ReLU-mask source.  The BN forward attaches it to its output; the
    consumer conv's backward fills ``pre`` (partials, rows, data pointer of the gradient it
    wrote) and the BN backward uses it when that gradient is exactly its dy.  ``join``: the
    output also feeds a residual shortcut (fork): the conv's gradient is the BN's whole output
    gradient only when the shortcut's gradient was added in its epilogue."""

    __slots__ = ("x", "mean", "fcoef", "mask", "relu", "join", "pre")

    def __init__(self, x, mean, fcoef, mask, relu):
        self.x, self.mean, self.fcoef, self.mask, self.relu = x, mean, fcoef, mask, relu
        self.join = None
        self.pre = None


def _bn_link_of(x):
    link = getattr(x, "_mx_bnlink", None)
    if link is None or link[1] != x._version:  # written in place since the BN: not its output any more
        return None
    return link[0]


class GradJoin:
    """Joins the two input-gradient branches of a residual block without a separate add: the
    shortcut branch leaves its input gradient here -- the block's last batch norm (whose ``res``
    is the identity shortcut), or the projection shortcut's convolution (``conv2d(..., deposit=)``)
    -- and the block's first convolution adds it in its data-gradient epilogue
    (``nhwc_conv_dgrad(..., addend)``).  ``fork`` then passes that sum through unchanged.  If the
    first convolution's backward runs before the shortcut's, nothing is joined and ``fork`` adds.
    An identity shortcut's gradient is never materialised: the last BN leaves its own output
    gradient and ReLU mask bits (``amask``), and the conv's epilogue masks while it adds.  A
    stride-2 1x1 projection leaves its input gradient at half resolution (``sub2``: nonzero only
    at even (h, w), computed as a stride-1 GEMM on the output grid) and the 1x1 first conv's
    epilogue adds it there."""

    def __init__(self):
        self.dres = None
        self.amask = None
        self.sub2 = False
        self.consumed = False


def _mask_bits(g, mask):
    """g with element i zeroed unless bit i % 8 of mask[i // 8] is set (fallback of a lazy join)."""
    bits = (mask.view(-1, 1) >> torch.arange(8, device=mask.device, dtype=torch.uint8)) & 1
    return g * bits.view(g.shape).to(g.dtype)


class _Fork(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, join):
        ctx.join = join
        ctx.shape = x.shape
        ctx.set_materialize_grads(False)  # a lazy identity join leaves g_short undefined
        return x.view_as(x), x.view_as(x)

    @staticmethod
    def backward(ctx, g_main, g_short):
        j = ctx.join
        if j.consumed:  # g_main already includes g_short (added by the conv's epilogue)
            out = g_main
        elif g_short is None and j.dres is not None and j.sub2:  # half-resolution projection, not joined
            out = g_main.clone() if g_main is not None else j.dres.new_zeros(ctx.shape)
            out[:, ::2, ::2, :] += j.dres
        else:
            if g_short is None and j.dres is not None:  # lazy identity gradient, never joined
                g_short = _mask_bits(j.dres, j.amask) if j.amask is not None else j.dres
            if g_main is None or g_short is None:
                out = g_main if g_short is None else g_short
            else:
                out = g_main + g_short
        j.dres, j.amask, j.sub2, j.consumed = None, None, False, False
        return out, None


def fork(x, join: GradJoin):
    """(main, shortcut) aliases of a residual block's input; pass ``join`` to the block's first
    conv2d and last batch_norm so the two gradients are summed inside the conv's epilogue."""
    link = _bn_link_of(x)
    main, short = _Fork.apply(x, join)
    if link is not None:  # only the main branch's conv may compute the producing BN's statistics
        link.join = join
        main._mx_bnlink = (link, main._version)
    return main, short


class _Conv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, pad, packed=None, join=None, deposit=None, bnstat=None):
        Cn = native()
        # the BN that produced x (its backward statistics can ride this conv's data gradient)
        dstats = _BN_STATS_IN_DGRAD or x.numel() <= _BN_DGRAD_STATS_MAX
        ctx.bnlink = _bn_link_of(x) if (dstats and ctx.needs_input_grad[0]) else None
        N, H, W, Cp = x.shape
        K, C, R, S = w.shape
        sh, sw = stride
        ph, pw = pad
        P, Q = _out(H, R, sh, ph), _out(W, S, sw, pw)
        st = stream_of(x)
        need_dx = ctx.needs_input_grad[0] and Cp == C
        if packed is not None and (packed[1] is not None or not need_dx):
            wt, wtd = packed  # repacked for the whole model by WeightPack.refresh()
        else:
            wt = torch.empty((K * R * S * Cp,), device=x.device, dtype=BF16)
            # the data-gradient layout is produced in the same launch when backward will need it
            wtd = torch.empty((C * R * S * K,), device=x.device, dtype=BF16) if need_dx else None
            Cn.nhwc_repack_weight(w.data_ptr(), wt.data_ptr(), _p(wtd), K, C, R, S, Cp, st)
        y = torch.empty((N, P, Q, K), device=x.device, dtype=BF16)
        scr = _splitk_scratch(N * P * Q, K, R * S * Cp, x.device)
        gx = Cn.nhwc_conv_fwd(x.data_ptr(), wt.data_ptr(), y.data_ptr(), N, H, W, Cp, K, R, S, sh, sw, ph, pw, P, Q,
                              _p(scr), st, _p(bnstat[0]) if bnstat else 0, _p(bnstat[1]) if bnstat else 0)
        if bnstat:
            bnstat[2] = gx
        ctx.wtd = wtd
        ctx.join = join
        ctx.deposit = deposit
        ctx.save_for_backward(x, w)
        ctx.geom = (N, H, W, Cp, K, C, R, S, sh, sw, ph, pw, P, Q)
        return y

    @staticmethod
    def backward(ctx, dy):
        Cn = native()
        x, w = ctx.saved_tensors
        N, H, W, Cp, K, C, R, S, sh, sw, ph, pw, P, Q = ctx.geom
        dy = dy.contiguous()
        st = stream_of(dy)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            if Cp != C:
                raise NotImplementedError("nhwc conv: input gradient of a channel-padded input")
            wtd = ctx.wtd
            if wtd is None:
                wtd = torch.empty((C * R * S * K,), device=dy.device, dtype=BF16)
                Cn.nhwc_repack_weight(w.data_ptr(), 0, wtd.data_ptr(), K, C, R, S, Cp, st)
            if (_SUB2_DEPOSIT and ctx.deposit is not None and R == S == 1 and (sh, sw) == (2, 2)
                    and (ph, pw) == (0, 0) and H == 2 * P and W == 2 * Q):
                # stride-2 1x1 projection: its input gradient is nonzero at even (h, w) only --
                # computed there as a stride-1 GEMM on the P x Q grid and left at half resolution
                # for the block's first conv to add (GradJoin.sub2); nothing returned to autograd
                dxc = torch.empty((N, P, Q, C), device=dy.device, dtype=BF16)
                n = Cn.nhwc_conv_dgrad_scratch_floats(N, P, Q, C, K, 1, 1, 1, 1, 0, 0, P, Q)
                scr = torch.empty((n,), device=dy.device, dtype=torch.float32) if n else None
                Cn.nhwc_conv_dgrad(dy.data_ptr(), wtd.data_ptr(), dxc.data_ptr(), N, P, Q, C, K, 1, 1, 1, 1, 0, 0,
                                   P, Q, _p(scr), st)
                ctx.deposit.dres, ctx.deposit.amask, ctx.deposit.sub2 = dxc, None, True
            else:
                dx = torch.empty((N, H, W, C), device=dy.device, dtype=BF16)
                n = Cn.nhwc_conv_dgrad_scratch_floats(N, H, W, C, K, R, S, sh, sw, ph, pw, P, Q)
                scr = torch.empty((n,), device=dy.device, dtype=torch.float32) if n else None
                j = ctx.join
                add, sub = None, False
                if j is not None and j.dres is not None:
                    if j.dres.shape == dx.shape and not j.sub2:
                        add = j.dres
                    elif (j.sub2 and R == S == 1 and (sh, sw) == (1, 1) and H % 2 == 0 and W % 2 == 0
                          and j.dres.shape == (N, H // 2, W // 2, C)):
                        add, sub = j.dres, True
                amask = j.amask if add is not None else None
                link = ctx.bnlink
                if link is not None and link.join is not None and add is None:
                    link = None  # the shortcut's gradient is not in this sum: not the BN's whole dy
                bpart = None
                if link is not None and link.x.shape == dx.shape:
                    rows = Cn.nhwc_conv_dgrad_bn_rows(N, H, W, C, K, R, S, sh, sw, ph, pw, P, Q)
                    bpart = torch.empty((rows * 2 * C,), device=dy.device, dtype=torch.float32)
                rows = Cn.nhwc_conv_dgrad(dy.data_ptr(), wtd.data_ptr(), dx.data_ptr(), N, H, W, C, K, R, S, sh, sw,
                                          ph, pw, P, Q, _p(scr), st, _p(add), _p(bpart),
                                          _p(link.x) if bpart is not None else 0,
                                          _p(link.mean) if bpart is not None else 0,
                                          _p(link.fcoef) if bpart is not None else 0,
                                          _p(link.mask) if bpart is not None else 0,
                                          bool(link.relu) if bpart is not None else False, _p(amask), sub)
                if bpart is not None and rows > 0:
                    # (partials, rows, the gradient tensor's address and version): autograd may sum
                    # another consumer's gradient INTO dx in place (var.add_(old_var)) before the BN
                    # sees it -- same address, bumped version -- and then these partials are stale
                    link.pre = (bpart, rows, dx.data_ptr(), dx._version)
                if add is not None:
                    j.consumed = True
                if ctx.deposit is not None:
                    # picked up by the block's first conv (GradJoin)
                    ctx.deposit.dres, ctx.deposit.amask, ctx.deposit.sub2 = dx, None, False
        if ctx.needs_input_grad[1]:
            sink = _grad_sink(w)
            dw = sink if sink is not None else torch.empty_like(w)
            part = torch.empty((Cn.nhwc_wgrad_scratch_floats(N, Cp, K, R, S, P, Q),), device=dy.device,
                               dtype=torch.float32)
            def _wgrad():
                Cn.nhwc_conv_wgrad(dy.data_ptr(), x.data_ptr(), dw.data_ptr(), N, H, W, C, Cp, K, R, S, sh, sw, ph,
                                   pw, P, Q, sink is not None, part.data_ptr(), st)
            if _ops._WGRAD_DEFER and sink is not None:
                _ops.wgrad_defer_call(_wgrad, part, dy.device, st)
            else:
                _wgrad()
            if sink is not None:
                dw = None
        return dx, dw, None, None, None, None, None, None


def conv2d(x, w, stride=1, padding=0, pack: WeightPack | None = None, join: GradJoin | None = None,
           deposit: GradJoin | None = None, bn: torch.nn.BatchNorm2d | None = None):
    """bf16 NHWC convolution; ``pack`` supplies weights already repacked by WeightPack.refresh(),
    ``join`` (see ``fork``) adds a residual block's shortcut gradient to this conv's input gradient,
    ``deposit`` leaves this conv's input gradient in that join (a projection shortcut).  ``bn``: the
    training BatchNorm that consumes the output; the conv's epilogue then computes that BN's
    partial statistics where the kernel allows it (``batch_norm`` picks them up and skips its
    statistics pass)."""
    s = (stride, stride) if isinstance(stride, int) else tuple(stride)
    p = (padding, padding) if isinstance(padding, int) else tuple(padding)
    bnstat = None
    if bn is not None and bn.training and _BN_STATS_IN_CONV:
        N_, H_, W_, _ = x.shape
        K, _, R, S = w.shape
        P, Q = _out(H_, R, s[0], p[0]), _out(W_, S, s[1], p[1])
        rows = native().nhwc_conv_bn_rows(N_, H_, W_, x.shape[3], K, R, S, s[0], s[1], p[0], p[1], P, Q)
        if rows <= 16384:
            shift = bn.running_mean if bn.track_running_stats else None
            bnstat = [torch.empty((rows * 2 * K,), device=x.device, dtype=torch.float32), shift, 0]
    y = _Conv.apply(x, w, s, p, pack.get(w) if pack is not None else None, join, deposit, bnstat)
    if bnstat and bnstat[2] > 0:
        y._mx_bnpre = (bnstat[0], bnstat[2], bnstat[1], y._version)  # (partials, rows, shift, version)
    return y


# False: every BN runs its own statistics passes, forward and backward (the conv-epilogue
# statistics measured a win on every ResNet-50 layer, docs/BENCHMARKS.md; tests may flip it)
_BN_STATS_IN_CONV = True
# stride-2 1x1 projection shortcuts deposit their input gradient at half resolution (GradJoin.sub2;
# False: full resolution through the parity-class data gradient -- tests compare the two)
_SUB2_DEPOSIT = True
# Backward BN statistics in the consuming conv's data-gradient epilogue: OFF by default.  Measured
# per layer at batch 256 (scripts/bench_nhwc_layers.py, profiles/r4_d/rn_layers.log) the epilogue
# adds 2.9 ms to the step's data gradients (the LDS-DMA kernel runs one block per CU, so the x
# re-read and the reduction of every tile are fully exposed) against the 1.6 ms of separate
# statistics passes it removes.  Tests switch it on to keep the path exact.
_BN_STATS_IN_DGRAD = False
# ... except on tensors of at most this many elements (MXDDP_BN_DGRAD_STATS_MAX; 0 = never), where
# the separate statistics pass is mostly its fixed per-kernel cost (~5 us a launch at batch 32).
# ResNet-50 (profiles/r4_r/, two runs each): batch 32 5,332 img/s at 0, 5,352 at 4M (layers 2-4),
# 5,266 at every size; batch 256 unchanged (its smallest BN tensor has 6.4M elements)
_BN_DGRAD_STATS_MAX = int(os.environ.get("MXDDP_BN_DGRAD_STATS_MAX", "4000000"))
_LAZY_JOIN = True  # identity-shortcut gradient masked in the joining conv's epilogue (tests flip it)
# how many BN backward passes took their statistics from a conv epilogue / ran their own pass
BN_BWD_STATS = {"epilogue": 0, "pass": 0}


class _BN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, rm, rv, nbt, res, relu, momentum, eps, join=None, pre=None):
        Cn = native()
        N, H, W, C = x.shape
        npix = N * H * W
        y = torch.empty_like(x)
        mean = torch.empty((C,), device=x.device, dtype=torch.float32)
        invstd = torch.empty_like(mean)
        scr = torch.empty((Cn.nhwc_bn_scratch_floats(npix, C),), device=x.device, dtype=torch.float32)
        # ReLU without residual: keep the affine coefficients, the backward rebuilds the mask from x
        fcoef = torch.empty((2 * C,), device=x.device, dtype=torch.float32) if (relu and res is None and C <= 512) \
            else None
        # any other ReLU: the forward stores its mask as bits (1/16 of y's bytes), read by the
        # backward's two passes instead of y
        mask = torch.empty((npix * C // 8,), device=x.device, dtype=torch.uint8) if (relu and fcoef is None) else None
        part, rows, shift = pre if pre is not None else (None, 0, None)
        Cn.nhwc_bn_fwd(x.data_ptr(), _p(res), y.data_ptr(), _p(gamma), _p(beta), mean.data_ptr(), invstd.data_ptr(),
                       _p(rm), _p(rv), _p(nbt), npix, C, float(momentum), float(eps), bool(relu), scr.data_ptr(),
                       stream_of(x), _p(fcoef), _p(mask), _p(part), rows, _p(shift))
        ctx.fcoef = fcoef
        ctx.mask = mask
        ctx.save_for_backward(x, gamma, mean, invstd)
        ctx.relu, ctx.has_res = bool(relu), res is not None
        ctx.join = join
        ctx.refs = (gamma, beta)
        # for the consuming conv's data gradient: its epilogue can compute this BN's backward
        # statistics (the mask source must be the one this backward uses: fcoef, else the bits)
        ctx.link = _BnLink(x, mean, fcoef, mask, bool(relu))
        return y

    @staticmethod
    def backward(ctx, dy):
        Cn = native()
        x, gamma, mean, invstd = ctx.saved_tensors
        N, H, W, C = x.shape
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        # identity shortcut joined in the block's first conv: its gradient (dy masked by this BN's
        # ReLU bits) is not written here, the conv's epilogue reads dy and the bits instead
        lazy = ctx.has_res and ctx.join is not None and _LAZY_JOIN and (not ctx.relu or ctx.mask is not None)
        dres = torch.empty_like(x) if (ctx.has_res and not lazy) else None
        g_ref, b_ref = ctx.refs
        gs, bs = _grad_sink(g_ref), _grad_sink(b_ref)
        direct = gs is not None and bs is not None
        dg, db = (gs, bs) if direct else (torch.empty((C,), device=x.device), torch.empty((C,), device=x.device))
        scr = torch.empty((Cn.nhwc_bn_scratch_floats(N * H * W, C),), device=x.device, dtype=torch.float32)
        # backward statistics from the consuming conv's data-gradient epilogue, valid only for
        # exactly the gradient tensor that conv wrote, unmodified since (a second consumer's
        # gradient accumulated into it in place bumps its version)
        pre = ctx.link.pre
        ctx.link.pre = None
        if pre is not None and (pre[2] != dy.data_ptr() or pre[3] != dy._version):
            pre = None
        BN_BWD_STATS["epilogue" if pre is not None else "pass"] += 1
        Cn.nhwc_bn_bwd(dy.data_ptr(), x.data_ptr(), 0, _p(gamma), mean.data_ptr(), invstd.data_ptr(),
                       dx.data_ptr(), _p(dres), dg.data_ptr(), db.data_ptr(), N * H * W, C, ctx.relu, direct,
                       scr.data_ptr(), stream_of(dy), _p(ctx.fcoef), _p(ctx.mask),
                       _p(pre[0]) if pre is not None else 0, pre[1] if pre is not None else 0)
        if direct:
            dg = db = None
        if lazy:
            ctx.join.dres, ctx.join.amask = dy, (ctx.mask if ctx.relu else None)
        elif ctx.join is not None and dres is not None:
            ctx.join.dres, ctx.join.amask = dres, None  # picked up by the block's first conv (epilogue)
        return dx, dg, db, None, None, None, dres, None, None, None, None, None


def batch_norm(x, bn: torch.nn.BatchNorm2d, relu: bool = False, res: torch.Tensor | None = None,
               join: GradJoin | None = None):
    """Training-mode BN of an NHWC bf16 tensor with the module's parameters / buffers (running
    stats and num_batches_tracked updated on device), fused ReLU and residual add (y = relu(bn(x) +
    res)).  Eval mode uses the running statistics (plain tensor math)."""
    if bn.training or not bn.track_running_stats:
        mom = bn.momentum if bn.momentum is not None else 0.1
        nbt = bn.num_batches_tracked if (bn.training and bn.track_running_stats) else None
        # partial statistics from the producing conv's epilogue (conv2d(..., bn=bn)), valid only
        # for this exact tensor and shifted by this BN's running mean
        # (an in-place change of x since the conv bumped its version: the partials are stale)
        pre = getattr(x, "_mx_bnpre", None)
        if pre is not None and (pre[2] is not (bn.running_mean if bn.track_running_stats else None)
                                or pre[0].numel() < pre[1] * 2 * x.shape[-1] or pre[3] != x._version):
            pre = None
        if pre is not None:
            pre = pre[:3]
        y = _BN.apply(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, nbt, res, relu, mom, bn.eps, join, pre)
        link = getattr(y.grad_fn, "link", None)  # the node is the Function's ctx
        if link is not None:
            y._mx_bnlink = (link, y._version)
        return y
    y = (x.float() - bn.running_mean) * torch.rsqrt(bn.running_var + bn.eps) * bn.weight + bn.bias
    if res is not None:
        y = y + res.float()
    return (y.relu() if relu else y).to(BF16)


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        N, H, W, C = x.shape
        P, Q = _out(H, k, s, p), _out(W, k, s, p)
        y = torch.empty((N, P, Q, C), device=x.device, dtype=BF16)
        arg = torch.empty((N, P, Q, C), device=x.device, dtype=torch.uint8)
        native().nhwc_maxpool_fwd(x.data_ptr(), y.data_ptr(), arg.data_ptr(), N, H, W, C, P, Q, k, s, p, stream_of(x))
        ctx.save_for_backward(arg)
        ctx.geom = (N, H, W, C, P, Q, k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        N, H, W, C, P, Q, k, s, p = ctx.geom
        dy = dy.contiguous()
        dx = torch.empty((N, H, W, C), device=dy.device, dtype=BF16)
        native().nhwc_maxpool_bwd(dy.data_ptr(), arg.data_ptr(), dx.data_ptr(), N, H, W, C, P, Q, k, s, p,
                                  stream_of(dy))
        return dx, None, None, None


def max_pool2d(x, k, s, p):
    return _MaxPool.apply(x, k, s, p)


class _GAP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        N, H, W, C = x.shape
        y = torch.empty((N, C), device=x.device, dtype=torch.float32)
        native().nhwc_gap_fwd(x.data_ptr(), y.data_ptr(), N, H * W, C, stream_of(x))
        ctx.geom = (N, H, W, C)
        return y

    @staticmethod
    def backward(ctx, dy):
        N, H, W, C = ctx.geom
        dy = dy.contiguous()
        dx = torch.empty((N, H, W, C), device=dy.device, dtype=BF16)
        native().nhwc_gap_bwd(dy.data_ptr(), dx.data_ptr(), N, H * W, C, stream_of(dy))
        return dx


def global_avg_pool(x):
    """bf16 [N, H, W, C] -> fp32 [N, C] (the classifier runs on fp32 features)."""
    return _GAP.apply(x)
