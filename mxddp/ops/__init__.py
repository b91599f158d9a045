"""Differentiable ops backed by the gfx950 HIP kernels in ``mxddp/csrc``.

Every op has two implementations selected by the *device of its input* only:

* CUDA (= ROCm HIP) tensors -> the native kernels (``mxddp._C``).  There is no silent
  fallback: if the extension cannot be loaded the op raises.
* CPU tensors -> plain PyTorch reference math (BASELINE config 1, CPU single process,
  and the fp32 oracle that the GPU numerics tests compare against).

Reference call sites replaced (cuDNN/cuBLAS/ATen via torch.nn in the reference):
conv / BN / pool / linear in ``pytorch/model.py:28-33,62-77``, CrossEntropyLoss in
``pytorch/single_gpu.py:70``, Keras layers in ``tensorflow2/mnist_single.py:16-26``.
"""
from __future__ import annotations

import os
import weakref

import torch
import torch.nn.functional as F

from .. import native

__all__ = [
    "conv2d", "linear", "relu", "max_pool2d", "avg_pool2d", "batch_norm", "cross_entropy",
    "shortcut_pad_add", "stream_of", "refresh_filters", "invalidate_filters",
]


_TORCH_REFERENCE = False  # bench/debug only: route GPU tensors through stock PyTorch ops


class torch_reference_mode:
    """Context manager: run GPU tensors through stock PyTorch-ROCm ops instead of the mxddp
    kernels.  Used only by ``bench.py --impl torch`` to measure the baseline; never a default."""

    def __enter__(self):
        global _TORCH_REFERENCE
        self._prev, _TORCH_REFERENCE = _TORCH_REFERENCE, True
        return self

    def __exit__(self, *exc):
        global _TORCH_REFERENCE
        _TORCH_REFERENCE = self._prev


def torch_reference_active() -> bool:
    """True inside ``torch_reference_mode``: models must not take a native-only path."""
    return _TORCH_REFERENCE


def _native(t: torch.Tensor) -> bool:
    return t.is_cuda and not _TORCH_REFERENCE


def stream_of(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _p(t):
    return 0 if t is None else t.data_ptr()


def _check(t: torch.Tensor, name: str):
    if t.dtype != torch.float32:
        raise TypeError(f"mxddp native op: {name} must be float32, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"mxddp native op: {name} must be contiguous")


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


# ------------------------------------------------------------- direct gradient writing
# Parameters re-homed into a flat buffer (mxddp.parallel.flat.FlatParams) carry
# ``_mx_grad_ready``: their ``.grad`` is a view of the flat gradient buffer, so the backward
# kernels accumulate straight into it (accumulate=True; zero_grad zeroes the buffer once per
# step) and the op returns None to autograd.  That removes one temporary gradient tensor and
# one autograd accumulation kernel per parameter per step (415 for PyramidNet).  Autograd still
# runs the parameter's AccumulateGrad node (with no gradient) and its post-accumulate-grad
# hooks, so DDP's bucket-readiness hook fires exactly as on the returned-gradient path.
def _grad_sink(p):
    if p is None or not p.requires_grad:
        return None
    cb = getattr(p, "_mx_grad_ready", None)
    g = p.grad
    if cb is None or g is None or not g.is_contiguous() or g.dtype != torch.float32:
        return None
    return g


def _grad_done(p):
    """Gradient written in place; readiness is signalled by autograd's post-accumulate hook."""
    return None


# ------------------------------------------------------------- persistent Winograd filters
# A 3x3 stride-1 conv on the Winograd path needs its filters transformed (forward: G w G^T,
# data gradient: of the flipped / transposed w) once per weight update.  Instead of one
# transform launch per conv per forward, every such conv registers persistent filter buffers in
# a per-device native bank (csrc WinoFilterBank) and the optimizer re-transforms ALL of them in
# one launch per 64 convs right after its step (refresh_filters).  A forward uses the banked
# filters only while they are provably current: same bank generation (no unreported raw write
# since the last refresh) and same tensor version (no torch in-place write, e.g. a checkpoint
# load); otherwise it transforms as before, into the bank's buffers.
class _Bank:
    def __init__(self):
        self.native = native().WinoFilterBank()
        self.entries = {}  # (weight data_ptr, K, C) -> entry
        self.gen = 0


_BANKS: dict = {}


class _FilterEntry:
    __slots__ = ("ref", "w", "U", "Ud", "version", "gen")

    def __init__(self, param, U, Ud):
        # the native bank keeps raw pointers: the entry holds the weight storage (a detached
        # alias, same version counter) and both buffers; `ref` lets a dead model's entries go
        self.ref, self.w, self.U, self.Ud = weakref.ref(param), param.detach(), U, Ud
        self.version, self.gen = -1, -1


def _rebuild(bank) -> None:
    dead = [k for k, e in bank.entries.items() if e.ref() is None]
    for k in dead:
        del bank.entries[k]
    bank.native.clear()
    for e in bank.entries.values():
        bank.native.add(e.w.data_ptr(), e.U.data_ptr(), _p(e.Ud), e.w.shape[0], e.w.shape[1])


_BANK_ON = True  # False: per-conv transforms (tests compare the two)


# ------------------------------------------------------ deferred weight-gradient reductions
# (csrc/wgrad_defer.h) A conv whose weight gradient goes straight into a flat gradient buffer
# (FlatParams sink) may leave its split-K partial planes for the optimizer to sum: the mxddp
# optimizers call flush_wgrad() before their update, which sums every pending plane set of the
# device in a few batched launches -- one reduce launch per conv per step fewer (PyramidNet ~100,
# ResNet-50 53).  Opt-in (set_wgrad_defer), and only sound when nothing but the optimizer reads
# the gradient between the backward and the step: no DDP bucket all-reduce (world size 1), no
# in-process replica exchange, no gradient clipping.  The scratch planes of each deferred call
# are kept alive here until the flush.
_WGRAD_DEFER = False
_WGRAD_KEEP: dict = {}
# Pending partial planes are flushed early (on the backward's own stream) once they pass this
# many bytes, so a batch is summed while its planes still sit in the Infinity Cache instead of
# after the whole backward has pushed them out to HBM (MXDDP_WGRAD_FLUSH_MB; 0 = only at the step)
_WGRAD_FLUSH_BYTES = int(float(os.environ.get("MXDDP_WGRAD_FLUSH_MB", "64")) * (1 << 20))


def set_wgrad_defer(on: bool) -> None:
    global _WGRAD_DEFER
    _WGRAD_DEFER = bool(on)


def set_wgrad_flush_mb(mb: float) -> None:
    global _WGRAD_FLUSH_BYTES
    _WGRAD_FLUSH_BYTES = int(float(mb) * (1 << 20))


def wgrad_defer_call(fn, keep, device, stream=None):
    """Run one weight-gradient call that may defer its reduction; keeps `keep` (its partial
    planes) alive until the flush if it did.  Past _WGRAD_FLUSH_BYTES of pending planes the
    device's pending reductions are summed right away on `stream` (the call's own stream)."""
    C = native()
    C.wgrad_defer_set(True)
    try:
        out = fn()
        took = C.wgrad_defer_took()
    finally:
        C.wgrad_defer_set(False)
    if took:
        ent = _WGRAD_KEEP.setdefault(device, [0, []])
        ent[0] += keep.numel() * keep.element_size()
        ent[1].append(keep)
        if _WGRAD_FLUSH_BYTES > 0 and ent[0] >= _WGRAD_FLUSH_BYTES:
            with torch.cuda.device(device):
                C.wgrad_defer_flush(stream if stream is not None else torch.cuda.current_stream(device).cuda_stream)
            del _WGRAD_KEEP[device]
    return out


def flush_wgrad(device=None) -> int:
    """Sum every deferred weight-gradient reduction of `device` (current stream); returns how
    many.  Called by the mxddp optimizers before their update."""
    if not _WGRAD_KEEP:
        return 0
    n = 0
    for dev in list(_WGRAD_KEEP):
        if device is not None and torch.device(dev) != torch.device(device):
            continue
        with torch.cuda.device(dev):
            n += native().wgrad_defer_flush(torch.cuda.current_stream(dev).cuda_stream)
        del _WGRAD_KEEP[dev]
    return n


def _filter_entry(w, geom, needs_dgrad):
    """This conv's banked filters (created and registered on first use), or None if the shape
    does not run the Winograd path or the weight is not a leaf parameter."""
    if not (_BANK_ON and w.is_leaf):
        return None
    C = native()
    nf = C.conv_fwd_filter_floats(*geom)
    if not nf:
        return None
    bank = _BANKS.get(w.device)
    if bank is None:
        bank = _BANKS[w.device] = _Bank()
    key = (w.data_ptr(), w.shape[0], w.shape[1])
    ent = bank.entries.get(key)
    if ent is not None and ent.ref() is not w:  # storage reused by another tensor
        ent = None
    if ent is None or (needs_dgrad and ent.Ud is None):
        nd = C.conv_dgrad_filter_floats(*geom) if needs_dgrad else 0
        U = torch.empty((nf,), device=w.device, dtype=torch.float32)
        Ud = torch.empty((nd,), device=w.device, dtype=torch.float32) if nd else None
        ent = _FilterEntry(w, U, Ud)
        bank.entries[key] = ent
        _rebuild(bank)
    return ent, bank


def refresh_filters(device=None) -> None:
    """Re-transform every banked Winograd filter (one launch per 64 convs, on the current stream).
    Called by the mxddp optimizers right after their (raw-pointer) weight update."""
    for dev, bank in _BANKS.items():
        if device is not None and dev != device:
            continue
        bank.gen += 1
        if any(e.ref() is None for e in bank.entries.values()):
            _rebuild(bank)
        if bank.entries:
            bank.native.refresh(torch.cuda.current_stream(dev).cuda_stream)
            for e in bank.entries.values():
                e.version, e.gen = e.w._version, bank.gen


def invalidate_filters(device=None) -> None:
    """Weights changed behind torch's back without a refresh: banked filters are stale."""
    for dev, bank in _BANKS.items():
        if device is None or dev == device:
            bank.gen += 1


# --------------------------------------------------------------------------- conv2d
class _Conv2d(torch.autograd.Function):
    """``in_ss`` ([Cin, 2], optional): x is a folded BN's INPUT and the convolution consumes
    relu?(x * in_ss[c, 0] + in_ss[c, 1]) (``bn_conv``); the forward and the weight gradient form it
    while staging their input tiles, and the gradient returned for x is the gradient of that
    (unstored) BN output, which the folded BN's backward turns into its own."""

    @staticmethod
    def forward(ctx, x, w, b, stride, padding, dilation, relu, in_ss=None, in_relu=False):
        C = native()
        x = x.contiguous()
        _check(x, "input"); _check(w, "weight")
        N, Cin, H, W = x.shape
        K, Cw, R, S = w.shape
        if Cw != Cin:
            raise ValueError(f"conv2d: weight expects {Cw} input channels, got {Cin}")
        sh, sw = stride; ph, pw = padding; dh, dw = dilation
        P = (H + 2 * ph - dh * (R - 1) - 1) // sh + 1
        Q = (W + 2 * pw - dw * (S - 1) - 1) // sw + 1
        y = torch.empty((N, K, P, Q), device=x.device, dtype=x.dtype)
        st = stream_of(x)
        geom = (N, Cin, H, W, K, R, S, sh, sw, ph, pw, dh, dw)
        fe = _filter_entry(w, geom, ctx.needs_input_grad[0])
        if fe is not None:  # Winograd layer: banked filters (see refresh_filters)
            ent, bank = fe
            fresh = ent.gen == bank.gen and ent.version == w._version
            C.conv2d_fwd(x.data_ptr(), w.data_ptr(), _p(b), y.data_ptr(), *geom, bool(relu), st, ent.U.data_ptr(),
                         _p(ent.Ud), fresh, _p(in_ss), bool(in_relu))
            if not fresh:  # transformed just now, into the bank's buffers
                ent.version, ent.gen = w._version, bank.gen
            wd = ent.Ud if ctx.needs_input_grad[0] else None
        else:
            ns = C.conv_scratch_floats(*geom)
            scr = torch.empty((ns,), device=x.device, dtype=x.dtype) if ns else None
            nd = C.conv_dgrad_filter_floats(*geom) if ctx.needs_input_grad[0] else 0
            wd = torch.empty((nd,), device=x.device, dtype=x.dtype) if nd else None
            C.conv2d_fwd(x.data_ptr(), w.data_ptr(), _p(b), y.data_ptr(), *geom, bool(relu), st, _p(scr), _p(wd),
                         False, _p(in_ss), bool(in_relu))
        ctx.dgrad_filters = wd
        ctx.in_ss, ctx.in_relu = in_ss, bool(in_relu)
        ctx.geom = (N, Cin, H, W, K, R, S, sh, sw, ph, pw, dh, dw, P, Q)
        ctx.relu = relu
        ctx.has_bias = b is not None
        ctx.bias_ref = b
        ctx.save_for_backward(x, w, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        C = native()
        x, w, y = ctx.saved_tensors
        N, Cin, H, W, K, R, S, sh, sw, ph, pw, dh, dw, P, Q = ctx.geom
        dy = dy.contiguous()
        st = stream_of(dy)
        if ctx.relu:
            g = torch.empty_like(dy)
            C.relu_bwd(dy.data_ptr(), y.data_ptr(), g.data_ptr(), dy.numel(), st)
            dy = g
        dx = dw_ = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            # scratch for the 3x3 paths' transformed / flipped filters (none needed otherwise)
            wt, pre = ctx.dgrad_filters, True
            if wt is None:
                ns = C.conv_scratch_floats(N, Cin, H, W, K, R, S, sh, sw, ph, pw, dh, dw)
                wt, pre = (torch.empty((ns,), device=dy.device, dtype=dy.dtype) if ns else None), False
            C.conv2d_dgrad(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), N, Cin, H, W, K, R, S, sh, sw, ph, pw,
                           dh, dw, 0, False, st, 0 if wt is None else wt.data_ptr(), pre)
        b = ctx.bias_ref
        bias_done = False
        if ctx.needs_input_grad[1]:
            sink = _grad_sink(w)
            dw_ = sink if sink is not None else torch.empty_like(w)
            ns = C.conv_wgrad_scratch_floats(N, Cin, H, W, K, R, S, sh, sw, ph, pw, dh, dw)
            ws = torch.empty((ns,), device=dy.device, dtype=dy.dtype) if ns else None
            # the bias gradient rides along as an extra GEMM column when both gradients go to the
            # same kind of destination (both flat-buffer sinks, or both fresh tensors)
            db_t = None
            if ctx.has_bias and ctx.needs_input_grad[2]:
                bsink = _grad_sink(b)
                if (bsink is None) == (sink is None):
                    db_t = bsink if bsink is not None else torch.empty((K,), device=dy.device, dtype=dy.dtype)
            def _wgrad():
                return C.conv2d_wgrad(dy.data_ptr(), x.data_ptr(), dw_.data_ptr(), N, Cin, H, W, K, R, S, sh, sw, ph,
                                      pw, dh, dw, sink is not None, st, _p(ws), _p(db_t), _p(ctx.in_ss), ctx.in_relu)
            if _WGRAD_DEFER and sink is not None and dy.is_cuda:
                bias_done = wgrad_defer_call(_wgrad, ws, dy.device, st)
            else:
                bias_done = _wgrad()
            if sink is not None:
                _grad_done(w)
                dw_ = None
            if bias_done:
                if db_t is bsink:
                    _grad_done(b)
                    db = None
                else:
                    db = db_t
        if ctx.has_bias and ctx.needs_input_grad[2] and not bias_done:
            sink = _grad_sink(b)
            db = sink if sink is not None else torch.empty((K,), device=dy.device, dtype=dy.dtype)
            C.bias_grad(dy.data_ptr(), db.data_ptr(), N, K, P * Q, sink is not None, st)
            if sink is not None:
                _grad_done(b)
                db = None
        return dx, dw_, db, None, None, None, None, None, None


def conv2d(x, w, b=None, stride=1, padding=0, dilation=1, relu=False, in_ss=None, in_relu=False):
    stride, padding, dilation = _pair(stride), _pair(padding), _pair(dilation)
    if _native(x):
        return _Conv2d.apply(x, w, b, stride, padding, dilation, relu, in_ss, in_relu)
    if in_ss is not None:
        x = x * in_ss[:, 0].view(1, -1, 1, 1) + in_ss[:, 1].view(1, -1, 1, 1)
        x = F.relu(x) if in_relu else x
    y = F.conv2d(x, w, b, stride, padding, dilation)
    return F.relu(y) if relu else y


# --------------------------------------------------------------------------- linear
class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, relu):
        C = native()
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        _check(x2, "input"); _check(w, "weight")
        M, K = x2.shape
        N = w.shape[0]
        y = torch.empty((M, N), device=x.device, dtype=x.dtype)
        st = stream_of(x)
        # ReLU in the GEMM epilogue (or in the split-K finish pass)
        C.linear_fwd(x2.data_ptr(), w.data_ptr(), _p(b), y.data_ptr(), M, N, K, bool(relu), st)
        ctx.relu = relu
        ctx.has_bias = b is not None
        ctx.bias_ref = b
        ctx.in_shape = x.shape
        ctx.save_for_backward(x2, w, y if relu else None)
        return y.reshape(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        C = native()
        x2, w, y = ctx.saved_tensors
        M, K = x2.shape
        N = w.shape[0]
        dy = dy.reshape(M, N).contiguous()
        st = stream_of(dy)
        # the fused ReLU's mask as one relu_bwd pass (applying it as the three GEMM / reduction
        # kernels load dy measured no faster inside a captured step: MLP 468-470k vs 471-480k)
        dm = 0
        if ctx.relu:
            g = torch.empty_like(dy)
            C.relu_bwd(dy.data_ptr(), y.data_ptr(), g.data_ptr(), dy.numel(), st)
            dy = g
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty((M, K), device=dy.device, dtype=dy.dtype)
            C.linear_dgrad(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), M, N, K, 0, False, st, dm)
            dx = dx.reshape(ctx.in_shape)
        if ctx.needs_input_grad[1]:
            sink = _grad_sink(w)
            dw = sink if sink is not None else torch.empty_like(w)
            C.linear_wgrad(dy.data_ptr(), x2.data_ptr(), dw.data_ptr(), M, N, K, sink is not None, st, dm)
            if sink is not None:
                _grad_done(w)
                dw = None
        if ctx.has_bias and ctx.needs_input_grad[2]:
            b = ctx.bias_ref
            sink = _grad_sink(b)
            db = sink if sink is not None else torch.empty((N,), device=dy.device, dtype=dy.dtype)
            C.bias_grad(dy.data_ptr(), db.data_ptr(), M, N, 1, sink is not None, st, dm)
            if sink is not None:
                _grad_done(b)
                db = None
        return dx, dw, db, None


def linear(x, w, b=None, relu=False):
    if _native(x):
        return _Linear.apply(x, w, b, relu)
    y = F.linear(x, w, b)
    return F.relu(y) if relu else y


# --------------------------------------------------------------------------- relu
class _Relu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        y = torch.empty_like(x)
        native().relu_fwd(x.data_ptr(), y.data_ptr(), x.numel(), stream_of(x))
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        native().relu_bwd(dy.data_ptr(), y.data_ptr(), dx.data_ptr(), dy.numel(), stream_of(dy))
        return dx


def relu(x):
    return _Relu.apply(x) if _native(x) else F.relu(x)


# --------------------------------------------------------------------------- pooling
def _pool_out(H, k, s, p, ceil):
    if ceil:
        o = -(-(H + 2 * p - k) // s) + 1
        if (o - 1) * s >= H + p:  # last window must start inside the (left-padded) input
            o -= 1
    else:
        o = (H + 2 * p - k) // s + 1
    return o


class _MaxPool2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p, ceil):
        x = x.contiguous()
        _check(x, "input")
        N, Cc, H, W = x.shape
        P, Q = _pool_out(H, k[0], s[0], p[0], ceil), _pool_out(W, k[1], s[1], p[1], ceil)
        y = torch.empty((N, Cc, P, Q), device=x.device, dtype=x.dtype)
        idx = torch.empty((N, Cc, P, Q), device=x.device, dtype=torch.int32)
        native().maxpool2d_fwd(x.data_ptr(), y.data_ptr(), idx.data_ptr(), N, Cc, H, W, k[0], k[1], s[0], s[1],
                               p[0], p[1], P, Q, stream_of(x))
        ctx.save_for_backward(idx)
        ctx.shape = (N, Cc, H, W, P, Q)
        # non-overlapping windows: the backward is a gather (no zero fill, no atomics)
        ctx.gather = (s[0], s[1]) if (tuple(k) == tuple(s) and tuple(p) == (0, 0)) else (0, 0)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        N, Cc, H, W, P, Q = ctx.shape
        dy = dy.contiguous()
        dx = torch.empty((N, Cc, H, W), device=dy.device, dtype=dy.dtype)
        native().maxpool2d_bwd(dy.data_ptr(), idx.data_ptr(), dx.data_ptr(), N, Cc, H, W, P, Q, stream_of(dy),
                               *ctx.gather)
        return dx, None, None, None, None


def max_pool2d(x, kernel_size, stride=None, padding=0, ceil_mode=False):
    k = _pair(kernel_size)
    s = _pair(stride if stride is not None else kernel_size)
    p = _pair(padding)
    if _native(x):
        return _MaxPool2d.apply(x, k, s, p, ceil_mode)
    return F.max_pool2d(x, k, s, p, ceil_mode=ceil_mode)


class _AvgPool2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p, ceil):
        x = x.contiguous()
        _check(x, "input")
        N, Cc, H, W = x.shape
        P, Q = _pool_out(H, k[0], s[0], p[0], ceil), _pool_out(W, k[1], s[1], p[1], ceil)
        y = torch.empty((N, Cc, P, Q), device=x.device, dtype=x.dtype)
        native().avgpool2d_fwd(x.data_ptr(), y.data_ptr(), N, Cc, H, W, k[0], k[1], s[0], s[1], p[0], p[1], P, Q,
                               stream_of(x))
        ctx.args = (N, Cc, H, W, k, s, p, P, Q)
        return y

    @staticmethod
    def backward(ctx, dy):
        N, Cc, H, W, k, s, p, P, Q = ctx.args
        dy = dy.contiguous()
        dx = torch.empty((N, Cc, H, W), device=dy.device, dtype=dy.dtype)
        native().avgpool2d_bwd(dy.data_ptr(), dx.data_ptr(), N, Cc, H, W, k[0], k[1], s[0], s[1], p[0], p[1], P, Q,
                               stream_of(dy))
        return dx, None, None, None, None


def avg_pool2d(x, kernel_size, stride=None, padding=0, ceil_mode=False):
    k = _pair(kernel_size)
    s = _pair(stride if stride is not None else kernel_size)
    p = _pair(padding)
    if _native(x):
        return _AvgPool2d.apply(x, k, s, p, ceil_mode)
    return F.avg_pool2d(x, k, s, p, ceil_mode=ceil_mode)


# --------------------------------------------------------------------------- batch norm
class _BatchNorm(torch.autograd.Function):
    """Train / eval BN (+ fused ReLU).  Two PyramidNet fusions (pytorch/model.py:40-50):

    * ``residual`` (tensor [N, Cr, H, W], Cr <= C): the block's identity shortcut with zero
      channel padding is added inside the normalise pass, y[:, :Cr] += residual; its gradient
      is handed back as a view of dy (no copy kernel).
    * ``tap``: a second output aliasing the input x for the shortcut branch; the gradient that
      branch sends back is added inside the dx pass, so the block input's two gradients are
      never summed by a separate launch (read in place from the next block's output gradient).
    """

    @staticmethod
    def forward(ctx, x, gamma, beta, running_mean, running_var, training, momentum, eps, relu, num_batches=None,
                residual=None, tap=False):
        C = native()
        x = x.contiguous()
        _check(x, "input")
        N, Cc = x.shape[0], x.shape[1]
        HW = x.numel() // (N * Cc)
        y = torch.empty_like(x)
        st = stream_of(x)
        res_c = 0
        if residual is not None:
            residual = residual.contiguous()
            _check(residual, "residual")
            res_c = residual.shape[1]
            if residual.shape[0] != N or residual.shape[2:] != x.shape[2:] or not 0 < res_c <= Cc or relu:
                raise ValueError("batch_norm residual: [N, Cr <= C, H, W] of the input's size, no fused ReLU")
        if training:
            mean = torch.empty((Cc,), device=x.device, dtype=torch.float32)
            invstd = torch.empty_like(mean)
            part = _bn_part(x.device, C.bn_partial_floats(N, Cc, HW))
            C.bn_fwd_train(x.data_ptr(), _p(gamma), _p(beta), y.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                           _p(running_mean), _p(running_var), N, Cc, HW, float(momentum), float(eps), bool(relu),
                           part.data_ptr(), st, _p(num_batches), _p(residual), res_c)
        else:
            mean = running_mean
            invstd = (running_var + eps).rsqrt()
            C.bn_fwd_eval(x.data_ptr(), _p(gamma), _p(beta), y.data_ptr(), running_mean.data_ptr(),
                          running_var.data_ptr(), N, Cc, HW, float(eps), bool(relu), st)
            if residual is not None:
                y[:, :res_c] += residual
        ctx.save_for_backward(x, gamma, mean, invstd, y if relu else None)
        ctx.dims = (N, Cc, HW)
        ctx.has_affine = gamma is not None
        ctx.affine_refs = (gamma, beta)
        ctx.res_c = res_c
        ctx.tap = tap
        if tap:
            return y, x
        return y

    @staticmethod
    def backward(ctx, dy, dtap=None):
        x, gamma, mean, invstd, y = ctx.saved_tensors
        N, Cc, HW = ctx.dims
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        g_ref, b_ref = ctx.affine_refs
        gs, bs = (_grad_sink(g_ref), _grad_sink(b_ref)) if ctx.has_affine else (None, None)
        direct = gs is not None and bs is not None
        if direct:
            dg, db = gs, bs
        else:
            dg = torch.empty((Cc,), device=x.device) if ctx.has_affine else None
            db = torch.empty((Cc,), device=x.device) if ctx.has_affine else None
        ext, ext_c = None, 0
        if dtap is not None:
            # usually a channel slice of the next block's output gradient: read it in place
            s_ = dtap.stride()
            W = x.shape[-1] if x.dim() >= 3 else 1
            in_place = (dtap.dim() == 4 and s_[3] == 1 and s_[2] == W and s_[1] == HW and s_[0] % HW == 0
                        and s_[0] // HW >= Cc and dtap.dtype == torch.float32)
            ext = dtap if in_place else dtap.contiguous()
            ext_c = s_[0] // HW if in_place else Cc
        part = _bn_part(x.device, native().bn_partial_floats(N, Cc, HW))
        native().bn_bwd(dy.data_ptr(), x.data_ptr(), _p(y), _p(gamma), mean.data_ptr(), invstd.data_ptr(),
                        dx.data_ptr(), _p(dg), _p(db), N, Cc, HW, direct, part.data_ptr(), stream_of(dy),
                        _p(ext), ext_c)
        if direct:
            _grad_done(g_ref)
            _grad_done(b_ref)
            dg = db = None
        dres = dy.narrow(1, 0, ctx.res_c) if ctx.res_c and ctx.needs_input_grad[10] else None
        return dx, dg, db, None, None, None, None, None, None, None, dres, None


_BN_PART: dict = {}
_BN_PART_RETIRED: list = []


def _bn_part(device, n, stream=None):
    """Partial-sum scratch of the split-reduction BN kernels (ops_bn.hip), one per (device,
    stream): every call rewrites what it reads and the BN calls of one stream are ordered, so one
    buffer serves them all (and a captured graph replays without any reset); BNs issued on two
    streams at once get two buffers (no cross-stream race on the partials).  When a wider layer
    needs a bigger buffer the old one is RETIRED, never freed: a hipGraph captured earlier bakes
    its address into its kernel arguments, and freeing it would leave those replays writing into
    memory the caching allocator has handed to someone else."""
    if stream is None:
        stream = torch.cuda.current_stream(device).cuda_stream
    key = (device, stream)
    buf = _BN_PART.get(key)
    if buf is None or buf.numel() < n:
        if buf is not None:
            _BN_PART_RETIRED.append(buf)
        buf = torch.empty((max(n, 8192),), dtype=torch.float32, device=device)
        _BN_PART[key] = buf
    return buf


def batch_norm(x, gamma, beta, running_mean, running_var, training, momentum=0.1, eps=1e-5, relu=False,
               num_batches=None, residual=None, tap=False):
    """``num_batches`` (int64 tensor, GPU path): incremented on device by the BN kernel
    (BatchNorm2d.num_batches_tracked) instead of a separate launch per layer.
    ``residual``: y[:, :Cr] += residual (identity shortcut, zero channel padding; no ReLU).
    ``tap``: return (y, x_alias); the gradient of x_alias is summed into dx by the BN kernel."""
    if _native(x):
        return _BatchNorm.apply(x, gamma, beta, running_mean, running_var, training, momentum, eps, relu,
                                num_batches if training else None, residual, tap)
    if num_batches is not None and training:
        num_batches.add_(1)
    y = F.batch_norm(x, running_mean, running_var, gamma, beta, training, momentum, eps)
    y = F.relu(y) if relu else y
    if residual is not None:
        y = y + F.pad(residual, (0, 0, 0, 0, 0, y.shape[1] - residual.shape[1]))
    return (y, x) if tap else y


# ------------------------------------------------- BN folded into the next 3x3 convolution
# PyramidNet's blocks run bn1 -> conv1 and bn2 -> ReLU -> conv2 (pytorch/model.py:40-50).  When
# the convolution takes the Winograd path, the BN's normalise pass is not run at all: the BN
# launches only its statistics (and writes a per-channel (scale, shift) table), the convolution's
# forward and weight-gradient kernels apply relu?(x * scale + shift) while staging their input
# tiles, and the BN backward recomputes its ReLU mask from x.  The BN output tensor is never
# written or read: one full pass over the activation (write + re-read) less per folded BN.
# Measured (docs/ROUND6.md, profiles/r6_bnfold/): the BN kernels save ~0.26 ms per PyramidNet
# step but the convolutions' staging, which now does the affine per window element (4x
# redundant over the overlapping 4x4 windows), costs more -- off by default (MXDDP_BN_FOLD=1).
_BN_FOLD = os.environ.get("MXDDP_BN_FOLD", "0") != "0"


def set_bn_fold(on: bool) -> None:
    global _BN_FOLD
    _BN_FOLD = bool(on)


class _BatchNormFold(torch.autograd.Function):
    """Training BN whose normalise pass the consuming convolution performs (``bn_conv``).  Returns
    (h, ss[, x_alias]): h aliases x and stands for the BN output (its gradient, from the
    convolution, is the gradient of that output), ss = [C, 2] (scale, shift); ``tap`` as in
    ``_BatchNorm``."""

    @staticmethod
    def forward(ctx, x, gamma, beta, running_mean, running_var, momentum, eps, relu, num_batches=None, tap=False):
        C = native()
        x = x.contiguous()
        _check(x, "input")
        N, Cc = x.shape[0], x.shape[1]
        HW = x.numel() // (N * Cc)
        mean = torch.empty((Cc,), device=x.device, dtype=torch.float32)
        invstd = torch.empty_like(mean)
        ss = torch.empty((Cc, 2), device=x.device, dtype=torch.float32)
        part = _bn_part(x.device, C.bn_partial_floats(N, Cc, HW))
        C.bn_fwd_train(x.data_ptr(), _p(gamma), _p(beta), 0, mean.data_ptr(), invstd.data_ptr(), _p(running_mean),
                       _p(running_var), N, Cc, HW, float(momentum), float(eps), bool(relu), part.data_ptr(),
                       stream_of(x), _p(num_batches), 0, 0, ss.data_ptr())
        ctx.save_for_backward(x, gamma, mean, invstd, ss)
        ctx.dims = (N, Cc, HW)
        ctx.relu = bool(relu)
        ctx.has_affine = gamma is not None
        ctx.affine_refs = (gamma, beta)
        ctx.mark_non_differentiable(ss)
        if tap:
            return x, ss, x
        return x, ss

    @staticmethod
    def backward(ctx, dh, _dss, dtap=None):
        x, gamma, mean, invstd, ss = ctx.saved_tensors
        N, Cc, HW = ctx.dims
        dh = dh.contiguous()
        dx = torch.empty_like(x)
        g_ref, b_ref = ctx.affine_refs
        gs, bs = (_grad_sink(g_ref), _grad_sink(b_ref)) if ctx.has_affine else (None, None)
        direct = gs is not None and bs is not None
        if direct:
            dg, db = gs, bs
        else:
            dg = torch.empty((Cc,), device=x.device) if ctx.has_affine else None
            db = torch.empty((Cc,), device=x.device) if ctx.has_affine else None
        ext, ext_c = None, 0
        if dtap is not None:  # the shortcut branch's gradient, read in place when it can be
            s_ = dtap.stride()
            W = x.shape[-1] if x.dim() >= 3 else 1
            in_place = (dtap.dim() == 4 and s_[3] == 1 and s_[2] == W and s_[1] == HW and s_[0] % HW == 0
                        and s_[0] // HW >= Cc and dtap.dtype == torch.float32)
            ext = dtap if in_place else dtap.contiguous()
            ext_c = s_[0] // HW if in_place else Cc
        part = _bn_part(x.device, native().bn_partial_floats(N, Cc, HW))
        native().bn_bwd(dh.data_ptr(), x.data_ptr(), 0, _p(gamma), mean.data_ptr(), invstd.data_ptr(), dx.data_ptr(),
                        _p(dg), _p(db), N, Cc, HW, direct, part.data_ptr(), stream_of(dh), _p(ext), ext_c,
                        ss.data_ptr() if ctx.relu else 0)
        if direct:
            _grad_done(g_ref)
            _grad_done(b_ref)
            dg = db = None
        return dx, dg, db, None, None, None, None, None, None, None


def _fold_ok(x, bn, conv) -> bool:
    if not (_BN_FOLD and _native(x) and x.dim() == 4 and bn.training and bn.track_running_stats
            and bn.running_mean is not None and conv.bias is None and not getattr(conv, "fuse_relu", False)
            and conv.groups == 1 and conv.weight.dtype == torch.float32):
        return False
    N, Cin, H, W = x.shape
    K, _, R, S = conv.weight.shape
    (sh, sw), (ph, pw), (dh, dw) = _pair(conv.stride), _pair(conv.padding), _pair(conv.dilation)
    # the Winograd path (its forward and weight gradient both stage the input through registers)
    return native().conv_fwd_filter_floats(N, Cin, H, W, K, R, S, sh, sw, ph, pw, dh, dw) > 0


def bn_conv(x, bn, conv, tap=False):
    """``conv(bn(x))`` (``bn``: an mxddp BatchNorm2d, ReLU fused or not; ``conv``: its Conv2d),
    with the BN's normalise pass folded into the convolution where it runs the Winograd path in
    training; the plain two-op chain otherwise.  ``tap`` as in ``batch_norm``: also return an
    alias of x for the shortcut branch."""
    if not _fold_ok(x, bn, conv):
        h = bn(x, tap=tap)
        if tap:
            h, xs = h
            return conv(h), xs
        return conv(h)
    mom = bn.momentum if bn.momentum is not None else 0.1
    out = _BatchNormFold.apply(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, mom, bn.eps, bn.fuse_relu,
                               bn.num_batches_tracked, tap)
    h, ss = out[0], out[1]
    y = conv2d(h, conv.weight, None, conv.stride, conv.padding, conv.dilation, in_ss=ss, in_relu=bn.fuse_relu)
    return (y, out[2]) if tap else y


# --------------------------------------------------------------------------- loss
class _CrossEntropy(torch.autograd.Function):
    """Fused log_softmax + NLL (mean).  Forward computes loss AND dlogits in one kernel."""

    @staticmethod
    def forward(ctx, logits, target):
        C = native()
        logits = logits.contiguous()
        _check(logits, "logits")
        B, K = logits.shape
        # int32 targets are used as they are (no cast launch); the kernel sums loss / B, so the
        # mean needs no division launch
        tgt = (target if target.dtype == torch.int32 else target.to(torch.int32)).contiguous()
        acc = torch.zeros(2, device=logits.device, dtype=torch.float32)
        dl = torch.empty_like(logits)
        C.xent_fwd_bwd(logits.data_ptr(), tgt.data_ptr(), 0, dl.data_ptr(), acc.data_ptr(), acc.data_ptr() + 4,
                       B, K, 1.0 / B, stream_of(logits), 1.0 / B)
        ctx.save_for_backward(dl)
        correct = acc[1]
        # the correct count must carry no autograd history: a caller accumulating it across steps
        # (corr_acc.add_(corr)) would otherwise chain every step's graph to the next and keep the
        # parameters' grad accumulators of the FIRST step alive -- with the stream they were
        # created on, so a later hipGraph capture ran the DDP hooks (and their bucket all-reduce)
        # outside the capture (ranks then trained on un-reduced gradients)
        ctx.mark_non_differentiable(correct)
        ctx.set_materialize_grads(False)
        return acc[0], correct

    @staticmethod
    def backward(ctx, dloss, _dcorrect):
        if dloss is None:
            return None, None
        (dl,) = ctx.saved_tensors
        return dl * dloss, None


def cross_entropy(logits, target, return_correct=False):
    """Mean cross-entropy = NLL(log_softmax(logits)); optionally also #correct (on device)."""
    if _native(logits):
        loss, correct = _CrossEntropy.apply(logits, target)
    else:
        loss = F.cross_entropy(logits, target)
        correct = (logits.argmax(1) == target).sum().to(torch.float32)
    return (loss, correct) if return_correct else loss


# --------------------------------------------------------------------------- PyramidNet shortcut
class _ShortcutAdd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, out, x, stride):
        out = out.contiguous()
        x = x.contiguous()
        N, Cin, H, W = x.shape
        _, Cout, P, Q = out.shape
        # in place: `out` (the block's last BN output) has no other consumer and BN's backward
        # does not read its own output, so the residual add needs no copy
        native().shortcut_pad_add(x.data_ptr(), out.data_ptr(), N, Cin, H, W, Cout, P, Q, stride, stream_of(x))
        ctx.mark_dirty(out)
        ctx.dims = (N, Cin, H, W, Cout, P, Q, stride)
        return out

    @staticmethod
    def backward(ctx, dy):
        N, Cin, H, W, Cout, P, Q, stride = ctx.dims
        dy = dy.contiguous()
        dx = torch.empty((N, Cin, H, W), device=dy.device, dtype=dy.dtype)
        native().shortcut_pad_add_bwd(dy.data_ptr(), dx.data_ptr(), N, Cin, H, W, Cout, P, Q, stride, False,
                                      stream_of(dy))
        return dy, dx, None


def shortcut_pad_add(out, x, stride):
    """out + AvgPool2d(2,2,ceil)(F.pad(x, channels -> out.C)) (pytorch/model.py:17-21,49)."""
    if _native(out):
        if out.is_leaf and out.requires_grad:  # the in-place add needs a non-leaf (or grad-free) tensor
            out = out.clone()
        return _ShortcutAdd.apply(out, x, stride)
    sc = F.pad(x, (0, 0, 0, 0, 0, out.shape[1] - x.shape[1]))
    if stride == 2:
        sc = F.avg_pool2d(sc, 2, 2, ceil_mode=True)
    return out + sc


# --------------------------------------------------------------------------- precision
def set_compute_dtype(dtype: str) -> None:
    """GEMM-shaped ops (conv / linear) compute in ``fp32`` (exact fp32 MFMA, default) or
    ``bf16`` (bf16 operands rounded while staged into LDS, fp32 accumulation, fp32 tensors and
    master weights) -- the mixed-precision path of BASELINE config 5 (ResNet-50 bf16)."""
    p = {"fp32": 0, "float32": 0, "bf16": 1, "bfloat16": 1}[dtype]
    native().set_gemm_precision(p)


def compute_dtype() -> str:
    return "bf16" if native().gemm_precision() == 1 else "fp32"
