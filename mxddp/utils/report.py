"""Chainer trainer-extension equivalents (chainer/train_mnist.py:85-115) and Keras ``model.summary()``
(tensorflow2/mnist_single.py:28).

* ``LogReport``  -- the JSON list ``<out>/log`` Chainer's LogReport writes after every epoch
  (keys ``epoch``, ``iteration``, ``main/loss``, ``main/accuracy``, ``validation/main/loss``,
  ``validation/main/accuracy``, ``elapsed_time``);
* ``PrintReport`` -- the fixed-width table Chainer prints (columns of chainer/train_mnist.py:113-115);
* ``dump_graph`` -- ``<out>/cg.dot``, the Graphviz computational graph of the loss
  (``extensions.dump_graph('main/loss')``, chainer/train_mnist.py:89), built by walking the
  autograd graph of the first iteration's loss;
* ``model_summary`` -- Keras-style layer / output shape / parameter table.

ChainerMN registers the reporting extensions on rank 0 only (chainer/train_mnist_multi.py:108-113);
callers pass ``enabled=is_main``.
"""
from __future__ import annotations

import json
import os

import torch
import torch.nn as nn

PRINT_COLUMNS = ["epoch", "main/loss", "validation/main/loss", "main/accuracy", "validation/main/accuracy",
                 "elapsed_time"]


class LogReport:
    def __init__(self, out: str, enabled: bool = True, filename: str = "log"):
        self.path = os.path.join(out, filename)
        self.enabled = enabled
        self.log: list[dict] = []
        if enabled:
            os.makedirs(out, exist_ok=True)

    def append(self, entry: dict):
        self.log.append(entry)
        if not self.enabled:
            return
        tmp = self.path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(self.log, f, indent=4)
        os.replace(tmp, self.path)


class PrintReport:
    def __init__(self, columns=PRINT_COLUMNS, enabled: bool = True, out=print):
        self.columns = list(columns)
        self.enabled = enabled
        self._out = out
        self._header_done = False
        self._widths = [max(10, len(c)) for c in self.columns]

    def header(self) -> str:
        return "".join(c.ljust(w + 2) for c, w in zip(self.columns, self._widths)).rstrip()

    def row(self, entry: dict) -> str:
        cells = []
        for c, w in zip(self.columns, self._widths):
            v = entry.get(c)
            if v is None:
                s = ""
            elif isinstance(v, float):
                s = f"{v:<{w}g}"[:w]
            else:
                s = str(v)
            cells.append(s.ljust(w + 2))
        return "".join(cells).rstrip()

    def __call__(self, entry: dict):
        if not self.enabled:
            return
        if not self._header_done:
            self._out(self.header())
            self._header_done = True
        self._out(self.row(entry))


def dump_graph(loss: torch.Tensor, path: str, params: dict | None = None) -> int:
    """Write the autograd graph that produced `loss` as Graphviz DOT (function nodes as boxes,
    parameters / inputs as ellipses, edges in data-flow direction).  Returns the node count."""
    names = {id(p): n for n, p in (params or {}).items()}
    nodes, edges, seen = {}, [], set()
    keep = []  # grad_fn wrappers are created on access: hold them so their ids stay unique

    def nid(obj):
        return f"n{id(obj)}"

    def visit(fn):
        if fn is None or id(fn) in seen:
            return
        seen.add(id(fn))
        keep.append(fn)
        var = getattr(fn, "variable", None)
        if var is not None:  # AccumulateGrad: a leaf (parameter)
            label = names.get(id(var), "param") + "\\n" + "x".join(map(str, var.shape))
            nodes[nid(fn)] = f'{nid(fn)} [label="{label}", shape="ellipse"];'
        else:
            nodes[nid(fn)] = f'{nid(fn)} [label="{type(fn).__name__}", shape="box"];'
        for nxt, _ in getattr(fn, "next_functions", ()):
            if nxt is None:
                continue
            keep.append(nxt)
            visit(nxt)
            edges.append(f"{nid(nxt)} -> {nid(fn)};")

    visit(loss.grad_fn)
    out = [f'n_loss [label="main/loss\\n{tuple(loss.shape)}", shape="ellipse", style="filled"];']
    if loss.grad_fn is not None:
        edges.append(f"{nid(loss.grad_fn)} -> n_loss;")
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(path, "w") as f:
        f.write("digraph graphname{rankdir=TB;\n")
        f.write("\n".join(list(nodes.values()) + out + edges))
        f.write("\n}\n")
    return len(nodes) + 1


@torch.no_grad()
def model_summary(model: nn.Module, input_shape, name: str | None = None) -> str:
    """Keras ``Model.summary()``-style table: one row per leaf module with its output shape
    (batch dimension shown as None) and parameter count, plus totals."""
    rows, hooks = [], []
    leaves = [(n, m) for n, m in model.named_modules() if n and not list(m.children())]

    def hook(n, m):
        def f(_mod, _inp, out):
            shape = tuple(out.shape) if torch.is_tensor(out) else ()
            rows.append((f"{n} ({type(m).__name__})", ("None",) + tuple(map(str, shape[1:])),
                         sum(p.numel() for p in m.parameters(recurse=False))))
        return f

    for n, m in leaves:
        hooks.append(m.register_forward_hook(hook(n, m)))
    was_training = model.training
    model.eval()
    try:
        dev = next(model.parameters()).device
        model(torch.zeros((1,) + tuple(input_shape), device=dev))
    finally:
        for h in hooks:
            h.remove()
        model.train(was_training)
    total = sum(p.numel() for p in model.parameters())
    trainable = sum(p.numel() for p in model.parameters() if p.requires_grad)
    w = (34, 26, 10)
    line = "_" * sum(w)
    out = [f'Model: "{name or type(model).__name__}"', line,
           "Layer (type)".ljust(w[0]) + "Output Shape".ljust(w[1]) + "Param #", "=" * sum(w)]
    for layer, shape, n in rows:
        out.append(layer.ljust(w[0]) + ("(" + ", ".join(shape) + ")").ljust(w[1]) + str(n))
    out += ["=" * sum(w), f"Total params: {total:,}", f"Trainable params: {trainable:,}",
            f"Non-trainable params: {total - trainable:,}", line]
    return "\n".join(out)
