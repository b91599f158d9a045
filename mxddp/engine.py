"""Python face of the native fused MNIST-CNN DDP training step (``mxddp._C.MnistEngine``).

One ``FusedMnistTrainer.step()`` = one hipGraph launch that runs: Philox synthetic batch
(or a caller-provided batch) -> fused forward -> fused backward -> bucketed RCCL
all-reduce on a side stream (2 buckets, overlapped with the conv backward) -> flat SGD
with momentum / weight decay / 1/world_size folded in.  Loss and accuracy accumulate on
device and are read only at log intervals (fixes the two host syncs per step of
pytorch/distributed_data_parallel.py:135-138).

The parameters are one flat fp32 buffer in MnistCNN ``state_dict`` order, so
``state_dict()`` is key-for-key the reference-style checkpoint of ``models.MnistCNN``.
"""
from __future__ import annotations

import os

import torch

from . import native
from .fused import FusedTrainerBase
from .models.mnist_cnn import MnistCNN

_LAYOUT = [  # (name, shape) in state_dict order == flat offsets of MnistLayout (mnist_engine.h)
    ("conv1.weight", (32, 1, 3, 3)), ("conv1.bias", (32,)),
    ("conv2.weight", (64, 32, 3, 3)), ("conv2.bias", (64,)),
    ("fc1.weight", (128, 9216)), ("fc1.bias", (128,)),
    ("fc2.weight", (10, 128)), ("fc2.bias", (10,)),
]


class FusedMnistTrainer(FusedTrainerBase):
    LAYOUT = _LAYOUT
    MODEL = MnistCNN

    def __init__(self, batch: int = 64, device: torch.device | int = 0, comm=None, seed: int = 1, lr: float = 0.1,
                 momentum: float = 0.9, weight_decay: float = 1e-4, variant: int = 1, use_graph: bool = True,
                 init_model: MnistCNN | None = None, graph_mode: int | None = None,
                 steps_per_graph: int | None = None, force_collectives: bool = False, transport: str = "auto",
                 peer=None, rccl_variants=None):
        C = native()
        self.C = C
        n = self._init_flat(batch, device, comm, seed, init_model)
        assert n == C.MNIST_NUM_PARAMS
        self.mom = torch.zeros(n, device=self.device)
        self.lr = torch.full((1,), lr, device=self.device)
        self._lr_host = lr
        wsb = C.mnist_workspace_bytes(batch)
        self.workspace = torch.empty(wsb // 4 + 64, dtype=torch.float32, device=self.device)
        if os.environ.get("MXDDP_POISON_WORKSPACE"):  # debug: NaN-fill to catch reads before writes
            self.workspace.fill_(float("nan"))
        torch.cuda.synchronize(self.device)
        self.eng = C.MnistEngine(batch, self.params.data_ptr(), self.grads.data_ptr(), self.mom.data_ptr(),
                                 self.workspace.data_ptr(), wsb, comm, seed, momentum, weight_decay,
                                 self.lr.data_ptr(), self.metrics.data_ptr(), variant)
        self._init_runtime(comm, peer, transport, force_collectives, rccl_variants, use_graph, graph_mode,
                           steps_per_graph)

    def _default_mode(self) -> int:
        # MXDDP_GRAPH_MODE: 0 = eager launches, 1 = whole step(s) incl. RCCL collectives in one
        # graph, 2 = compute graphs with eager collectives in between.  Default (-1): the engine
        # picks 1 at world size 1, eager when real collectives run (see autotune()).
        if self.graph_mode is not None:
            return self.graph_mode
        return int(os.environ.get("MXDDP_GRAPH_MODE", "-1"))

    def _candidate_strategies(self, transport: str) -> list:
        return ["ovl", "inl", "one"] + (["co"] if transport == "peer" else [])

    def _set_buckets(self, strat: str):
        """ovl: fc bucket overlapped on the side stream; inl: both buckets in order; one: a
        single all-reduce of the whole gradient after the conv backward; co (peer transport): the
        fc bucket's exchange co-scheduled in the first blocks of the conv-backward launch."""
        co = strat == "co" and self.eng.set_coscheduled(True)
        if not co:
            self.eng.set_coscheduled(False)
        self.eng.set_merged(strat == "one")
        self.eng.set_overlap(strat == "ovl")
        self.bucket_strategy = "co" if co else ("inl" if strat == "co" else strat)

    def _opt_tensors(self) -> dict:
        return {"mom": self.mom}

    def _after_param_load(self):
        self.eng.repack()  # conv2 weights pre-packed in MFMA fragment order + accumulator resets

    def phase_profile(self, steps: int = 20) -> dict:
        """In-kernel phase timings of the fused step (MnistFused::trace, s_memrealtime at 100 MHz).
        Runs `steps` eager steps with every block of each fused kernel stamping its phase
        boundaries.  Returns per kernel: block start spread (us after the first block started;
        median / max), block duration (median / max) and the median time from block start to
        each phase mark."""
        names = ["F2_fwd", "F3_fc1", "F5_head_fc1bwd", "F6_wgrad", "F7_dgrad", "CO_exchange"]
        buf = torch.zeros(7 * 1024 * 8, dtype=torch.int32, device=self.device)
        self.eng.set_trace(buf.data_ptr())
        acc = {n: [] for n in names}
        try:
            for _ in range(steps):
                with torch.cuda.stream(self.stream):  # the engine's stream, not torch's current one
                    buf.zero_()
                self.eng.step()
                self.eng.sync()
                t = buf.view(7, 1024, 8).cpu().to(torch.int64) & 0xFFFFFFFF
                # one time base for the conv-backward launch (F6 / F7 blocks and the co-scheduled
                # exchange blocks share it): [first start, median end, last end] per block kind
                t67 = t[3:6]
                live67 = t67[:, :, 0] != 0
                if live67[2].any():
                    o = t67[:, :, 0][live67].min()
                    win = {}
                    for k, n in ((3, "F6_wgrad"), (4, "F7_dgrad"), (5, "CO_exchange")):
                        lv = t[k, :, 0] != 0
                        if lv.any():
                            end = t[k][lv].max(dim=1).values
                            win[n] = [round((t[k, :, 0][lv].min() - o).item() * 0.01, 2),
                                      round((end.double().median() - o).item() * 0.01, 2),
                                      round((end.max() - o).item() * 0.01, 2)]
                    acc.setdefault("_f67_window", []).append(win)
                for k, n in enumerate(names):
                    t0 = t[k, :, 0]
                    live = t0 != 0
                    if not live.any():
                        continue
                    t0 = t0[live]
                    tk = t[k][live]
                    last = tk.max(dim=1).values
                    rec = {"start_med": (t0 - t0.min()).double().median().item() * 0.01,
                           "start_max": (t0 - t0.min()).max().item() * 0.01,
                           "dur_med": (last - t0).double().median().item() * 0.01,
                           "dur_max": (last - t0).max().item() * 0.01,
                           "kernel": (last.max() - t0.min()).item() * 0.01}
                    rec["phases"] = [((tk[:, ph] - t0)[tk[:, ph] != 0]).double().median().item() * 0.01
                                     for ph in range(1, 8) if (tk[:, ph] != 0).any()]
                    # the 4 slowest blocks: (block, start, phase marks) in us after the kernel's first start
                    ids = torch.nonzero(live).flatten()
                    t00 = t0.min()
                    rec["slowest"] = [(int(ids[i]), [round((int(v) - int(t00)) * 0.01, 2) for v in tk[i] if v != 0])
                                      for i in torch.argsort(last, descending=True)[:4].tolist()]
                    acc[n].append(rec)
        finally:
            self.eng.set_trace(0)
        out = {}
        wins = acc.pop("_f67_window", [])[1:]
        if wins:  # [start, median end, last end] us after the conv-backward launch's first block
            out["F67_launch_window"] = {n: [round(sum(w[n][i] for w in wins) / len(wins), 2) for i in range(3)]
                                        for n in wins[0] if all(n in w for w in wins)}
        for n, runs in acc.items():
            runs = runs[1:]  # drop the first (cold) step
            if not runs:
                continue
            avg = {k: round(sum(r[k] for r in runs) / len(runs), 2) for k in runs[0] if k not in ("phases", "slowest")}
            avg["slowest_last_step"] = runs[-1]["slowest"]
            m = min(len(r["phases"]) for r in runs)
            avg["phases"] = [round(sum(r["phases"][i] for r in runs) / len(runs), 2) for i in range(m)]
            out[n] = avg
        return out
