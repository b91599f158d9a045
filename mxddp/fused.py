"""Shared Python face of the native fused training engines (``mxddp._C.MnistEngine``,
``KerasEngine``, ``MlpEngine``).

Each engine runs a model's whole training step -- on-device synthetic batch (or a caller's
batch), fused forward / backward kernels, the gradient all-reduce when ranks or replicas exist,
the optimizer -- from C++ on one stream, captured into hipGraphs.  What is the same for all of
them lives here:

* flat fp32 parameters in the model's ``state_dict`` order (checkpoints are key-for-key the
  layer model's), DDP-constructor semantics (rank 0's weights broadcast);
* the gradient transport at world size > 1: RCCL (in xGMI-sized communicator variants) or the
  direct xGMI peer all-reduce, validated against RCCL before use;
* ``autotune()``: times every (transport x bucket strategy x eager / graph) candidate on a few
  real steps on THIS machine, the slowest rank deciding, and keeps the fastest
  (reference hot loop: pytorch/distributed_data_parallel.py:123-148);
* device-side metrics read only at log points, the data-stream position for resume, snapshots
  for scratch trials.

Subclasses set ``LAYOUT`` / ``MODEL`` and build ``self.eng``; optimizer state tensors are listed
by ``_opt_tensors()``.
"""
from __future__ import annotations

import os
import sys
import time

import torch

from . import native


def _numel(shape) -> int:
    k = 1
    for s in shape:
        k *= s
    return k


class FusedTrainerBase:
    LAYOUT: list = []       # (name, shape) in state_dict order == the engine's flat offsets
    MODEL: type = None      # layer model with the same state_dict
    STRATEGIES = ("ovl", "inl", "one")  # bucket strategies the engine supports (see _set_buckets)
    IMAGE = (1, 28, 28)

    # --------------------------------------------------------------- construction
    def _init_flat(self, batch, device, comm, seed, init_model, slack: int = 1024):
        self.device = torch.device("cuda", device) if isinstance(device, int) else device
        self.batch = batch
        self.comm = comm
        if init_model is None:
            torch.manual_seed(seed)
            init_model = self.MODEL()
        sd = init_model.state_dict()
        flat = torch.cat([sd[k].detach().reshape(-1).float().cpu() for k, _ in self.LAYOUT])
        n = flat.numel()
        self.params = flat.to(self.device)
        # + zeroed slack: the all-reduce of the bucket that ends at the end of the gradient is
        # padded to a multiple of world_size x channels x 16 B (Reducer::set_padding)
        self._grad_slack = slack
        self._grad_store = torch.zeros(n + slack, device=self.device)
        self.grads = self._grad_store[:n]
        self.metrics = torch.zeros(4, device=self.device)
        torch.cuda.synchronize(self.device)
        if comm is not None and comm.world_size > 1:  # DDP ctor semantics: rank 0's weights everywhere
            C = native()
            comm.broadcast(self.params.data_ptr(), self.params.data_ptr(), n, C.DType.f32, 0,
                           torch.cuda.current_stream(self.device).cuda_stream)
            torch.cuda.synchronize(self.device)
        return n

    def _init_runtime(self, comm, peer, transport, force_collectives, rccl_variants, use_graph, graph_mode,
                      steps_per_graph):
        """After self.eng exists: stream, counters, transport choice."""
        self.use_graph = use_graph
        self.graph_mode = graph_mode
        self.steps_per_graph = steps_per_graph
        self._external = False
        self._capture_done = False
        self.tuned = None
        self.bucket_strategy = "ovl"
        self.eng_comm = comm
        if force_collectives:
            self.eng.set_force_collectives(True)
        self.rccl_variants = rccl_variants  # [(name, Comm)] timed by autotune(); None = comm.py's list
        self.stream = torch.cuda.ExternalStream(self.eng.stream, device=self.device)
        self.steps = 0
        self.steps_at_reset = 0  # self.steps when the device metrics were last zeroed
        self.world_size = comm.world_size if comm is not None else (peer.world_size if peer is not None else 1)
        self._set_padding(comm)
        # gradient transport (world size > 1): RCCL, or the direct xGMI peer all-reduce
        # (parallel/peer.py) -- validated against RCCL on every rank before it may be used;
        # "auto" lets autotune() time both
        self.transport = transport
        self.peer = None
        if peer is not None:  # caller-provided peer transport (peer-only job: no RCCL communicator)
            self.peer, self.transport = peer, "peer"
            self.eng.set_peer(peer)
        elif self.world_size > 1 and transport in ("auto", "peer"):
            from .parallel import peer as _peer

            pc = _peer.peer_comm()
            if pc is not None and _peer.validate(pc, comm):
                self.peer = pc
            elif transport == "peer":
                raise RuntimeError("peer transport requested but unavailable / failed validation")
        if self.peer is not None and transport == "peer":
            self.eng.set_peer(self.peer)

    # --------------------------------------------------------------- stepping
    def step(self, n: int = 1):
        """Run n training steps (graph replays once captured; first call warms up + captures)."""
        if n <= 0:
            return
        if self.use_graph and not self._capture_done:
            self.eng.step()          # warm-up: lazy RCCL/kernel init outside the capture
            self.eng.sync()
            self._capture(self._default_mode())
            n -= 1
            self.steps += 1
        if n > 0:
            self.eng.replay(n)
            self.steps += n

    def compute_only_ms(self, steps: int) -> float | None:
        """Device ms per step of this rank's step with every bucket collective removed (the
        Reducer keeps its fences and joins: ``set_dry_collectives``), launched the way the
        timed steps were (the same graph mode, recaptured without the collectives).  The bench
        reports ``exposed comm = timed step - this``.  The replicas' weights diverge during the
        pass (each applies its local gradient), so it runs only after the measurement; the
        original launch mode is recaptured afterwards.  None when the step has no collective.
        The co-scheduled exchange (strategy "co") runs inside a compute kernel and stays."""
        if not self.eng.reducer_active or steps <= 0:
            return None
        C = native()
        mode = self.eng.graph_mode if self._capture_done else None
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        C.set_dry_collectives(True)
        ran = 2 + steps
        try:
            self.eng.uncapture()
            if mode:
                self._capture(mode)
                ran += self.eng.warm_graphs()
            self.eng.replay(2)
            self.eng.sync()
            ev0.record(self.stream)
            self.eng.replay(steps)
            ev1.record(self.stream)
            self.eng.sync()
        finally:
            self.discarded_steps = getattr(self, "discarded_steps", 0) + ran
            C.set_dry_collectives(False)
            self.eng.uncapture()
            if mode:
                self._capture(mode)
        return ev0.elapsed_time(ev1) / steps

    def warm_graphs(self) -> int:
        """Launch every captured multi-step graph once (untimed warm-up; they are real training
        steps, counted in self.steps): a replay whose step count needs a graph never launched
        before would otherwise pay that graph's first-launch cost.  Returns the steps run."""
        if self.use_graph and not self._capture_done:
            self.step(1)
        n = self.eng.warm_graphs()
        self.steps += n
        return n

    def _default_mode(self) -> int:
        # 0 = eager launches, 1 = whole step(s) incl. collectives in one graph.  Default: 1 at
        # world size 1, eager when real collectives run until autotune() picks (env override
        # MXDDP_GRAPH_MODE)
        if self.graph_mode is not None:
            return self.graph_mode
        env = int(os.environ.get("MXDDP_GRAPH_MODE", "-1"))
        if env >= 0:
            return env
        return 0 if self.world_size > 1 else 1

    def _capture(self, mode: int, spg: int | None = None):
        if spg is None:
            spg = self.steps_per_graph
        if spg is None:
            spg = int(os.environ.get("MXDDP_STEPS_PER_GRAPH", "32"))
        if self._external:
            spg = 1  # a caller-provided batch is copied in before EVERY step
        self.eng.capture(mode, spg)
        self._capture_done = True

    # --------------------------------------------------------------- DDP launch strategy
    def _candidate_strategies(self, transport: str) -> list:
        return list(self.STRATEGIES)

    def autotune(self, trial_steps: int = 24, include_graphs: bool | None = None, restore: bool = True,
                 budget_s: float | None = None) -> dict:
        """Pick the fastest launch strategy for the DDP step on THIS machine by timing a few real
        training steps of each (they count as warm-up).  Candidates: gradient transport (RCCL in
        each configured communicator variant, or the direct xGMI peer all-reduce when it
        validated) x bucket strategy (``STRATEGIES``: "ovl" first bucket all-reduced on the side
        stream overlapping the rest of the backward, "inl" the buckets in order on the compute
        stream, "one" a single all-reduce of the whole gradient, "co" the exchange co-scheduled
        inside another launch of the step) x (eager launches, or the step captured in one
        hipGraph -- RCCL included, MXDDP_AUTOTUNE_GRAPHS=0 keeps RCCL eager: at 8 GPUs an eager
        step is ~7 host launches per ~70 us of device work, a graph is one).  The
        slowest rank's time decides, so every rank picks the same strategy.

        Fail fast, never raise for a peer candidate: before a peer-transport strategy is timed,
        two steps of it run from a snapshot with the 2 s validate timeout and are compared with
        the same two steps over RCCL (or over the standalone peer kernel when the job has no
        RCCL); a strategy that times out or disagrees on ANY rank is marked ``inf`` on every
        rank, the transport is re-synchronised (peer.resync) and the training state restored.  A
        standalone-kernel failure, or a failure while timing, drops the peer transport for the
        rest of the autotune.

        Trial steps are always scratch: validation and failed trials restart from the snapshot
        taken on entry, and the trainer is put back to that snapshot at the end, so the state
        after autotune does not depend on which candidates ran or validated.  Every trial step
        is counted in ``discarded_steps`` (``restore`` is kept for callers; it no longer changes
        anything).

        Wall-time cap: ``budget_s`` (default MXDDP_AUTOTUNE_BUDGET_S, else 90 s).  Before each
        candidate the slowest rank's elapsed autotune time is agreed on; once it is over the
        budget (and at least one candidate has a time) the remaining candidates are skipped on
        every rank and listed in ``tuned["skipped"]``.  Returns {candidate: ms/step}."""
        from .parallel import comm as pc

        if include_graphs is None:
            include_graphs = os.environ.get("MXDDP_AUTOTUNE_GRAPHS", "1") == "1"
        if not self.eng.reducer_active or self._external:
            return {}
        comms = self._rccl_candidates()
        rccl_names = [f"rccl:{v}" if len(comms) > 1 else "rccl" for v in comms]
        transports = rccl_names + (["peer"] if self.peer is not None else [])
        if self.transport == "peer" and self.peer is not None:
            transports = ["peer"]
        elif self.transport == "rccl":
            transports = rccl_names
        snap0 = self.snapshot()
        cands = []
        for tr in transports:
            strats = self._candidate_strategies(tr)
            cands += [(tr, 0, st) for st in strats]
            if self.use_graph and (include_graphs or tr == "peer"):
                cands += [(tr, 1, st) for st in strats]
        if budget_s is None:
            budget_s = float(os.environ.get("MXDDP_AUTOTUNE_BUDGET_S", "90"))
        t_start = time.perf_counter()
        skipped = []
        trial_run = 0  # trial steps run (all scratch: restored below)
        results = {}
        self._peer_ok = {}   # strategy -> agreed validation verdict (peer transport)
        self._peer_ref = None
        peer_dead = False
        if self.peer is not None:
            self.peer.set_timeout_ms(float(os.environ.get("MXDDP_PEER_VALIDATE_TIMEOUT_MS", "2000")))
        try:
            for tr, mode, strat in cands:
                key = (tr, mode, strat)
                if skipped or (any(v < float("inf") for v in results.values())
                               and pc.all_reduce_max(time.perf_counter() - t_start) > budget_s):
                    skipped.append(f"{tr}/{mode}/{strat}")  # every rank agreed on the same point
                    continue
                if tr == "peer":
                    if peer_dead:
                        results[key] = float("inf")
                        continue
                    if strat not in self._peer_ok:
                        self._peer_ok[strat] = self._validate_peer_strategy(strat, comms, rccl_names, snap0)
                        if not self._peer_ok[strat] and strat != "co":
                            peer_dead = True  # the standalone kernels themselves fail: no peer candidate can work
                    if not self._peer_ok[strat]:
                        results[key] = float("inf")
                        continue
                    self._peer_resync()
                self.eng.uncapture()
                self._use_transport(tr, comms)
                self._set_buckets(strat)
                failed = 0.0
                try:  # capture issues no collective, so a local failure here is safe to agree on
                    if mode:
                        self._capture(mode)
                except RuntimeError:
                    failed = 1.0
                # every rank reaches this all-reduce before any collective of the candidate, so a
                # candidate that failed to capture on ANY rank is skipped by ALL ranks together
                if pc.all_reduce_max(failed) > 0:
                    self.eng.uncapture()
                    results[key] = float("inf")
                    continue
                # HIP errors of a replay are not swallowed (peers may be inside the collectives);
                # a peer exchange that timed out is: its error word is agreed on below
                self.eng.replay(2)
                self.eng.sync()
                pc.barrier()
                t0 = time.perf_counter()
                self.eng.replay(trial_steps)
                self.eng.sync()
                dt = pc.all_reduce_max(time.perf_counter() - t0)
                self.steps += 2 + trial_steps
                trial_run += 2 + trial_steps
                bad = 1.0 if (tr == "peer" and self.peer.error()) else 0.0
                if pc.all_reduce_max(bad) > 0:
                    results[key] = float("inf")
                    peer_dead = True
                    self.eng.uncapture()
                    self._use_transport(rccl_names[0] if rccl_names else "peer", comms)
                    self._peer_resync()
                    self.restore(snap0)  # the failed trial's steps trained on garbage gradients
                    continue
                results[key] = dt / trial_steps * 1e3
        finally:
            if self.peer is not None:
                self.peer.set_timeout_ms(float(os.environ.get("MXDDP_PEER_TIMEOUT_MS", "30000")))
        best = min(results, key=results.get) if results else None
        if best is None or results[best] == float("inf"):
            raise RuntimeError(f"autotune: no launch strategy works on this machine ({results})")
        self.eng.uncapture()
        if best[0] == "peer":
            self._peer_resync()
        self._use_transport(best[0], comms)
        self._set_buckets(best[2])
        if best[1]:
            self._capture(best[1])
        self._capture_done = True
        self.restore(snap0)
        self.discarded_steps = getattr(self, "discarded_steps", 0) + trial_run
        self.tuned = {"transport": best[0], "graph_mode": best[1], "buckets": best[2],
                      "trials_ms": {f"{t}/{m}/{s}": round(v, 4) for (t, m, s), v in results.items()},
                      "wall_s": round(time.perf_counter() - t_start, 2), "budget_s": budget_s}
        if skipped:
            self.tuned["skipped"] = skipped
            if pc.info().rank == 0:
                print(f"mxddp autotune: {budget_s:.0f} s budget reached; {len(skipped)} candidate(s) not timed: "
                      + ", ".join(skipped), file=sys.stderr, flush=True)
        if self._peer_ok:
            self.tuned["peer_validated"] = dict(self._peer_ok)
        return results

    # ------------------------------------------------------------ candidate validation
    def _peer_resync(self):
        from .parallel import peer as _peer

        if self.peer is not None:
            _peer.resync(self.peer)

    def _state_delta(self, snap: dict) -> torch.Tensor:
        """What a step changed: parameters and the float optimizer state, minus the snapshot."""
        parts = [(self.params - snap["params"]).flatten()]
        for k, t in self._opt_tensors().items():
            if t.dtype == torch.float32 and t.numel() == self.params.numel():
                parts.append((t - snap["opt"][k]).flatten())
        return torch.cat(parts)

    def _run_from(self, snap: dict, steps: int = 2) -> torch.Tensor:
        """`steps` eager steps from `snap` with the current strategy; returns their state delta
        and puts the trainer back to `snap` (scratch steps, counted in discarded_steps)."""
        self.restore(snap)
        self.eng.replay(steps)
        self.eng.sync()
        d = self._state_delta(snap)
        self.restore(snap)
        self.discarded_steps = getattr(self, "discarded_steps", 0) + steps
        return d

    def _validate_peer_strategy(self, strat: str, comms: dict, rccl_names: list, snap0: dict) -> bool:
        """Collective: two steps of the peer transport with bucket strategy `strat` against the
        same two steps of the reference (RCCL's first variant with its first strategy, or the
        standalone peer kernel with the first strategy when the job has no RCCL).  The verdict is
        agreed over the ranks; a failed candidate leaves the transport re-synchronised."""
        from .parallel import comm as pc

        if self._peer_ref is None:
            ref_tr = rccl_names[0] if rccl_names else "peer"
            ref_strat = self._candidate_strategies(ref_tr)[0]
            self.eng.uncapture()
            if ref_tr == "peer":
                self._peer_resync()
            self._use_transport(ref_tr, comms)
            self._set_buckets(ref_strat)
            ref = self._run_from(snap0)
            ok = not (ref_tr == "peer" and self.peer.error())
            if pc.all_reduce_max(0.0 if ok else 1.0) > 0:
                self._peer_resync()
                if ref_tr == "peer":
                    self._peer_ok[ref_strat] = False
                    return False
                raise RuntimeError("autotune: the RCCL reference step failed")
            self._peer_ref = ref
            if ref_tr == "peer" and strat == ref_strat:
                return True
        self.eng.uncapture()
        self._peer_resync()
        self._use_transport("peer", comms)
        self._set_buckets(strat)
        d = self._run_from(snap0)
        err = self.peer.error()
        ok, why = not err, f"peer timeout (rank {err - 1} never arrived)" if err else ""
        if ok:
            ref = self._peer_ref
            rel = ((d - ref).norm() / ref.norm().clamp_min(1e-30)).item()
            ok = rel <= float(os.environ.get("MXDDP_VALIDATE_RTOL", "1e-3"))
            why = "" if ok else f"disagrees with the reference steps (relative {rel:.3g}; {self._where_differs(d, ref)})"
        if not ok:  # the driver's logs say why a candidate was dropped
            print(f"mxddp autotune: rank {pc.info().rank}: peer strategy {strat!r} rejected: {why}",
                  file=sys.stderr, flush=True)
        ok = pc.all_reduce_max(0.0 if ok else 1.0) == 0.0
        if not ok:
            self._peer_resync()
        return ok

    def _where_differs(self, d: torch.Tensor, ref: torch.Tensor) -> str:
        """Which part of the state delta a rejected candidate got wrong: the parameter tensors
        (LAYOUT names) whose delta differs from the reference, with the fraction of their
        elements that differ -- one bucket or a partial slice points at the exchange."""
        bad = ((d - ref).abs() > 1e-6 * ref.abs().max().clamp_min(1e-30)).cpu()
        out, off = [], 0
        for name, shape in getattr(self, "LAYOUT", ()):
            k = _numel(shape)
            frac = bad[off:off + k].float().mean().item() if k else 0.0
            if frac > 0:
                out.append(f"{name} {frac:.0%}")
            off += k
        if off < bad.numel() and bad[off:].any():
            out.append(f"optimizer state {bad[off:].float().mean().item():.0%}")
        return "differing: " + (", ".join(out) if out else "none")

    def _rccl_candidates(self) -> dict:
        """{variant name: Comm} the autotune times: the caller's list, else (world size > 1, or
        MXDDP_RCCL_VARIANTS set) comm.py's xGMI-sized variants over the same ranks, else just
        the trainer's own communicator."""
        if self.rccl_variants is not None:
            return dict(self.rccl_variants)
        if self.comm is None:
            return {}
        from .parallel import comm as pc

        if self.world_size > 1 or "MXDDP_RCCL_VARIANTS" in os.environ:
            out = {}
            for v in pc.rccl_variants():
                c, why = None, ""
                try:  # a variant RCCL refuses (config field, version) is dropped, not fatal
                    c = self.comm if v == "default" else pc.rccl_comm(force=True, variant=v)
                except Exception as e:  # noqa: BLE001 - any init failure
                    why = str(e).splitlines()[0] if str(e) else type(e).__name__
                # every rank must agree (a communicator some ranks lack cannot run collectives)
                if pc.all_reduce_max(0.0 if c is not None or v == "default" else 1.0) > 0:
                    if why:
                        print(f"mxddp autotune: RCCL variant {v!r} dropped: {why}", file=sys.stderr, flush=True)
                    continue
                if c is not None:
                    out[v] = c
            if out:
                return out
        return {"default": self.comm}

    def _set_padding(self, comm):
        ctas = 0
        if comm is not None:
            from .parallel import comm as pc

            ctas = pc.parse_variant(comm.variant)["ctas"]
        mult = max(1, self.world_size) * max(ctas, 32) * 4  # elements of 4 B: 16-B chunks per channel
        self.eng.set_bucket_padding(self.params.numel() + self._grad_slack, mult)

    def _use_transport(self, tr: str, comms: dict):
        if tr == "peer":
            self.eng.set_peer(self.peer)
            return
        self.eng.set_peer(None)
        name = tr.split(":", 1)[1] if ":" in tr else next(iter(comms), "default")
        c = comms.get(name, self.comm)
        if c is not None and c is not self.eng_comm:
            self.eng.set_comm(c)
            self.eng_comm = c
        self._set_padding(c)

    def _set_buckets(self, strat: str):
        """ovl: first bucket overlapped on the side stream; inl: the buckets in order; one: a
        single all-reduce of the whole gradient after the backward."""
        self.eng.set_merged(strat == "one")
        self.eng.set_overlap(strat == "ovl")
        self.bucket_strategy = strat

    def _check_peer(self):
        if self.peer is not None and self.peer.error():
            raise RuntimeError(f"peer all-reduce: rank {self.peer.error() - 1} never arrived (timeout)")

    @property
    def active_transport(self) -> str:
        if self.world_size == 1 and not self.eng.reducer_active:
            return "none"
        if self.eng.peer_active:
            return "peer"
        return "rccl" if self.eng_comm is None else f"rccl:{self.eng_comm.variant}"

    # --------------------------------------------------------------- data
    def set_batch(self, x: torch.Tensor, y: torch.Tensor):
        """Use a caller-provided batch (real MNIST) instead of the on-device generator.  The
        first call drops captured multi-step graphs: the batch is copied in before every step."""
        if not self._external:
            self.eng.set_external_batch(True)
            if self._capture_done and self.eng.captured:
                self.eng.uncapture()
                self._capture_done = False
            self._external = True
        # x / y were produced (and allocated) on the caller's stream: the engine stream waits for
        # that work before copying, and the caller's stream waits for the copy -- otherwise the
        # caller's next batch can reuse their memory before this step's copy has run
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            self._x_view().copy_(x.reshape(self._x_view().shape), non_blocking=True)
            self._y_view().copy_(y.to(torch.int32), non_blocking=True)
        cur.wait_stream(self.stream)

    def _view(self, ptr, count, dtype=torch.float32):
        off = (ptr - self.workspace.data_ptr()) // 4
        return self.workspace[off:off + count].view(dtype)

    def _x_view(self):
        d = _numel(self.IMAGE)
        return self._view(self.eng.x_ptr, self.batch * d).view(self.batch, *self.IMAGE)

    def _y_view(self):
        return self._view(self.eng.y_ptr, self.batch, torch.int32)

    def _counter_view(self):
        return self._view(self.eng.counter_ptr, 4, torch.int32)

    def data_state(self) -> torch.Tensor:
        """Position of the on-device synthetic data stream (Philox counter), for resume state."""
        self.eng.sync()
        return self._counter_view().cpu().clone()

    def load_data_state(self, ctr: torch.Tensor):
        self.eng.sync()
        self._counter_view().copy_(ctr.to(torch.int32).to(self.device))
        torch.cuda.synchronize(self.device)

    # --------------------------------------------------------------- metrics / lr
    def set_lr(self, lr: float):
        if lr != self._lr_host:
            with torch.cuda.stream(self.stream):
                self.lr.fill_(lr)
            self._lr_host = lr

    def synchronize(self):
        self.eng.sync()

    def read_metrics(self, reset: bool = True):
        """(loss_sum, correct) accumulated since the last reset (one host sync)."""
        self.eng.sync()
        if self.comm is not None:
            self.comm.check_async_error()  # surface a failed/aborted peer at log boundaries
        self._check_peer()
        m = self.metrics[:2].tolist()
        if reset:
            with torch.cuda.stream(self.stream):
                self.metrics.zero_()
            self.eng.sync()
            self.steps_at_reset = self.steps
        return m[0], m[1]

    # --------------------------------------------------------------- state
    def _opt_tensors(self) -> dict:
        """Optimizer state tensors on the device (snapshot / restore)."""
        return {}

    def _after_param_load(self):
        """Re-derive engine-side packed weights after the parameters changed outside the engine."""

    def snapshot(self) -> dict:
        """Device copies of everything a training step changes (weights, optimizer state,
        data-stream position, metric accumulators): restore() puts the trainer back exactly."""
        self.eng.sync()
        return {"params": self.params.clone(), "opt": {k: t.clone() for k, t in self._opt_tensors().items()},
                "ctr": self._counter_view().clone(), "metrics": self.metrics.clone(), "steps": self.steps,
                "steps_at_reset": self.steps_at_reset}

    def restore(self, snap: dict):
        self.eng.sync()
        opt = self._opt_tensors()
        with torch.cuda.stream(self.stream):
            self.params.copy_(snap["params"])
            for k, t in snap["opt"].items():
                opt[k].copy_(t)
            self._counter_view().copy_(snap["ctr"])
            self.metrics.copy_(snap["metrics"])
        self.eng.sync()
        self.steps, self.steps_at_reset = snap["steps"], snap["steps_at_reset"]
        self._after_param_load()
        self.eng.sync()

    def state_dict(self) -> dict:
        self.eng.sync()
        out, off = {}, 0
        for name, shape in self.LAYOUT:
            k = _numel(shape)
            out[name] = self.params[off:off + k].view(shape).detach().cpu().clone()
            off += k
        return out

    def load_state_dict(self, sd: dict):
        flat = torch.cat([sd[k].detach().reshape(-1).float().cpu() for k, _ in self.LAYOUT])
        self.eng.sync()
        self.params.copy_(flat.to(self.device))
        torch.cuda.synchronize(self.device)
        self._after_param_load()
        self.eng.sync()

    def to_module(self):
        m = self.MODEL()
        m.load_state_dict(self.state_dict())
        return m


class AdamTrainerBase(FusedTrainerBase):
    """Fused engines trained with the reference's Adam (Keras / Chainer epsilon-hat form): flat
    m / v and the step count on the device ({completed steps, step being applied})."""

    def _init_adam(self, n: int, lr: float):
        self.m = torch.zeros(n, device=self.device)
        self.v = torch.zeros(n, device=self.device)
        self.adam_state = torch.zeros(2, dtype=torch.int32, device=self.device)
        self.lr = torch.full((1,), lr, device=self.device)
        self._lr_host = lr

    def _opt_tensors(self) -> dict:
        return {"m": self.m, "v": self.v, "adam_state": self.adam_state, "lr": self.lr}

    @property
    def adam_steps(self) -> int:
        # [0] committed by the next forward, [1] written by the last update
        self.eng.sync()
        return int(self.adam_state.max().item())

    def optimizer_state(self) -> dict:
        self.eng.sync()
        return {"lr": self._lr_host, "m": self.m.cpu(), "v": self.v.cpu(), "steps": int(self.adam_state.max().item())}

    def load_optimizer_state(self, st: dict):
        self.eng.sync()
        self.m.copy_(st["m"].to(self.device))
        self.v.copy_(st["v"].to(self.device))
        self.adam_state.fill_(int(st["steps"]))
        self.set_lr(float(st["lr"]))
        torch.cuda.synchronize(self.device)


class FusedReplicas:
    """In-process replica data parallelism on a fused engine (MirroredStrategy /
    DataParallel / Chainer ParallelUpdater semantics): ONE process drives one trainer per device,
    the global batch = replicas x per-replica batch, gradients averaged every step by the peer
    transport opened in-process (device peer access over xGMI, no IPC), so every replica's whole
    step -- forward, backward, all-reduce, optimizer -- is one graph launch on its own stream
    and the replicas synchronise on the GPUs.  Every replica's work is launched before the host
    waits on any of them.  ``make(device, peer)`` builds one replica's trainer."""

    def __init__(self, devices, make, blocks: int = 32, peer_bytes: int = 8 << 20):
        C = native()
        self.devices = [torch.device(d) for d in devices]
        n = len(self.devices)
        self.peers = [None] * n
        if n > 1:
            self.peers = []
            for i, d in enumerate(self.devices):
                with torch.cuda.device(d):
                    self.peers.append(C.PeerComm(i, n, d.index, peer_bytes, blocks))
            for pc, d in zip(self.peers, self.devices):
                with torch.cuda.device(d):
                    pc.open_local(self.peers)
        self.trainers = []
        for pc, d in zip(self.peers, self.devices):
            with torch.cuda.device(d):
                self.trainers.append(make(d, pc))
        self._captured = False

    def _each(self, fn):
        for t, d in zip(self.trainers, self.devices):
            with torch.cuda.device(d):
                fn(t)

    def step(self, n: int = 1):
        if n <= 0:
            return
        t0 = self.trainers[0]
        if t0.use_graph and not self._captured:
            self._each(lambda t: t.eng.step())  # every replica launched before any host wait
            self._each(lambda t: t.eng.sync())
            self._each(lambda t: t._capture(1))
            self._each(lambda t: setattr(t, "steps", t.steps + 1))
            self._captured = True
            n -= 1
        if n > 0:
            self._each(lambda t: t.eng.replay(n))
            self._each(lambda t: setattr(t, "steps", t.steps + n))

    def timed_steps(self, n: int) -> float:
        """Run n steps; returns the slowest replica's DEVICE time of them in seconds.  Every
        replica first runs one tiny peer all-reduce on its own stream, so the replicas' start
        events fire together however far apart the host launched them (bench.py)."""
        C = native()
        self.synchronize()
        evs = []
        for t, d, pc in zip(self.trainers, self.devices, self.peers):
            with torch.cuda.device(d):
                if pc is not None:
                    buf = torch.zeros(64, device=d)
                    t.stream.wait_stream(torch.cuda.current_stream(d))
                    pc.all_reduce(buf.data_ptr(), buf.numel(), C.DType.f32, t.eng.stream, C.RedOp.sum)
                    buf.record_stream(t.stream)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(t.stream)
                evs.append((e0, e1))
        self.step(n)
        for t, d, (_, e1) in zip(self.trainers, self.devices, evs):
            with torch.cuda.device(d):
                e1.record(t.stream)
        self.synchronize()
        return max(e0.elapsed_time(e1) for e0, e1 in evs) * 1e-3

    def set_batch(self, x: torch.Tensor, y: torch.Tensor):
        xs, ys = x.chunk(len(self.trainers)), y.chunk(len(self.trainers))
        for t, d, xi, yi in zip(self.trainers, self.devices, xs, ys):
            with torch.cuda.device(d):
                if not t._external:
                    self._captured = False
                t.set_batch(xi.to(d, non_blocking=True), yi.to(d, non_blocking=True))

    def synchronize(self):
        self._each(lambda t: t.eng.sync())
        for pc in self.peers:
            if pc is not None and pc.error():
                raise RuntimeError(f"replica all-reduce: replica {pc.error() - 1} never arrived (timeout)")

    def read_metrics(self):
        self.synchronize()
        ls = cs = 0.0
        for t, d in zip(self.trainers, self.devices):
            with torch.cuda.device(d):
                a, b = t.read_metrics()
            ls, cs = ls + a, cs + b
        return ls, cs

    def state_dict(self) -> dict:
        return self.trainers[0].state_dict()

    def to_module(self):
        return self.trainers[0].to_module()
