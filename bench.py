#!/usr/bin/env python3
"""Headline benchmark: MNIST CNN data-parallel training throughput on MI355X.

Metric (BASELINE.json): images/sec for the WHOLE job, MNIST CNN DDP, B=64 per rank
(weak scaling), fp32, synthetic 28x28 data generated on device, random-init weights.
Each timed step is a full training step: forward, backward, bucketed RCCL all-reduce
(N>1), SGD(momentum 0.9, wd 1e-4) update.

    python bench.py --gpus 1 --steps 200 --warmup 20
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 200 --warmup 20

Timing: W untimed warm-up steps (the first also captures the hipGraph), then device sync +
barrier + device sync, one tiny alignment all-reduce on the step stream (world size > 1), a
start event, K timed steps, an end event, device sync; the time is the MAX over ranks of the
event-timed K steps (the host clock of the same region is reported as host_ms_per_step).
``warmup_steps_run`` in the JSON counts every untimed step that really ran (autotune trials,
the capture step and the first launch of each captured graph included).
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

METRIC = "images/sec (whole node) MNIST CNN DDP at 1/2/4/8 MI355X; scaling efficiency"
BASELINE_VALUE = None  # BASELINE.json "published": {} -- no MNIST number exists upstream
# secondary models: their own metric names (the headline METRIC is the default mnist_cnn run)
MODEL_METRIC = {
    "resnet50": "images/sec (whole node) ResNet-50 synthetic-ImageNet DDP (BASELINE config 5)",
    "pyramidnet110": "images/sec (whole node) PyramidNet-110 CIFAR-10 DDP (reference pytorch/README.md benchmark)",
    "keras_cnn": "images/sec (whole node) Keras MNIST CNN (reference tensorflow2/, Adam)",
    "mlp": "images/sec (whole node) Chainer MNIST MLP (reference chainer/, Adam)",
}


# --ab KEY=VALUE: measured-once kernel choices kept switchable for A/B runs (docs/BENCHMARKS.md)
AB_SWITCHES = {
    "gk2": ("nhwc_conv_set_gk2", "bf16 NHWC convs, two-stage 128 x 128 tiles: 0 = 8 waves of 64 x 32, 1 = 64 x 64 wave "
                                 "tiles in two k-groups on 16x16x32 MFMAs, 2 = the same on 32x32x16"),
    "fc1_defer": ("mnist_set_fc1_defer", "fused MNIST, world size 1: fc1 weight gradient + SGD in the conv-backward "
                                         "launch's last blocks, resident beside the conv blocks at three per CU (2, "
                                         "default), after F7W's blocks at two per CU (1), or folded into F5 (0)"),
    "w2_defer": ("mlp_set_w2_defer", "fused MLP: the dW2 tile + Adam as extra resident blocks of the l1-backward "
                                     "launch (1) or inside the l2-backward launch (0, default)"),
    "f67_order": ("mnist_set_f67_order", "fused MNIST, batch 64: XCD-aware placement of the conv-backward launch's "
                                         "F6W / F7W / fc1 blocks (1, default) or the plain order (0)"),
    "wgrad_defer": ("ops.set_wgrad_defer", "layer path, world size 1: conv weight-gradient split reductions summed by "
                                           "the optimizer in batched launches (1, default) or one launch per conv (0)"),
    "bn_fold": ("ops.set_bn_fold", "PyramidNet: BN normalise pass folded into the next Winograd conv's input staging "
                                   "(1) or run as its own pass (0, default)"),
    "wgrad_flush_mb": ("ops.set_wgrad_flush_mb", "deferred weight-gradient reductions: flush early past this many MB of "
                                                 "pending partial planes (0 = only at the optimizer step; default 64)"),
    "conv_tile256": ("nhwc_conv_set_glds256", "bf16 NHWC convs, 256x256-tile LDS-DMA kernel on big layers (0/1)"),
    "glds_deep": ("nhwc_conv_set_glds_deep", "bf16 NHWC convs, 128 x 128 two-stage tiles on >= 4 k-tile layers (0 off, 1 >= 192 tiles, 2 all, 3 under-filled only)"),
    "wgrad_tile256": ("nhwc_wgrad_set_tile256", "bf16 NHWC weight gradient, 256 x 256 tiles (1) or 128 x 128 (0)"),
}


def _apply_ab(items) -> dict:
    out = {}
    if not items:
        return out
    from mxddp import native

    for it in items:
        k, sep, v = it.partition("=")
        if not sep or k not in AB_SWITCHES:
            raise SystemExit(f"bench.py: --ab {it!r}: expected KEY=VALUE with KEY in {sorted(AB_SWITCHES)}")
        name = AB_SWITCHES[k][0]
        if name.startswith("ops."):  # a Python-level switch of mxddp.ops
            from mxddp import ops

            getattr(ops, name[4:])(int(v))
        else:
            getattr(native(), name)(int(v))
        out[k] = int(v)
    return out


def _metric(model: str) -> str:
    return MODEL_METRIC.get(model, METRIC)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--batch", type=int, default=64, help="per-rank batch (reference: 64)")
    ap.add_argument("--impl", choices=["fused", "layers", "torch", "replica"], default="fused",
                    help="fused: native hipGraph step (default); layers: mxddp ops + DDP reducer; "
                         "torch: stock PyTorch-ROCm DDP (comparison only); replica: ONE process drives --gpus "
                         "GPUs (MirroredStrategy / DataParallel parity, BASELINE config 4; not via torchrun)")
    ap.add_argument("--variant", type=int, default=1, help="fused kernel variant (0 = generic igemm)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--graph-mode", type=int, default=None, choices=[0, 1, 2],
                    help="fused engine: 0 = eager launches, 1 = whole step(s) incl. RCCL in one graph, 2 = compute "
                         "graphs + eager collectives (default: 1 at world size 1, else autotuned; env MXDDP_GRAPH_MODE)")
    ap.add_argument("--no-autotune", action="store_true",
                    help="fused engine, world size > 1: skip timing the launch strategies before the warm-up")
    ap.add_argument("--steps-per-graph", type=int, default=None, help="fused engine, graph mode 1: steps unrolled per graph")
    ap.add_argument("--force-collectives", action="store_true",
                    help="fused engine: issue the RCCL bucket all-reduces even at world size 1 (measures the DDP path)")
    ap.add_argument("--buckets", default=None, choices=["ovl", "inl", "one", "co"],
                    help="fused MNIST engine: pin the bucket strategy instead of autotuning it (ovl: fc bucket "
                         "all-reduce on the side stream overlapping the conv backward; inl: both buckets in order; "
                         "one: one all-reduce of the whole gradient)")
    ap.add_argument("--transport", default="auto", choices=["auto", "rccl", "peer"],
                    help="fused engine, world size > 1: gradient all-reduce over RCCL's ring, the direct xGMI "
                         "peer all-reduce, or auto (validated + timed during the untimed warm-up)")
    ap.add_argument("--channels-last", action="store_true",
                    help="--impl torch: channels_last memory format (stock PyTorch's NHWC convs, for a fair bf16 baseline)")
    ap.add_argument("--min-warmup-ms", type=float, default=300.0,
                    help="keep running untimed warm-up steps until this much wall time of warm-up ran (GPU "
                         "clock ramp of a fresh process); counted in warmup_steps_run")
    ap.add_argument("--grad-comm-dtype", default="fp32", choices=["fp32", "bf16"],
                    help="layers path DDP: bf16 gradient all-reduce (opt-in; fp32 master gradients)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--lr", type=float, default=0.01, help="SGD lr (momentum 0.9, wd 1e-4 as the reference)")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"],
                    help="GEMM precision of the layers path (headline is fp32, >= the reference's precision)")
    ap.add_argument("--ab", action="append", default=[], metavar="KEY=VALUE",
                    help="A/B switch of a native kernel choice (repeatable; the build default when absent): "
                         + "; ".join(f"{k}: {h}" for k, (_, h) in AB_SWITCHES.items()))
    ap.add_argument("--cpu", action="store_true",
                    help="BASELINE config 1: single process on the CPU (the reference's single_gpu.py CPU fallback)")
    ap.add_argument("--phase-profile", type=int, default=0, metavar="STEPS",
                    help="fused MNIST engine: instead of the benchmark, print the in-kernel phase timings of STEPS "
                         "eager steps (every block stamps its phase boundaries; shows the co-scheduled exchange "
                         "blocks against the conv-backward blocks of the same launch)")
    ap.add_argument("--model", default="mnist_cnn",
                    help="headline: mnist_cnn (fused).  keras_cnn and mlp have fused engines too; pyramidnet110 and "
                         "resnet50 run the layers path")
    return ap.parse_args()


_PHASE = ["start"]


def _phase(name: str, rank: int, ws: int):
    """Where this rank is (world size > 1: also on stderr, so the log of a multi-GPU job that
    stalls says which phase each rank reached)."""
    _PHASE[0] = name
    if ws > 1:
        print(f"bench.py: rank {rank}/{ws}: {name} (t={time.perf_counter() - _T0:.1f} s)", file=sys.stderr, flush=True)


_T0 = time.perf_counter()


def _arm_deadline():
    """Whole-run deadline (MXDDP_BENCH_DEADLINE_S, default 900 s; 0 = off): past it, every
    thread's Python stack is dumped to stderr and the process exits non-zero (faulthandler's
    own watchdog thread, no GIL needed), so a rank stuck in a collective ends the job with a
    traceback naming the call instead of hanging until the driver's limit."""
    import faulthandler

    t = float(os.environ.get("MXDDP_BENCH_DEADLINE_S", "900"))
    if t > 0:
        faulthandler.dump_traceback_later(t, exit=True)
    return t


def main():
    a = parse()
    import torch

    from mxddp.parallel import comm as C

    _arm_deadline()
    ws_env = int(os.environ.get("WORLD_SIZE", "1"))
    if a.cpu:
        return _cpu(a)
    if a.impl == "replica":
        if ws_env != 1:
            print("bench.py: --impl replica is single-process (do not launch it with torchrun)", file=sys.stderr)
            sys.exit(2)
        return _replica(a)
    if ws_env != a.gpus:
        if ws_env == 1 and a.gpus > 1:
            print(f"bench.py: --gpus {a.gpus} needs a launcher (torch.distributed.run)", file=sys.stderr)
            sys.exit(2)
    _phase("rendezvous", int(os.environ.get("RANK", "0")), ws_env)
    # host collectives of the bench are short: a peer that died shows up within minutes
    inf = C.init_distributed(use_gpu=True, timeout_s=float(os.environ.get("MXDDP_GLOO_TIMEOUT_S", "600")))
    ab = _apply_ab(a.ab)
    a.ab_applied = ab
    if a.dtype != "fp32":
        if a.impl == "fused":
            a.impl = "layers"  # the fused MNIST engine is fp32-only
        from mxddp import ops as _ops

        _ops.set_compute_dtype(a.dtype)
    dev = inf.device
    _phase("rccl init", inf.rank, inf.world_size)
    comm = C.rccl_comm(force=a.force_collectives)
    if comm is not None and comm.nranks != inf.world_size:
        raise SystemExit(f"bench.py: rank {inf.rank}: RCCL communicator has {comm.nranks} ranks, the job "
                         f"{inf.world_size} (--gpus {a.gpus})")
    _phase("build", inf.rank, inf.world_size)
    B = a.batch
    tr = None  # the fused engine, when one runs

    if a.model not in ("mnist_cnn", "keras_cnn", "mlp") and a.impl == "fused":
        a.impl = "layers"
    if a.impl == "fused" and a.steps_per_graph is None and 1 < a.steps <= 64:
        # a short timed run (the driver's 20 steps) as ONE graph launch instead of the 2^k
        # remainder graphs of the default 32-step graph: the same steps, one launch latency less
        # (916k -> 925k img/s at 20 steps, profiles/r4_n/)
        a.steps_per_graph = a.steps
    if a.impl == "fused" and a.model in ("keras_cnn", "mlp"):
        # native fused Keras-CNN (csrc/keras_kernels.hip, Keras Adam) / Chainer-MLP step
        # (csrc/mlp_kernels.hip, Chainer Adam)
        peer = None
        if comm is None and inf.world_size > 1:
            from mxddp.parallel import peer as P

            peer = P.peer_comm()
            if peer is None:
                raise SystemExit("bench.py: ranks share a GPU and the peer transport is unavailable")
        kw = dict(batch=B, device=dev, comm=comm, seed=a.seed, use_graph=not a.no_graph,
                  steps_per_graph=a.steps_per_graph, peer=peer, force_collectives=a.force_collectives)
        if a.model == "mlp":
            from mxddp.mlp_engine import FusedMlpTrainer

            tr = FusedMlpTrainer(graph_mode=a.graph_mode, transport=a.transport, **kw)
        else:
            from mxddp.keras_engine import FusedKerasTrainer

            tr = FusedKerasTrainer(**kw)
        run = tr.step
        if a.buckets is not None and hasattr(tr, "autotune"):
            tr._set_buckets(a.buckets)
            a.no_autotune = True
        if hasattr(tr, "autotune") and a.graph_mode is None and not a.no_autotune and tr.eng.reducer_active:
            _phase("autotune", inf.rank, inf.world_size)
            tr.step(1)
            tr.autotune()  # untimed: a few real steps per candidate strategy, before the warm-up
        tr.warm_graphs()
    elif a.impl == "fused":
        from mxddp.engine import FusedMnistTrainer

        peer = None
        if comm is None and inf.world_size > 1:  # ranks share a GPU (rehearsal): peer transport only
            from mxddp.parallel import peer as P

            peer = P.peer_comm()
            if peer is None:
                raise SystemExit("bench.py: ranks share a GPU and the peer transport is unavailable")
            if inf.rank == 0:
                print(f"bench.py: {inf.local_world_size} ranks share {torch.cuda.device_count()} GPU(s): "
                      "peer transport only (functional rehearsal, not a scaling measurement)", file=sys.stderr)
        tr = FusedMnistTrainer(batch=B, device=dev, comm=comm, seed=a.seed, variant=a.variant, lr=a.lr,
                               use_graph=not a.no_graph, graph_mode=a.graph_mode, steps_per_graph=a.steps_per_graph,
                               force_collectives=a.force_collectives, transport=a.transport, peer=peer)
        run = tr.step
        if a.buckets is not None:
            tr._set_buckets(a.buckets)
            a.no_autotune = True
        if a.graph_mode is None and not a.no_autotune and tr.eng.reducer_active:
            _phase("autotune", inf.rank, inf.world_size)
            tr.step(1)
            tr.autotune()  # untimed: a few real steps per candidate strategy, before the warm-up
        if a.phase_profile:
            prof = tr.phase_profile(a.phase_profile)
            if inf.rank == 0:
                print(json.dumps({"phase_profile": prof, "world_size": inf.world_size,
                                  "buckets": getattr(tr, "bucket_strategy", None), "transport": tr.active_transport}, indent=1))
            C.shutdown()
            return
        tr.warm_graphs()  # untimed: first launch of every captured graph (real steps)
    else:
        run = _layers_or_torch(a, torch, inf, dev, comm, B)

    _phase("warm-up", inf.rank, inf.world_size)
    run(a.warmup)
    # clock ramp: a freshly started process's GPU runs its first ~100 ms of steps slower
    # (profiles/r3_intercept): keep stepping, untimed, until --min-warmup-ms of warm-up ran
    # (the slowest rank's elapsed time decides, so every rank runs the same number of steps)
    extra = 0
    torch.cuda.synchronize(dev)
    t_w = time.perf_counter()
    while C.all_reduce_max(time.perf_counter() - t_w) * 1e3 < a.min_warmup_ms:
        n = max(1, min(32, a.steps))
        run(n)
        extra += n
        torch.cuda.synchronize(dev)
    # every untimed step that ran before the timed region: autotune trials, the capture step,
    # the first launch of every captured graph, the requested warm-up and the clock-ramp steps
    warmup_run = (tr.steps + getattr(tr, "discarded_steps", 0) if tr is not None
                  else a.warmup + extra + getattr(a, "layers_eager_steps", 0))
    # Timed region, device-aligned: after the host barrier, ONE tiny all-reduce on the stream the
    # steps run on (the job's RCCL communicator, or the peer transport when ranks share a GPU)
    # lines the ranks' devices up whatever the skew with which their hosts left the barrier; a
    # start event right after it and an end event after the K steps give each rank's device
    # time of exactly those K steps, and the slowest rank decides.  The host clock around the
    # same region (barrier exit -> own device sync) is reported next to it.
    st = tr.stream if tr is not None else torch.cuda.current_stream(dev)
    align_comm, align_peer = (tr.comm, tr.peer) if tr is not None else (comm, _layers_peer(inf, comm))
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    _phase("timed steps", inf.rank, inf.world_size)
    C.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    aligned = C.device_align(st, align_comm, align_peer)
    ev0.record(st)
    run(a.steps)
    ev1.record(st)
    torch.cuda.synchronize(dev)
    # each rank stops its own host clock after its own device sync; the closing barrier runs
    # outside the timed region, so no host collective is inside it
    t_rank = time.perf_counter() - t0
    dev_rank = ev0.elapsed_time(ev1) * 1e-3
    C.barrier()
    dt = C.all_reduce_max(dev_rank)
    dt_host = C.all_reduce_max(t_rank)

    if a.impl == "fused":
        # per-image averages over every step since the device accumulators were last zeroed
        # (autotune zeroes them; warm-up, graph pre-launch and timed steps all accumulate):
        # count the steps BEFORE any reset -- and before the diagnosis pass below, whose
        # collective-free steps add to the accumulators but are not training steps
        loss_sum, correct = tr.read_metrics(reset=False)
        seen = max(1, (tr.steps - tr.steps_at_reset) * B)
        extra = {"train_loss_avg": round(loss_sum / seen, 5), "train_acc": round(correct / seen, 5),
                 "train_images": seen}
    else:
        extra = {}
        if a.impl == "layers" and a.dtype == "bf16":
            from mxddp.ops import nhwc as _nhwc

            # BN backward passes whose statistics came from the consuming conv's data-gradient
            # epilogue vs their own statistics pass (counted while the step was traced / captured)
            extra = {"bn_bwd_stats": dict(_nhwc.BN_BWD_STATS)}

    # Multi-GPU diagnosis (after the measurement, outside the timed region): what RCCL reports
    # for the communicator the steps used, and how much of the step the gradient exchange left
    # exposed -- the same steps, same launch mode, with the collectives removed (replicas
    # diverge from here on; nothing is measured after this)
    diag = {}
    if comm is not None or inf.world_size > 1:
        _phase("diagnosis", inf.rank, inf.world_size)
        used = getattr(tr, "eng_comm", None) or comm
        diag["rccl"] = C.rccl_diag(used)
        if tr is not None and hasattr(tr, "compute_only_ms"):
            dry = tr.compute_only_ms(max(1, min(a.steps, 200)))
            if dry is not None:
                dry = C.all_reduce_max(dry)
                full_ms = dt / a.steps * 1e3
                diag["compute_only_ms_per_step"] = round(dry, 4)
                diag["exposed_comm_ms_per_step"] = round(full_ms - dry, 4)
                if getattr(tr.eng, "coscheduled", False):
                    diag["exposed_comm_note"] = "co-scheduled exchange runs inside F67 and stays in the compute-only pass"
    if inf.rank == 0:
        from mxddp.models import get_spec

        spec = get_spec(a.model)
        total_imgs = a.gpus * B * a.steps
        value = total_imgs / dt
        out = {
            "metric": _metric(a.model),
            "value": round(value, 1),
            "unit": "images/sec",
            "n_gpus": a.gpus,
            "steps": a.steps,
            "warmup": a.warmup,
            "warmup_steps_run": warmup_run,
            "ms_per_step": round(dt / a.steps * 1e3, 4),
            # the same region on each rank's host clock (barrier exit -> own device sync, max)
            "host_ms_per_step": round(dt_host / a.steps * 1e3, 4),
            "timing": f"device events after a {aligned} alignment all-reduce" if aligned != "none" else "device events",
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None if BASELINE_VALUE is None else round(value / BASELINE_VALUE, 3),
            "dtype": a.dtype,
            "grad_comm_dtype": a.grad_comm_dtype if a.impl == "layers" else "fp32",
            "data": _data_desc(spec),
            "config": {"model": a.model, "global_batch": B * a.gpus, "per_rank_batch": B, "seq_len": None,
                       "image": "x".join(map(str, spec.input_shape)), "parallelism": f"dp{a.gpus}", "impl": a.impl,
                       # how the timed steps were actually launched (autotune may pick eager mode 0)
                       "graph": _fused_graph(a, tr) or getattr(a, "layers_graph", False),
                       **_fused_config(a, tr), **({"ab": ab} if ab else {})},
            **extra,
            **diag,
        }
        if C.shared_devices():
            out["shared_gpu_rehearsal"] = True  # several ranks on one GPU: not a scaling number
        print(json.dumps(out), flush=True)
    _phase("done", inf.rank, inf.world_size)
    C.shutdown()


def _layers_peer(inf, comm):
    """The layer path's peer transport when the job has no RCCL communicator (ranks sharing a
    GPU: the DDP reducer exchanges over it), for the timed region's alignment all-reduce."""
    if comm is not None or inf.world_size == 1:
        return None
    from mxddp.parallel import peer as P

    return P.peer_comm()


def _fused_graph(a, tr) -> bool:
    if a.impl != "fused":
        return False
    if a.model == "keras_cnn":
        return bool(tr.eng.captured)
    return tr.eng.graph_mode != 0


def _fused_config(a, tr) -> dict:
    if a.impl != "fused":
        return {}
    if a.model == "keras_cnn":
        return {"optimizer": "adam (Keras eps-hat, lr 1e-3)", "graph_mode": tr.eng.graph_mode,
                "buckets": tr.bucket_strategy if tr.eng.reducer_active else "none",
                "transport": tr.active_transport, "autotune": tr.tuned, "steps_per_graph": a.steps_per_graph}
    if a.model == "mlp":
        return {"optimizer": "adam (Chainer eps-hat, lr 1e-3)", "graph_mode": tr.eng.graph_mode,
                "buckets": tr.bucket_strategy if tr.eng.reducer_active else "none",
                "transport": tr.active_transport, "autotune": tr.tuned, "steps_per_graph": a.steps_per_graph}
    return {"graph_mode": tr.eng.graph_mode, "overlap": tr.eng.overlap, "merged_bucket": tr.eng.merged,
            "coscheduled_exchange": tr.eng.coscheduled,
            "transport": tr.active_transport, "force_collectives": a.force_collectives, "autotune": tr.tuned,
            "wt_stores": _wt_stores(), "steps_per_graph": a.steps_per_graph}


def _wt_stores() -> int:
    from mxddp import native

    return native().mnist_wt_stores()


def _replica(a):
    """In-process replica DP over --gpus GPUs (mxddp.parallel.replica): per-replica batch --batch,
    global batch --batch x --gpus, grouped RCCL all-reduce, flat optimizer per replica."""
    import torch

    from mxddp import native, ops
    from mxddp.models import build_model, get_spec
    from mxddp.optim import SGD, Adam
    from mxddp.parallel.replica import ReplicaGroup

    if a.dtype != "fp32":
        ops.set_compute_dtype(a.dtype)
    devices = [torch.device("cuda", i) for i in range(a.gpus)]
    spec = get_spec(a.model)
    torch.manual_seed(a.seed)
    if a.model in ("mnist_cnn", "keras_cnn", "mlp") and a.dtype == "fp32" and not a.no_graph:
        return _replica_fused(a, devices, spec)

    def make_opt(flat):
        if spec.optimizer == "adam":
            # Keras (1e-7) / Chainer (1e-8) epsilon-hat Adam
            return Adam(flat, lr=spec.lr, eps=1e-7 if a.model == "keras_cnn" else 1e-8, eps_hat=True)
        return SGD(flat, lr=a.lr, momentum=0.9, weight_decay=1e-4)

    # per-device step graphs (MXDDP_REPLICA_GRAPH=0: eager)
    grp = ReplicaGroup(build_model(a.model), devices, make_opt,
                       use_graph=not a.no_graph and os.environ.get("MXDDP_REPLICA_GRAPH", "1") == "1")
    B = a.batch * a.gpus
    D = 1
    for s_ in spec.input_shape:
        D *= s_
    C = native()
    dev = devices[0]
    tmpl = torch.empty(spec.num_classes * D, device=dev)
    ctr = torch.zeros(4, dtype=torch.int32, device=dev)
    x = torch.empty((B,) + tuple(spec.input_shape), device=dev)
    y = torch.empty(B, dtype=torch.int32, device=dev)
    C.synth_templates(tmpl.data_ptr(), spec.num_classes, D, a.seed, torch.cuda.current_stream(dev).cuda_stream)
    loss_fn = lambda o, t: ops.cross_entropy(o, t, return_correct=True)  # noqa: E731

    def run(n):
        for _ in range(n):
            C.synth_batch(x.data_ptr(), y.data_ptr(), tmpl.data_ptr(), B, D, spec.num_classes, a.seed, ctr.data_ptr(),
                          torch.cuda.current_stream(dev).cuda_stream)
            grp.step(x, y.long(), loss_fn)

    def sync_all():
        for d in devices:
            torch.cuda.synchronize(d)

    run(a.warmup)
    sync_all()
    # timed like the fused replicas (FusedReplicas.timed_steps): an alignment exchange across the
    # replicas, then per-device start / end events on each device's current stream (the steps'
    # work is ordered between them); the slowest replica's event time decides
    aligned = grp.align()
    evs = []
    for d in devices:
        with torch.cuda.device(d):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(torch.cuda.current_stream(d))
            evs.append((d, e0, e1))
    t0 = time.perf_counter()
    run(a.steps)
    for d, _, e1 in evs:
        with torch.cuda.device(d):
            e1.record(torch.cuda.current_stream(d))
    sync_all()
    dt_host = time.perf_counter() - t0
    dt = max(e0.elapsed_time(e1) for _, e0, e1 in evs) * 1e-3
    grp.close()
    value = B * a.steps / dt
    print(json.dumps({
        "metric": _metric(a.model), "value": round(value, 1), "unit": "images/sec", "n_gpus": a.gpus, "steps": a.steps,
        "warmup": a.warmup, "warmup_steps_run": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 4),
        "host_ms_per_step": round(dt_host / a.steps * 1e3, 4),
        "timing": f"device events after a {aligned} alignment exchange" if aligned != "none" else "device events",
        "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": a.dtype, "data": _data_desc(spec),
        "config": {"model": a.model, "global_batch": B, "per_rank_batch": a.batch, "seq_len": None,
                   "image": "x".join(map(str, spec.input_shape)), "parallelism": f"replica{a.gpus}",
                   "impl": "replica", "graph": grp._graphs is not None}}), flush=True)


def _replica_fused(a, devices, spec):
    """In-process replicas of the fused MNIST engine (one per GPU, peer transport opened in-process,
    every replica's step one hipGraph launch): MirroredStrategy / DataParallel semantics."""
    import torch

    if a.model == "keras_cnn":
        from mxddp.keras_engine import FusedKerasReplicas

        rep = FusedKerasReplicas(devices, batch=a.batch, seed=a.seed, steps_per_graph=a.steps_per_graph)
    elif a.model == "mlp":
        from mxddp.mlp_engine import FusedMlpReplicas

        rep = FusedMlpReplicas(devices, batch=a.batch, seed=a.seed, steps_per_graph=a.steps_per_graph)
    else:
        from mxddp.parallel.replica import FusedMnistReplicas

        rep = FusedMnistReplicas(devices, batch=a.batch, lr=a.lr, seed=a.seed, steps_per_graph=a.steps_per_graph)
    rep.step(a.warmup)
    rep.synchronize()
    t0 = time.perf_counter()
    dt = rep.timed_steps(a.steps)  # device events after an alignment exchange, slowest replica
    dt_host = time.perf_counter() - t0
    B = a.batch * len(devices)
    value = B * a.steps / dt
    print(json.dumps({
        "metric": _metric(a.model), "value": round(value, 1), "unit": "images/sec", "n_gpus": a.gpus, "steps": a.steps,
        "warmup": a.warmup, "warmup_steps_run": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 4),
        "host_ms_per_step": round(dt_host / a.steps * 1e3, 4),
        "timing": "device events after a peer alignment exchange" if len(devices) > 1 else "device events",
        "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": a.dtype, "data": _data_desc(spec),
        "config": {"model": a.model, "global_batch": B, "per_rank_batch": a.batch, "seq_len": None,
                   "image": "x".join(map(str, spec.input_shape)), "parallelism": f"replica{a.gpus}",
                   "impl": "replica-fused", "transport": "peer (in-process)" if len(devices) > 1 else "none",
                   "graph": True}}), flush=True)


def _cpu(a):
    """BASELINE config 1: the MNIST CNN (or --model) trained by ONE process on the CPU --
    mxddp's CPU op path (PyTorch math, the same functions the GPU kernels are tested against),
    flat SGD, synthetic class-conditional batches generated on the host."""
    import torch

    from mxddp import ops
    from mxddp.models import build_model, get_spec
    from mxddp.optim import SGD
    from mxddp.parallel.flat import FlatParams

    torch.manual_seed(a.seed)
    spec = get_spec(a.model)
    model = build_model(a.model)
    flat = FlatParams(model, torch.device("cpu"))
    opt = SGD(flat, lr=a.lr, momentum=0.9, weight_decay=1e-4)
    g = torch.Generator().manual_seed(a.seed)
    tmpl = torch.rand((spec.num_classes,) + tuple(spec.input_shape), generator=g)
    B = a.batch

    def batch():
        y = torch.randint(0, spec.num_classes, (B,), generator=g)
        return (tmpl[y] + 0.3 * torch.randn((B,) + tuple(spec.input_shape), generator=g)).clamp_(0, 1), y

    def run(n):
        for _ in range(n):
            x, y = batch()
            opt.zero_grad()
            ops.cross_entropy(model(x), y).backward()
            opt.step()

    run(a.warmup)
    t0 = time.perf_counter()
    run(a.steps)
    dt = time.perf_counter() - t0
    value = B * a.steps / dt
    print(json.dumps({
        "metric": _metric(a.model) + " [CPU, single process]", "value": round(value, 1), "unit": "images/sec",
        "n_gpus": 0, "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (host class-conditional, random-init weights)",
        "config": {"model": a.model, "global_batch": B, "per_rank_batch": B, "seq_len": None,
                   "image": "x".join(map(str, spec.input_shape)), "parallelism": "cpu1", "impl": "cpu",
                   "threads": torch.get_num_threads()}}), flush=True)


def _data_desc(spec):
    shape = "x".join(map(str, spec.input_shape[1:]))
    return f"synthetic (on-device class-conditional {shape}, random-init weights)"


def _layers_or_torch(a, torch, inf, dev, comm, B):
    """Layer-by-layer paths (mxddp ops + mxddp DDP, or stock torch DDP for comparison)."""
    import torch.nn.functional as F

    from mxddp import native
    from mxddp.models import build_model, get_spec

    torch.manual_seed(a.seed)
    spec = get_spec(a.model)
    model = build_model(a.model).to(dev)
    if a.impl == "layers":
        from mxddp import ops
        from mxddp.optim import SGD
        from mxddp.parallel.ddp import DistributedDataParallel as DDP

        net = DDP(model, grad_comm_dtype=a.grad_comm_dtype)
        opt = SGD(net.flat, lr=0.1, momentum=0.9, weight_decay=1e-4)
        if "wgrad_defer" not in a.ab_applied:
            # world size 1: nothing reads the gradients before the optimizer, which sums the convs'
            # deferred split reductions in batched launches (ops.set_wgrad_defer)
            ops.set_wgrad_defer(inf.world_size == 1 and not a.force_collectives)
        loss_fn = ops.cross_entropy
    else:
        import torch.nn as nn

        from mxddp import ops as _ops

        _ops.torch_reference_mode().__enter__()  # stock PyTorch-ROCm kernels for every op
        ref = model
        if inf.world_size > 1:
            import torch.distributed as dist

            raise SystemExit("--impl torch is single-GPU only in this harness")
        if a.channels_last:
            ref = ref.to(memory_format=torch.channels_last)
        net = ref
        opt = torch.optim.SGD(net.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
        loss_fn = lambda o, t: F.cross_entropy(o, t)  # noqa: E731
    Cn = native()
    D = 1
    for s_ in spec.input_shape:
        D *= s_
    nc = spec.num_classes
    tmpl = torch.empty(nc * D, device=dev)
    ctr = torch.zeros(4, dtype=torch.int32, device=dev)
    x = torch.empty((B,) + tuple(spec.input_shape), device=dev)
    y = torch.empty(B, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    Cn.synth_templates(tmpl.data_ptr(), nc, D, a.seed, st)

    import contextlib

    # stock-PyTorch comparison at the same compute precision: bf16 autocast (MIOpen/hipBLASLt bf16)
    amp = (torch.autocast("cuda", dtype=torch.bfloat16) if (a.impl == "torch" and a.dtype == "bf16")
           else contextlib.nullcontext())

    def step():
        Cn.synth_batch(x.data_ptr(), y.data_ptr(), tmpl.data_ptr(), B, D, nc, a.seed + inf.rank, ctr.data_ptr(),
                       torch.cuda.current_stream(dev).cuda_stream)
        opt.zero_grad()
        with amp:
            out = net(x.contiguous(memory_format=torch.channels_last) if a.channels_last else x)
            loss = loss_fn(out, y if a.impl == "layers" else y.long())  # mxddp's loss takes int32 labels
        loss.backward()
        opt.step()

    def run_eager(n):
        for _ in range(n):
            step()

    # Whole-step hipGraph for the layer path at ANY world size: the ~700 (ResNet-50) to ~1,500
    # (PyramidNet) kernel launches of a step -- with the DDP buffer broadcast and every bucket
    # all-reduce (RCCL or the peer transport, on the reducer's side stream) -- are replayed
    # without Python / autograd overhead.  Every op of the step is graph-safe (no host sync; LR,
    # Adam / BN step counters and the synthetic data counter live on the device).
    if a.impl == "layers" and not a.no_graph:
        from mxddp.parallel.graphed import capture_stream

        side = capture_stream(dev)  # its split-K planes are reserved before the capture
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            run_eager(2)  # allocator / autograd warm-up outside the capture
        a.layers_eager_steps = 2
        torch.cuda.current_stream(dev).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=side, capture_error_mode="thread_local"):
            step()

        def run_graph(n):
            for _ in range(n):
                graph.replay()

        a.layers_graph = True
        return run_graph
    return run_eager


if __name__ == "__main__":
    main()
