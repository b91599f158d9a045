"""mxddp trainer CLI: one entry point for every training mode of the reference.

Flag surface = a superset of ``pytorch/distributed_data_parallel.py:18-48`` (same long and
short flags, same defaults), so reference launch lines keep working::

    python -m mxddp.train -b 64 -e 10 --lr 0.1 --init-method tcp://127.0.0.1:13456 \
        --dist-backend nccl --rank 0 --world-size 1 -sm

plus ``--model`` (mnist_cnn | keras_cnn | mlp | pyramidnet110 | resnet50), ``--data``
(auto | synthetic | real), ``--mode`` (ddp | single | replica), ``--engine`` (auto | fused |
layers), ``--nproc-per-node`` (single-node torchrun-style spawner), ``--resume``, ...

Modes:
  ddp      one process per GPU (torch DDP / TF2 MultiWorkerMirrored / ChainerMN);
  single   one process, one device -- GPU or CPU (pytorch/single_gpu.py, mnist_single.py,
           chainer/train_mnist.py);
  replica  one process, N GPUs, global batch split (nn.DataParallel / MirroredStrategy /
           ParallelUpdater).
Log lines and checkpoint files follow the reference formats byte for byte.
"""
from __future__ import annotations

import argparse
import math
import os
import sys
import time

import torch


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="mxddp: MI355X-native data-parallel training")
    # ---- reference flags (pytorch/distributed_data_parallel.py:18-48)
    p.add_argument("--train-dir", "-td", type=str, default="./train_dir")
    p.add_argument("--dataset-dir", "-dd", type=str, default="./data")
    p.add_argument("--batch-size", "-b", type=int, default=64,
                   help="batch per NODE launch, divided by the processes spawned on it (reference semantics)")
    p.add_argument("--num-workers", type=int, default=4, help="accepted for compatibility (data is device-resident)")
    p.add_argument("--test-batch-size", "-tb", "--test-batchsize", type=int, default=1000)
    p.add_argument("--epochs", "-e", type=int, default=10)
    p.add_argument("--gpu-nums", "-g", type=int, default=0, help="replica mode: GPUs to use (0 = all visible)")
    p.add_argument("--learning-rate", "--lr", "-lr", type=float, default=None,
                   help="default: 0.1 for SGD models (reference), 1e-3 for Adam models (Keras/Chainer)")
    p.add_argument("--momentum", type=float, default=None)
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--log-interval", "-li", type=int, default=20)
    p.add_argument("--save-model", "-sm", action="store_true", default=False)
    p.add_argument("--weight-decay", "--wd", "-wd", type=float, default=None)
    p.add_argument("--init-method", default="tcp://127.0.0.1:13456", type=str)
    p.add_argument("--dist-backend", default="nccl", type=str, help="nccl (= RCCL on MI355X) or gloo")
    p.add_argument("--rank", default=0, type=int)
    p.add_argument("--world-size", default=1, type=int)
    p.add_argument("--rdzv-timeout", type=float, default=float(os.environ.get("MXDDP_RDZV_TIMEOUT", "1800")),
                   help="seconds a rank waits for the others at rendezvous / collectives (control plane)")
    # ---- mxddp extensions
    p.add_argument("--model", default="pyramidnet110",
                   help="mnist_cnn | keras_cnn | mlp | pyramidnet110 | resnet50 (default: the reference's model)")
    p.add_argument("--data", default="auto", choices=["auto", "synthetic", "real"])
    p.add_argument("--steps-per-epoch", type=int, default=None, help="synthetic data: batches per epoch")
    p.add_argument("--mode", default="auto", choices=["auto", "ddp", "single", "replica"])
    p.add_argument("--engine", default="auto", choices=["auto", "fused", "layers"],
                   help="fused = native hipGraph step (mnist_cnn + SGD on GPU); layers = HIP ops + DDP reducer")
    p.add_argument("--optimizer", default=None, choices=[None, "sgd", "adam"])
    p.add_argument("--lr-step-size", type=int, default=None, help="StepLR step (epochs); 0 = off; default 2 in ddp")
    p.add_argument("--lr-gamma", type=float, default=0.1)
    p.add_argument("--per-rank-batch", type=int, default=None, help="override: batch per process")
    p.add_argument("--nproc-per-node", type=int, default=1, help="spawn this many ranks on this node")
    p.add_argument("--cpu", action="store_true", help="force the CPU path (gloo)")
    p.add_argument("--no-graph", action="store_true",
                   help="fused engine / replica mode: launch eagerly instead of hipGraph replay")
    p.add_argument("--debug-sync", action="store_true",
                   help="synchronise and check for faults after every kernel launch (implies --no-graph)")
    p.add_argument("--bucket-cap-mb", type=float, default=25.0)
    p.add_argument("--transport", default="auto", choices=["auto", "rccl", "peer"],
                   help="gradient all-reduce: RCCL ring, direct xGMI peer all-reduce, or auto (validated + timed)")
    p.add_argument("--resume", type=str, default="", help="training-state file (mxddp_state_<rank>.pt) to resume")
    p.add_argument("--save-every", type=int, default=0, help="write the full training state every N epochs")
    p.add_argument("--eval", action="store_true", help="evaluate on the test split after training")
    p.add_argument("--eval-every", type=int, default=0, help="evaluate every N epochs (Chainer Evaluator)")
    p.add_argument("--mlp-units", type=int, default=1000, help="mlp hidden width (Chainer --unit)")
    p.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"],
                   help="GEMM compute precision: fp32 (exact, reference) or bf16 operands + fp32 accumulate")
    p.add_argument("--metrics-jsonl", type=str, default="", help="append JSONL metrics here")
    p.add_argument("--grad-comm-dtype", default="fp32", choices=["fp32", "bf16"],
                   help="layers path DDP: dtype of the gradient all-reduce (bf16: buckets cast to bf16 on the wire, "
                        "fp32 master gradients / weights; opt-in)")
    p.add_argument("--max-steps", type=int, default=0, help="stop after this many steps (0 = full epochs)")
    p.add_argument("--sync-set-epoch", action="store_true", default=True)
    p.add_argument("--tensorboard-dir", type=str, default="",
                   help="write TensorBoard event files here (TF2 TensorBoard callback; rank 0 only)")
    p.add_argument("--histogram-freq", type=int, default=1, help="TensorBoard weight histograms every N epochs (0 = off)")
    p.add_argument("--profile-batch", type=int, default=2,
                   help="TensorBoard profile_batch: host + device trace of this batch of the first epoch into "
                        "<tensorboard-dir>/plugins/profile (0 = off; only with --tensorboard-dir)")
    p.add_argument("--chainer-out", type=str, default="",
                   help="Chainer trainer extensions: LogReport (<dir>/log), PrintReport, dump_graph (<dir>/cg.dot)")
    p.add_argument("--summary", action="store_true", help="print a Keras-style model summary")
    p.add_argument("--profile-phases", action="store_true",
                   help="layers path: eager steps; log steps write fwd / bwd / opt device times and the DDP comm "
                        "window (ms) to the JSONL stream, with roctx ranges for rocprofv3 --marker-trace")
    p.add_argument("--epoch-checkpoints", action="store_true",
                   help="Keras ModelCheckpoint: weights-only <train-dir>/ckpt_<epoch>.pth every epoch (rank 0); "
                        "with --eval the final evaluation reloads the latest one first")
    return p


class _Reporter:
    """Per-epoch reporting of the reference frameworks' trainer extensions: TensorBoard scalars +
    weight histograms (TF2), Chainer LogReport / PrintReport / dump_graph.  Rank 0 only."""

    def __init__(self, args, inf):
        from .utils.report import LogReport, PrintReport
        from .utils.tensorboard import SummaryWriter

        main = inf.is_main
        self.tb = SummaryWriter(args.tensorboard_dir, enabled=main) if args.tensorboard_dir else None
        from .utils.tensorboard import DeviceTrace

        self.trace = DeviceTrace(args.tensorboard_dir, getattr(args, "profile_batch", 0), enabled=main)
        self.first_epoch = None
        self.hist_freq = args.histogram_freq
        self.log = LogReport(args.chainer_out, enabled=main) if args.chainer_out else None
        self.pr = PrintReport(enabled=main, out=lambda s: print(s, flush=True)) if args.chainer_out else None
        self.graph_path = os.path.join(args.chainer_out, "cg.dot") if (args.chainer_out and main) else None
        self.t0 = time.time()

    def around(self, epoch: int, bi: int, n: int = 1):
        """Wrap a step call covering batches [bi, bi + n) of `epoch` (TensorBoard profile_batch)."""
        if self.first_epoch is None:
            self.first_epoch = epoch
        return self.trace.around(epoch == self.first_epoch, bi, n)

    def first_loss(self, loss, model):
        if self.graph_path is not None and loss.grad_fn is not None:
            from .utils.report import dump_graph

            dump_graph(loss, self.graph_path, dict(model.named_parameters()))
            self.graph_path = None

    def epoch_end(self, epoch, step, loss, acc, val, model):
        if self.tb is not None:
            self.tb.add_scalar("epoch_loss", loss, epoch)
            self.tb.add_scalar("epoch_accuracy", acc, epoch)
            if val is not None:
                self.tb.add_scalar("epoch_val_loss", val[0], epoch)
                self.tb.add_scalar("epoch_val_accuracy", val[1] / 100.0, epoch)
            if self.hist_freq and epoch % self.hist_freq == 0 and model is not None:
                for n, p in model.named_parameters():
                    self.tb.add_histogram(n, p, epoch)
            self.tb.flush()
        if self.log is not None:
            e = {"epoch": epoch, "iteration": step, "main/loss": loss, "main/accuracy": acc,
                 "elapsed_time": time.time() - self.t0}
            if val is not None:
                e["validation/main/loss"], e["validation/main/accuracy"] = val[0], val[1] / 100.0
            self.log.append(e)
            self.pr(e)

    def close(self):
        if self.tb is not None:
            self.tb.close()


def fused_batch_ok(model: str, bs: int) -> bool:
    """Per-device batches the native fused engines take (csrc/*_kernels.hip): the MNIST CNN and
    the MLP pad a partial last 16-row MFMA tile with masked rows (so the reference's own batch
    sizes -- 100 for Chainer, 64 // 8 = 8 per rank for the DDP CLI on 8 GPUs -- run natively)."""
    if model == "mnist_cnn":
        return 1 <= bs <= 128
    if model == "keras_cnn":
        return bs % 8 == 0 and 8 <= bs <= 1024
    if model == "mlp":
        return 1 <= bs <= 512
    return False


def _resolve(args, spec, inf):
    opt = args.optimizer or spec.optimizer
    lr = args.learning_rate if args.learning_rate is not None else (spec.lr if opt == spec.optimizer else
                                                                   (0.1 if opt == "sgd" else 1e-3))
    mom = args.momentum if args.momentum is not None else (spec.momentum if opt == "sgd" else 0.0)
    if opt == "sgd" and args.momentum is None and spec.optimizer != "sgd":
        mom = 0.9
    wd = args.weight_decay if args.weight_decay is not None else spec.weight_decay
    mode = args.mode
    if mode == "auto":
        mode = "ddp"  # the reference's primary script; world_size 1 is a valid DDP job
    if args.lr_step_size is None:
        args.lr_step_size = 2 if mode == "ddp" else 0  # StepLR(2, 0.1) only in the DDP script
    if args.per_rank_batch:
        bs = args.per_rank_batch
    elif mode == "replica":
        bs = args.batch_size  # global batch split across replicas (DataParallel semantics)
    else:
        bs = max(1, args.batch_size // max(1, inf.local_world_size))  # pytorch/distributed_data_parallel.py:71
    return opt, lr, mom, wd, mode, bs


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    from .parallel import comm as C

    if args.nproc_per_node > 1 and "LOCAL_RANK" not in os.environ:
        from .launch import spawn_self

        return spawn_self(args.nproc_per_node, argv if argv is not None else sys.argv[1:], module="mxddp.train")

    use_gpu = torch.cuda.is_available() and not args.cpu
    backend = args.dist_backend if use_gpu else "gloo"
    inf = C.init_distributed(backend=backend, init_method=args.init_method, rank=args.rank,
                             world_size=args.world_size, use_gpu=use_gpu, timeout_s=args.rdzv_timeout)
    from .models import get_spec
    from .utils.seed import seed_everything

    seed_everything(args.seed)
    spec = get_spec(args.model)
    opt_name, lr, mom, wd, mode, bs = _resolve(args, spec, inf)
    if mode == "single" and inf.world_size > 1:
        raise SystemExit("--mode single cannot run with world_size > 1")
    engine = args.engine
    if engine == "auto":
        fusable = ((args.model == "mnist_cnn" and opt_name == "sgd") or
                   (args.model == "keras_cnn" and opt_name == "adam") or
                   (args.model == "mlp" and opt_name == "adam" and args.mlp_units == 1000)) and \
            fused_batch_ok(args.model, bs)
        engine = "fused" if (fusable and use_gpu and mode != "replica" and args.dtype == "fp32"
                             and not (backend == "gloo" and inf.world_size > 1)) else "layers"
    if engine == "fused" and use_gpu and backend == "gloo" and inf.world_size > 1:
        raise SystemExit("--engine fused all-reduces over RCCL / the xGMI peer transport; with --dist-backend gloo "
                         "use --engine layers (gradients over gloo) or --dist-backend nccl")
    if use_gpu:
        from . import native, ops

        ops.set_compute_dtype(args.dtype)
        if args.debug_sync:
            native().set_debug_sync(True)
            args.no_graph = True  # a captured graph cannot be synchronised per kernel
    if inf.is_main:
        print(f"==> mxddp | model {args.model} | mode {mode} | engine {engine} | world {inf.world_size} | "
              f"device {inf.device} | batch/rank {bs} | {opt_name} lr {lr} mom {mom} wd {wd}", flush=True)
    from .utils.logging import MetricsWriter

    mw = MetricsWriter(args.metrics_jsonl if (args.metrics_jsonl and inf.is_main) else None)
    try:
        if engine == "fused":
            _train_fused(args, inf, spec, lr, mom, wd, mode, bs, mw)
        elif mode == "replica":
            _train_replica(args, inf, spec, opt_name, lr, mom, wd, bs, mw)
        else:
            _train_layers(args, inf, spec, opt_name, lr, mom, wd, mode, bs, mw)
    finally:
        mw.close()
        C.shutdown()
    return 0


# ====================================================================================== helpers
def _model_kwargs(args, spec) -> dict:
    return {"n_units": args.mlp_units} if spec.name == "mlp" else {}


def _make_opt(name, flat, lr, mom, wd, spec):
    from .optim import SGD, Adam

    if name == "sgd":
        return SGD(flat, lr=lr, momentum=mom, weight_decay=wd)
    # Keras (1e-7) / Chainer (1e-8) epsilon-hat Adam for the reference Adam models
    return Adam(flat, lr=lr, eps=1e-7 if spec.name == "keras_cnn" else 1e-8, weight_decay=wd, eps_hat=True)


def _log_step(inf, mode, epoch, bi, nb, loss, acc, bt):
    from .utils import logging as L

    if mode == "ddp":
        print(L.ddp_step_line(inf.rank, epoch, bi, nb, loss, acc, bt), flush=True)
    elif inf.is_main:
        print(L.single_step_line(epoch, bi, nb, loss, acc, bt), flush=True)


def _log_epoch(inf, mode, seconds):
    from .utils import logging as L

    if mode == "ddp":
        print(L.ddp_epoch_line(inf.rank, seconds), flush=True)
    elif inf.is_main:
        print(L.single_epoch_line(seconds), flush=True)


_DEBUG_RANKSUM = os.environ.get("MXDDP_DEBUG_RANKSUM", "0") == "1"


def _print_rank_sums(inf, step, flat, runner):
    """MXDDP_DEBUG_RANKSUM=1: every rank's parameter checksum at each log step (rank 0 prints)."""
    import torch.distributed as dist

    cs = (flat.data.double().sum().item(), flat.grad.double().sum().item(), runner.captured)
    allcs = [None] * inf.world_size
    dist.all_gather_object(allcs, cs)
    if inf.is_main:
        print(f"[ranksum] step {step}: " + " | ".join(f"r{r} p={a:.9f} g={b:.9f} graph={c}"
                                                     for r, (a, b, c) in enumerate(allcs)), flush=True)


class _null:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


@torch.no_grad()
def evaluate(model, loader, device) -> tuple[float, float]:
    from . import ops

    model.eval()
    tot_loss = torch.zeros((), device=device)
    tot_corr = torch.zeros((), device=device)
    n = 0
    for x, y in loader:
        loss, corr = ops.cross_entropy(model(x), y, return_correct=True)
        tot_loss += loss * x.shape[0]
        tot_corr += corr
        n += x.shape[0]
    model.train()
    return (tot_loss / max(n, 1)).item(), (100.0 * tot_corr / max(n, 1)).item()


def _maybe_eval(args, inf, spec, model, bs, mw, epoch=None, force=False):
    """Held-out evaluation (TF2 model.evaluate, Chainer Evaluator).  Under DDP each rank
    evaluates its shard of the test set and the sums are all-reduced (ChainerMN
    create_multi_node_evaluator semantics, chainer/train_mnist_multi.py:102-104)."""
    periodic = epoch is not None and args.eval_every and epoch % args.eval_every == 0
    if not (force and args.eval) and not periodic:
        return None
    from .data import build_loader
    from .parallel import comm as C

    ws, rank = (inf.world_size, inf.rank)
    tb = max(1, min(args.test_batch_size, math.ceil(10000 / ws)))
    loader, kind = build_loader(spec.dataset, args.data, args.dataset_dir, tb, inf.device, ws, rank,
                                args.seed + 99, spec.input_shape, spec.num_classes, train=False,
                                steps=max(1, math.ceil(10000 / ws / tb)), template_seed=args.seed)
    loss, acc = evaluate(model, loader, inf.device)
    if ws > 1:
        loss, acc = [v / ws for v in C.all_reduce_sum([loss, acc])]
    if inf.is_main:
        tag = f"epoch {epoch} " if epoch is not None else ""
        print(f"Test ({kind}) {tag}: loss {loss:.4f} | acc {acc:.3f}", flush=True)
    mw.write(kind="eval", epoch=epoch, loss=loss, acc=acc)
    return loss, acc


def _reload_latest(args, inf, model):
    """tensorflow2/mnist_single.py:88-92: reload the latest epoch checkpoint before evaluating."""
    from .parallel import comm as C
    from .utils.checkpoint import latest_checkpoint

    C.barrier()  # rank 0 wrote it
    path = latest_checkpoint(args.train_dir)
    if path is None:
        return
    sd = torch.load(path, map_location="cpu", weights_only=True)
    with torch.no_grad():
        for k, v in model.state_dict().items():
            v.copy_(sd[k].to(v.device))
    if inf.is_main:
        print(f"==> restored {os.path.basename(path)} for evaluation", flush=True)


def _epoch_saves(args, inf, epoch, step, model_sd, opt_sd, sched_sd, loader=None, data_counters=None):
    """End-of-epoch saves every training mode honours: the full resume state every
    --save-every epochs (Chainer snapshot: chainer/train_mnist.py:91-93) and the Keras
    ModelCheckpoint weights ckpt_<epoch>.pth (tensorflow2/mnist_mirror_strategy.py:64)."""
    from .utils.checkpoint import save_epoch_weights, save_training_state

    if args.save_every and epoch % args.save_every == 0:
        extra = {}
        if loader is not None and hasattr(loader, "state_dict"):
            extra["data"] = loader.state_dict()
        if data_counters is not None:
            extra["data_counters"] = data_counters
        save_training_state(args.train_dir, inf.rank, model_sd, opt_sd, sched_sd, epoch, step, extra=extra)
    if args.epoch_checkpoints and inf.is_main:
        save_epoch_weights(model_sd, args.train_dir, epoch)


def _save_final(args, inf, mode, state_dict):
    if not args.save_model:
        return
    from .utils.checkpoint import save_model

    path = save_model(state_dict, args.train_dir, "replica" if mode == "replica" else
                      ("ddp" if mode == "ddp" else "single"), inf.rank)
    if mode == "ddp":
        print("From Rank: {}, model saved.".format(inf.rank), flush=True)
    elif inf.is_main:
        print(f"model saved to {path}", flush=True)


# ====================================================================================== layers
def _train_layers(args, inf, spec, opt_name, lr, mom, wd, mode, bs, mw):
    from . import ops
    from .data import build_loader
    from .models import build_model
    from .optim import StepLR
    from .parallel.ddp import DistributedDataParallel as DDP
    from .parallel.flat import FlatParams
    from .utils.checkpoint import load_training_state

    dev = inf.device
    torch.manual_seed(args.seed)
    model = build_model(spec.name, **_model_kwargs(args, spec)).to(dev)
    if mode == "ddp":
        net = DDP(model, bucket_cap_mb=args.bucket_cap_mb, transport=args.transport if dev.type == "cuda" else "auto",
                  grad_comm_dtype=args.grad_comm_dtype)
        flat = net.flat
    else:
        net, flat = model, FlatParams(model, dev)
    opt = _make_opt(opt_name, flat, lr, mom, wd, spec)
    # one process, no DDP exchange: the optimizer is the gradients' only reader, so the convs'
    # split weight-gradient reductions wait for it and run batched (ops.set_wgrad_defer)
    ops.set_wgrad_defer(dev.type == "cuda" and inf.world_size == 1)
    sched = StepLR(opt, args.lr_step_size, args.lr_gamma) if args.lr_step_size else None
    start_epoch = 1
    st = {}
    if args.resume:
        st = load_training_state(args.resume)
        model.load_state_dict(st["model"])
        opt.load_state_dict(st["optimizer"])
        if sched and st.get("scheduler"):
            sched.load_state_dict(st["scheduler"])
        start_epoch = st["epoch"] + 1
    if inf.is_main:
        print("From Rank: {}, The number of parameters of model is {}".format(
            inf.rank, sum(p.numel() for p in model.parameters())), flush=True)
    loader, kind = build_loader(spec.dataset, args.data, args.dataset_dir, bs, dev, inf.world_size, inf.rank,
                                args.seed, spec.input_shape, spec.num_classes, train=True,
                                steps=args.steps_per_epoch)
    step = 0
    if args.resume:  # data-stream position (Chainer snapshot keeps the iterator position)
        if "data" in st.get("extra", {}):
            loader.load_state_dict(st["extra"]["data"])
        step = int(st.get("step", 0))
    if inf.is_main:
        print(f"==> data: {kind}, {len(loader)} batches/epoch", flush=True)
        if args.summary:
            from .utils.report import model_summary

            print(model_summary(model, spec.input_shape, spec.name), flush=True)
    rep = _Reporter(args, inf)
    from .parallel.graphed import GraphedStep
    from .utils.profiler import PhaseTimer
    from .utils.profiler import range as roctx_range

    cuda = dev.type == "cuda"
    # --profile-phases: eager steps, and every log step is bracketed by device events per phase
    # (fwd / bwd+comm / opt) with roctx ranges, plus the reducer's comm window (first bucket
    # issued -> last bucket done); otherwise the whole step is ONE hipGraph at any world size
    # (parallel/graphed.py) and log steps record the step's device time
    profile = args.profile_phases and cuda
    reducer = getattr(net, "reducer", None) if mode == "ddp" else None
    loss_acc = torch.zeros((), device=dev)
    corr_acc = torch.zeros((), device=dev)
    pt = PhaseTimer(enabled=profile)
    timing = {"on": False}

    def train_step(x, y):
        opt.zero_grad()
        with pt.phase("fwd") if timing["on"] else _null(), roctx_range("fwd") if timing["on"] else _null():
            out = net(x)
            loss, corr = ops.cross_entropy(out, y, return_correct=True)
        if rep.graph_path is not None:
            rep.first_loss(loss, model)
        with pt.phase("bwd") if timing["on"] else _null(), roctx_range("bwd") if timing["on"] else _null():
            loss.backward()
        with pt.phase("opt") if timing["on"] else _null(), roctx_range("opt") if timing["on"] else _null():
            opt.step()
        loss_acc.add_(loss.detach())
        corr_acc.add_(corr)
        return loss.detach(), corr

    use_graph = cuda and not args.no_graph and not profile and not getattr(net, "gloo_data", False)
    runner = GraphedStep(train_step, dev, warmup=2, before_replay=opt._sync_lr, enabled=use_graph)
    for epoch in range(start_epoch, args.epochs + 1):
        if hasattr(loader, "sampler"):
            loader.sampler.set_epoch(epoch)
        net.train()
        loss_acc.zero_()
        corr_acc.zero_()
        total = 0
        t_epoch = t_log = time.time()
        last_log = 0
        for bi, (x, y) in enumerate(loader):
            log = bi % args.log_interval == 0
            timing["on"] = profile and log
            if reducer is not None and profile and hasattr(reducer, "set_timing"):
                reducer.set_timing(log)
            ev = None
            if cuda and log and not profile:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            with rep.around(epoch, bi):
                runner(x, y)
            if ev is not None:
                ev[1].record()
            total += x.shape[0]
            step += 1
            if log:
                _sync(dev)
                if hasattr(net, "check"):
                    net.check()  # a gradient collective that gave up must not go unnoticed
                if _DEBUG_RANKSUM and inf.world_size > 1:
                    _print_rank_sums(inf, step, flat, runner)
                now = time.time()
                bt = (now - t_log) / max(1, bi - last_log) if bi else now - t_log
                t_log, last_log = now, bi
                l_avg, acc = loss_acc.item() / (bi + 1), 100.0 * corr_acc.item() / total
                _log_step(inf, mode, epoch, bi, len(loader), l_avg, acc, bt)
                rec = dict(kind="step", epoch=epoch, step=step, loss=l_avg, acc=acc, batch_time=bt,
                           img_per_s=x.shape[0] * inf.world_size / max(bt, 1e-9), graph=runner.captured)
                if ev is not None:
                    rec["step_ms"] = ev[0].elapsed_time(ev[1])
                if profile:
                    rec.update({f"{k}_ms": v for k, v in pt.summary().items()})
                    pt.totals.clear()
                    pt.counts.clear()
                    if reducer is not None and hasattr(reducer, "last_comm_ms") and getattr(reducer, "active", False):
                        rec["comm_ms"] = reducer.last_comm_ms()
                mw.write(**rec)
            if args.max_steps and step >= args.max_steps:
                break
        _sync(dev)
        _log_epoch(inf, mode, time.time() - t_epoch)
        if sched:
            sched.step()
        val = _maybe_eval(args, inf, spec, model, bs, mw, epoch=epoch)
        nb_done = bi + 1
        rep.epoch_end(epoch, step, loss_acc.item() / max(1, nb_done), corr_acc.item() / max(1, total), val, model)
        _epoch_saves(args, inf, epoch, step, model.state_dict(), opt.state_dict(),
                     sched.state_dict() if sched else None, loader)
        if args.max_steps and step >= args.max_steps:
            break
    if args.epoch_checkpoints and args.eval:
        _reload_latest(args, inf, model)
    _maybe_eval(args, inf, spec, model, bs, mw, force=True)
    rep.close()
    _save_final(args, inf, mode, model.state_dict())


# ====================================================================================== replica
def _train_replica(args, inf, spec, opt_name, lr, mom, wd, bs, mw):
    from . import ops
    from .data import build_loader
    from .models import build_model
    from .optim import StepLR
    from .parallel.replica import ReplicaGroup

    if inf.world_size > 1:
        raise SystemExit("replica mode is single-process (use --mode ddp for multi-process)")
    if inf.device.type == "cuda":
        n = args.gpu_nums or torch.cuda.device_count()
        devices = [torch.device("cuda", i) for i in range(n)]
    else:
        devices = [torch.device("cpu")]
    per = bs // len(devices) if bs % len(devices) == 0 else 0
    if devices[0].type == "cuda" and args.dtype == "fp32" and args.engine != "layers" and per and (
            (spec.name == "mnist_cnn" and opt_name == "sgd") or
            (spec.name == "keras_cnn" and opt_name == "adam" and wd == 0.0) or
            (spec.name == "mlp" and opt_name == "adam" and args.mlp_units == 1000 and wd == 0.0)) and \
            fused_batch_ok(spec.name, per):
        return _train_replica_fused(args, inf, spec, lr, mom, wd, bs, devices, mw)
    torch.manual_seed(args.seed)
    model = build_model(spec.name, **_model_kwargs(args, spec))
    st, start_epoch = {}, 1
    if args.resume:
        from .utils.checkpoint import load_training_state

        st = load_training_state(args.resume)
        model.load_state_dict(st["model"])
        start_epoch = st["epoch"] + 1
    # per-device step graphs (MXDDP_REPLICA_GRAPH=0 or --no-graph: eager)
    group = ReplicaGroup(model, devices, lambda f: _make_opt(opt_name, f, lr, mom, wd, spec),
                         use_graph=(devices[0].type == "cuda" and not args.no_graph
                                    and os.environ.get("MXDDP_REPLICA_GRAPH", "1") == "1"))
    scheds = [StepLR(o, args.lr_step_size, args.lr_gamma) for o in group.optimizers] if args.lr_step_size else []
    loader, kind = build_loader(spec.dataset, args.data, args.dataset_dir, bs, devices[0], 1, 0, args.seed,
                                spec.input_shape, spec.num_classes, train=True, steps=args.steps_per_epoch)
    step = 0
    if st:  # every replica's optimizer / scheduler from the one saved state (replicas are identical)
        for o in group.optimizers:
            o.load_state_dict(st["optimizer"])
        for s_ in scheds:
            if st.get("scheduler"):
                s_.load_state_dict(st["scheduler"])
        if "data" in st.get("extra", {}):
            loader.load_state_dict(st["extra"]["data"])
        step = int(st.get("step", 0))
    print(f"==> replica mode on {len(devices)} device(s), global batch {bs}, data {kind}", flush=True)
    if args.summary:
        from .utils.report import model_summary

        print(model_summary(group.module, spec.input_shape, spec.name), flush=True)
    loss_fn = lambda o, t: ops.cross_entropy(o, t, return_correct=True)  # noqa: E731
    rep = _Reporter(args, inf)
    if rep.graph_path is not None:  # dump_graph from one replica-0 forward on a slice of the first batch
        x0, y0 = next(iter(loader))
        rep.first_loss(loss_fn(group.module(x0[:max(1, x0.shape[0] // len(devices))].to(devices[0])),
                               y0[:max(1, x0.shape[0] // len(devices))].to(devices[0]))[0], group.module)
        group.zero_grad()
    for epoch in range(start_epoch, args.epochs + 1):
        if hasattr(loader, "sampler"):
            loader.sampler.set_epoch(epoch)
        loss_sum = corr_sum = 0.0
        total = 0
        t_epoch = t_log = time.time()
        last_log = 0
        for bi, (x, y) in enumerate(loader):
            with rep.around(epoch, bi):
                group.step(x, y, loss_fn)
            total += x.shape[0]
            step += 1
            if bi % args.log_interval == 0:
                ls, c = group.read_metrics()  # syncs every replica's device
                loss_sum += ls
                corr_sum += c
                now = time.time()
                bt = (now - t_log) / max(1, bi - last_log) if bi else now - t_log
                t_log, last_log = now, bi
                _log_step(inf, "single", epoch, bi, len(loader), loss_sum / total, 100.0 * corr_sum / total, bt)
                mw.write(kind="step", epoch=epoch, step=step, loss=loss_sum / total, acc=100.0 * corr_sum / total,
                         batch_time=bt, img_per_s=x.shape[0] / max(bt, 1e-9), graph=group._graphs is not None)
            if args.max_steps and step >= args.max_steps:
                break
        ls, c = group.read_metrics()  # remainder since the last log line
        loss_sum, corr_sum = loss_sum + ls, corr_sum + c
        _log_epoch(inf, "single", time.time() - t_epoch)
        for s in scheds:
            s.step()
        val = _maybe_eval(args, inf, spec, group.module, bs, mw, epoch=epoch)
        rep.epoch_end(epoch, step, loss_sum / max(1, total), corr_sum / max(1, total), val, group.module)
        _epoch_saves(args, inf, epoch, step, group.module.state_dict(), group.optimizers[0].state_dict(),
                     scheds[0].state_dict() if scheds else None, loader)
        if args.max_steps and step >= args.max_steps:
            break
    if args.epoch_checkpoints and args.eval:
        _reload_latest(args, inf, group.module)
    _maybe_eval(args, inf, spec, group.module, bs, mw, force=True)
    rep.close()
    _save_final(args, inf, "replica", group.module.state_dict())


def _train_replica_fused(args, inf, spec, lr, mom, wd, bs, devices, mw):
    """Replica mode for the MNIST CNN on the fused engine: one FusedMnistTrainer per GPU in this
    process, gradients averaged by the in-process peer transport (parallel/replica.py)."""
    from .data import build_loader
    from .models import build_model
    from .parallel.replica import FusedMnistReplicas

    keras = spec.name == "keras_cnn"
    adam = spec.name in ("keras_cnn", "mlp")
    torch.manual_seed(args.seed)
    init = build_model(spec.name)
    st, start_epoch = {}, 1
    if args.resume:
        from .utils.checkpoint import load_training_state

        st = load_training_state(args.resume)
        init.load_state_dict(st["model"])
        start_epoch = st["epoch"] + 1
    if keras:
        from .keras_engine import FusedKerasReplicas

        rep = FusedKerasReplicas(devices, batch=bs // len(devices), lr=lr, seed=args.seed, init_model=init,
                                 use_graph=not args.no_graph)
    elif spec.name == "mlp":
        from .mlp_engine import FusedMlpReplicas

        rep = FusedMlpReplicas(devices, batch=bs // len(devices), lr=lr, seed=args.seed, init_model=init,
                               use_graph=not args.no_graph)
    else:
        rep = FusedMnistReplicas(devices, batch=bs // len(devices), lr=lr, momentum=mom, weight_decay=wd,
                                 seed=args.seed, init_model=init, use_graph=not args.no_graph)
    step = 0
    if st:
        ctrs = st.get("extra", {}).get("data_counters")
        for i, t in enumerate(rep.trainers):
            if "momentum" in st.get("optimizer", {}):
                t.mom.copy_(st["optimizer"]["momentum"].to(t.device))
            if "m" in st.get("optimizer", {}):
                t.load_optimizer_state(st["optimizer"])
            if ctrs is not None and i < len(ctrs):
                t.load_data_state(ctrs[i])
        step = int(st.get("step", 0))
    loader, kind = build_loader("mnist", args.data, args.dataset_dir, bs, devices[0], 1, 0, args.seed,
                                spec.input_shape, 10, train=True, steps=args.steps_per_epoch)
    print(f"==> replica mode (fused {spec.name} engine) on {len(devices)} device(s), global batch {bs}, data {kind}",
          flush=True)
    rep_ = _Reporter(args, inf)
    base_lr = lr
    for epoch in range(start_epoch, args.epochs + 1):
        if args.lr_step_size:
            for t in rep.trainers:
                t.set_lr(base_lr * args.lr_gamma ** ((epoch - 1) // args.lr_step_size))
        if hasattr(loader, "sampler"):
            loader.sampler.set_epoch(epoch)
        nb, bi = len(loader), 0
        t_epoch = t_log = time.time()
        loss_tot = corr_tot = 0.0
        it = None if kind == "synthetic" else iter(loader)
        while bi < nb:
            if it is None:
                n = 1 if bi % args.log_interval == 0 else min(args.log_interval - bi % args.log_interval, nb - bi)
                with rep_.around(epoch, bi, n):
                    rep.step(n)
            else:
                x, y = next(it)
                if x.shape[0] != bs:
                    bi += 1
                    continue
                n = 1
                rep.set_batch(x, y)
                with rep_.around(epoch, bi):
                    rep.step(1)
            bi += n
            step += n
            if (bi - 1) % args.log_interval == 0 or bi == nb:
                ls, cs = rep.read_metrics()
                loss_tot, corr_tot = loss_tot + ls, corr_tot + cs
                now = time.time()
                _log_step(inf, "single", epoch, bi - 1, nb, loss_tot / (bi * bs), 100.0 * corr_tot / (bi * bs),
                          (now - t_log) / max(1, n))
                t_log = now
            if args.max_steps and step >= args.max_steps:
                break
        rep.synchronize()
        _log_epoch(inf, "single", time.time() - t_epoch)
        model = rep.to_module().to(devices[0])
        val = _maybe_eval(args, inf, spec, model, bs, mw, epoch=epoch)
        rep_.epoch_end(epoch, step, loss_tot / max(1, bi * bs), corr_tot / max(1, bi * bs), val, model)
        t0_ = rep.trainers[0]
        opt_sd = t0_.optimizer_state() if adam else {"momentum": t0_.mom.cpu(), "lr": t0_._lr_host}
        _epoch_saves(args, inf, epoch, step, rep.state_dict(), opt_sd,
                     {"base_lr": base_lr}, None, data_counters=[t.data_state() for t in rep.trainers])
        if args.max_steps and step >= args.max_steps:
            break
    model = rep.to_module().to(devices[0])
    if args.epoch_checkpoints and args.eval:
        _reload_latest(args, inf, model)
    _maybe_eval(args, inf, spec, model, bs, mw, force=True)
    rep_.close()
    _save_final(args, inf, "replica", rep.state_dict())  # save_model adds the module. prefix


# ====================================================================================== fused
def _train_fused(args, inf, spec, lr, mom, wd, mode, bs, mw):
    """The native fused engines: MNIST CNN + SGD (engine.py), the reference's Keras CNN + Keras Adam
    (keras_engine.py) and Chainer MLP + Chainer Adam (mlp_engine.py); one hipGraph launch per step
    (or group of steps)."""
    from .data import build_loader
    from .models import build_model
    from .parallel import comm as C
    from .utils.checkpoint import load_training_state, save_training_state

    dev = inf.device
    keras = spec.name == "keras_cnn"
    adam = spec.name in ("keras_cnn", "mlp")
    torch.manual_seed(args.seed)
    init = build_model(spec.name)
    start_epoch = 1
    st = {}
    if args.resume:
        st = load_training_state(args.resume)
        init.load_state_dict(st["model"])
        start_epoch = st["epoch"] + 1
    comm = C.rccl_comm()
    peer = None
    if comm is None and inf.world_size > 1:  # ranks share a GPU: no RCCL, the peer transport carries the DDP
        from .parallel import peer as _peer

        peer = _peer.peer_comm()
        if peer is None:
            raise SystemExit("ranks share a GPU and the peer transport is unavailable")
    if keras:
        from .keras_engine import FusedKerasTrainer

        tr = FusedKerasTrainer(batch=bs, device=dev, comm=comm, seed=args.seed, lr=lr, eps=1e-7, weight_decay=wd,
                               eps_hat=True, use_graph=not args.no_graph, init_model=init, peer=peer)
        if args.resume and "m" in st.get("optimizer", {}):
            tr.load_optimizer_state(st["optimizer"])
    elif spec.name == "mlp":
        from .mlp_engine import FusedMlpTrainer

        tr = FusedMlpTrainer(batch=bs, device=dev, comm=comm, seed=args.seed, lr=lr, eps=1e-8, weight_decay=wd,
                             eps_hat=True, use_graph=not args.no_graph, init_model=init, peer=peer,
                             transport=args.transport)
        if args.resume and "m" in st.get("optimizer", {}):
            tr.load_optimizer_state(st["optimizer"])
    else:
        from .engine import FusedMnistTrainer

        tr = FusedMnistTrainer(batch=bs, device=dev, comm=comm, seed=args.seed, lr=lr, momentum=mom,
                               weight_decay=wd, use_graph=not args.no_graph, init_model=init, transport=args.transport,
                               peer=peer)
        if args.resume and "momentum" in st.get("optimizer", {}):
            tr.mom.copy_(st["optimizer"]["momentum"].to(dev))
    loader, kind = build_loader("mnist", args.data, args.dataset_dir, bs, dev, inf.world_size, inf.rank, args.seed,
                                spec.input_shape, 10, train=True, steps=args.steps_per_epoch)
    synthetic = kind == "synthetic"
    step = 0
    if args.resume:
        # data-stream position (Chainer snapshot keeps the iterator: chainer/train_mnist.py:91-93):
        # the on-device synthetic counter; a real-data sampler is re-seeded per epoch by set_epoch
        ex = st.get("extra", {})
        if "data_counter" in ex:
            tr.load_data_state(ex["data_counter"])
        step = int(st.get("step", 0))
    if inf.is_main:
        print("From Rank: {}, The number of parameters of model is {}".format(
            inf.rank, sum(p.numel() for p in init.parameters())), flush=True)
        print(f"==> data: {kind}, {len(loader)} batches/epoch, fused hipGraph step={'off' if args.no_graph else 'on'}",
              flush=True)
    rep = _Reporter(args, inf)
    if rep.graph_path is not None or (args.summary and inf.is_main):  # layer model: same graph / shapes
        from . import ops as _ops

        probe = tr.to_module()
        if args.summary and inf.is_main:
            from .utils.report import model_summary

            print(model_summary(probe, spec.input_shape, spec.name), flush=True)
        rep.first_loss(_ops.cross_entropy(probe(torch.zeros(2, 1, 28, 28)), torch.zeros(2, dtype=torch.long)), probe)
    base_lr = lr
    if hasattr(tr, "autotune") and tr.eng.reducer_active and synthetic and not args.no_graph:
        # pick transport / overlap / graph mode on this machine by timing real steps; they are
        # scratch: weights, momentum, data-stream position and metrics are restored afterwards,
        # so the trained model and --max-steps still match epochs x batches
        snap = tr.snapshot()
        tr.step(1)
        tr.autotune()
        tr.restore(snap)
        if inf.is_main:
            print(f"==> DDP step strategy: {tr.tuned}", flush=True)
    for epoch in range(start_epoch, args.epochs + 1):
        if args.lr_step_size:
            tr.set_lr(base_lr * args.lr_gamma ** ((epoch - 1) // args.lr_step_size))
        if hasattr(loader, "sampler"):
            loader.sampler.set_epoch(epoch)
        nb = len(loader)
        t_epoch = t_log = time.time()
        loss_tot, corr_tot, seen = 0.0, 0.0, 0
        bi = 0
        if synthetic:
            while bi < nb:
                n = 1 if bi % args.log_interval == 0 else min(args.log_interval - bi % args.log_interval, nb - bi)
                with rep.around(epoch, bi, n):
                    tr.step(n)
                bi += n
                step += n
                if (bi - 1) % args.log_interval == 0 or bi == nb:
                    ls, cs = tr.read_metrics()
                    loss_tot += ls
                    corr_tot += cs
                    seen_now = bi * bs
                    now = time.time()
                    bt = (now - t_log) / max(1, n)
                    t_log = now
                    _log_step(inf, mode, epoch, bi - 1, nb, loss_tot / seen_now, 100.0 * corr_tot / seen_now, bt)
                    mw.write(kind="step", epoch=epoch, step=step, loss=loss_tot / seen_now, acc=100.0 * corr_tot / seen_now,
                             batch_time=bt, img_per_s=bs * inf.world_size / max(bt, 1e-9))
                if args.max_steps and step >= args.max_steps:
                    break
        else:
            for x, y in loader:
                if x.shape[0] != bs:
                    continue  # the captured graph has a fixed batch (drop_last semantics)
                tr.set_batch(x, y)
                with rep.around(epoch, bi):
                    tr.step(1)
                step += 1
                if bi % args.log_interval == 0:
                    ls, cs = tr.read_metrics()
                    loss_tot += ls
                    corr_tot += cs
                    seen = (bi + 1) * bs
                    now = time.time()
                    bt = (now - t_log) / max(1, args.log_interval if bi else 1)
                    t_log = now
                    _log_step(inf, mode, epoch, bi, nb, loss_tot / seen, 100.0 * corr_tot / seen, bt)
                bi += 1
                if args.max_steps and step >= args.max_steps:
                    break
        tr.synchronize()
        _log_epoch(inf, mode, time.time() - t_epoch)
        if rep.tb is not None or rep.log is not None:
            ls, cs = tr.read_metrics()  # remainder since the last log line
            loss_tot, corr_tot = loss_tot + ls, corr_tot + cs
            seen = max(1, bi * bs)
            rep.epoch_end(epoch, step, loss_tot / seen, corr_tot / seen, None,
                          tr.to_module() if rep.tb is not None else None)
        if args.save_every and epoch % args.save_every == 0:
            opt_sd = tr.optimizer_state() if adam else {"momentum": tr.mom.cpu(), "lr": tr._lr_host}
            save_training_state(args.train_dir, inf.rank, tr.state_dict(), opt_sd, {"base_lr": base_lr}, epoch, step,
                                extra={"data_counter": tr.data_state(), "sampler_epoch": epoch})
        if args.epoch_checkpoints and inf.is_main:
            from .utils.checkpoint import save_epoch_weights

            save_epoch_weights(tr.state_dict(), args.train_dir, epoch)
        if args.max_steps and step >= args.max_steps:
            break
    model = tr.to_module().to(dev)
    if args.epoch_checkpoints and args.eval:
        _reload_latest(args, inf, model)
    _maybe_eval(args, inf, spec, model, bs, mw, force=True)
    rep.close()
    _save_final(args, inf, mode, tr.state_dict())


if __name__ == "__main__":
    sys.exit(main())
