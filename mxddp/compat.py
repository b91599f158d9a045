"""Drop-in entry points for every script of the reference, translated onto ``mxddp.train``.

A user of ``MyXiaoPao/distributed-training-dl`` keeps their launch lines: each reference
script's flags (names, short forms, defaults, semantics) are parsed here and mapped to one
``mxddp.train`` invocation.  ``examples/<track>/<script>.py`` are one-line wrappers.

| reference script                               | mxddp mapping                                    |
|------------------------------------------------|--------------------------------------------------|
| pytorch/single_gpu.py                          | pyramidnet110, --mode single                     |
| pytorch/data_parallel.py                       | pyramidnet110, --mode replica (global batch)     |
| pytorch/distributed_data_parallel.py           | pyramidnet110, --mode ddp (same flags)           |
| tensorflow2/mnist_single.py                    | keras_cnn + Adam, single, per-epoch ckpt, eval   |
| tensorflow2/mnist_mirror_strategy.py           | keras_cnn + Adam, --mode replica                 |
| tensorflow2/mnist_multi_worker_strategy.py     | keras_cnn + Adam, ddp from --worker_hosts/--task_index |
| chainer/train_mnist.py                         | mlp(--unit) + Adam, single (CPU with --gpu -1), per-epoch eval, snapshot/--resume |
| chainer/train_mnist_gpu.py                     | mlp + Adam, --mode replica over --gpu_number GPUs |
| chainer/train_mnist_multi.py                   | mlp + Adam, ddp; --communicator naive -> gloo/CPU |

Reference quirks that are FIXED rather than reproduced: ranks from the
launcher are unique (Q1), --seed is applied (Q4), set_epoch reshuffles (Q3), TF2 flags
--learning_rate is honoured only when given explicitly (Q9; the reference silently used
Adam's default 1e-3), checkpoint/TensorBoard writes are rank-0 only except the per-rank DDP
file the reference layout requires (Q6/Q10).
"""
from __future__ import annotations

import argparse
import sys

from . import train as _train

SCRIPTS = [
    "pytorch/single_gpu", "pytorch/data_parallel", "pytorch/distributed_data_parallel",
    "tensorflow2/mnist_single", "tensorflow2/mnist_mirror_strategy", "tensorflow2/mnist_multi_worker_strategy",
    "chainer/train_mnist", "chainer/train_mnist_gpu", "chainer/train_mnist_multi",
]


def _pytorch_parser(lr_flags, li_flags, wd_flags, tb_flags) -> argparse.ArgumentParser:
    p = argparse.ArgumentParser()
    p.add_argument("--train-dir", "-td", default="./train_dir")
    p.add_argument("--dataset-dir", "-dd", default="./data")
    p.add_argument("--batch-size", "-b", type=int, default=64)
    p.add_argument("--num-workers", type=int, default=4)
    p.add_argument(*tb_flags, dest="test_batch_size", type=int, default=1000)
    p.add_argument("--epochs", "-e", type=int, default=10)
    p.add_argument("--gpu-nums", "-g", type=int, default=0)
    p.add_argument(*lr_flags, dest="lr", type=float, default=0.1)
    p.add_argument("--momentum", type=float, default=0.9)
    p.add_argument("--seed", type=int, default=1)
    p.add_argument(*li_flags, dest="log_interval", type=int, default=20)
    p.add_argument("--save-model", "-sm", action="store_true")
    p.add_argument(*wd_flags, dest="wd", type=float, default=1e-4)
    return p


def _tf2_parser(multi_worker: bool, mirror: bool) -> argparse.ArgumentParser:
    p = argparse.ArgumentParser()
    p.add_argument("--train_dir", "-td", default="./train_dir")
    p.add_argument("--batch_size", "-b", type=int, default=64)
    p.add_argument("--test_batchsize", "-tb", type=int, default=1000)
    p.add_argument("--epochs", "-e", type=int, default=10)
    if mirror or multi_worker:
        p.add_argument("--gpu_nums", "-g", type=int, default=0)
        p.add_argument("--cpu_nums", "-c", type=int, default=0)
    p.add_argument("--learning_rate", "-lr", type=float, default=None)
    p.add_argument("--momentum", type=float, default=0.5)
    p.add_argument("--log_interval", type=int, default=10)
    p.add_argument("--save_model", "-sm", action="store_true")
    if multi_worker:
        p.add_argument("--worker_hosts", "-wh", required=True)
        p.add_argument("--job_name", "-j", default="worker")
        p.add_argument("--task_index", "-i", type=int, required=True)
    p.add_argument("--dataset_dir", "-dd", default="./data")
    return p


def _chainer_parser(kind: str) -> argparse.ArgumentParser:
    p = argparse.ArgumentParser()
    p.add_argument("--batchsize", "-b", type=int, default=400 if kind == "gpu" else 100)
    p.add_argument("--epoch", "-e", type=int, default=20)
    if kind == "single":
        p.add_argument("--frequency", "-f", type=int, default=-1)
        p.add_argument("--gpu", "-g", type=int, default=-1)
    else:
        p.add_argument("--gpu", "-g", action="store_true")
    if kind == "gpu":
        p.add_argument("--gpu_number", "-n", type=int, default=1)
    if kind == "multi":
        p.add_argument("--communicator", type=str, default="pure_nccl")
    p.add_argument("--out", "-o", default="result")
    p.add_argument("--resume", "-r", default="")
    p.add_argument("--unit", "-u", type=int, default=1000)
    p.add_argument("--noplot", dest="plot", action="store_false")
    p.add_argument("--dataset-dir", "-dd", default="./data")
    return p


def translate(script: str, argv: list[str]) -> list[str]:
    """Reference script name + its argv -> mxddp.train argv."""
    if script == "pytorch/distributed_data_parallel":
        return ["--model", "pyramidnet110", "--mode", "ddp"] + list(argv)
    if script in ("pytorch/single_gpu", "pytorch/data_parallel"):
        single = script.endswith("single_gpu")
        p = _pytorch_parser(["--learning-rate", "-lr"] if single else ["--learning-rate", "--lr"],
                            ["--log-interval", "-li"] if single else ["--log-interval"],
                            ["--weight-decay", "-wd"] if single else ["--weight-decay", "--wd"],
                            ["--test-batchsize", "-tb"])
        a = p.parse_args(argv)
        if single and a.gpu_nums > 1:  # pytorch/single_gpu.py:44-45
            raise ValueError("single_gpu.py: --gpu-nums must be <= 1")
        out = ["--model", "pyramidnet110", "--mode", "single" if single else "replica",
               "-td", a.train_dir, "-dd", a.dataset_dir, "-b", str(a.batch_size), "-tb", str(a.test_batch_size),
               "-e", str(a.epochs), "--lr", str(a.lr), "--momentum", str(a.momentum), "--seed", str(a.seed),
               "--log-interval", str(a.log_interval), "--wd", str(a.wd), "--lr-step-size", "0"]
        if not single:
            out += ["-g", str(a.gpu_nums)]
        return out + (["-sm"] if a.save_model else [])
    if script.startswith("tensorflow2/"):
        multi = script.endswith("multi_worker_strategy")
        mirror = script.endswith("mirror_strategy")
        a = _tf2_parser(multi, mirror).parse_args(argv)
        out = ["--model", "keras_cnn", "--optimizer", "adam", "-td", a.train_dir, "-dd", a.dataset_dir,
               "-tb", str(a.test_batchsize), "-e", str(a.epochs), "--log-interval", str(a.log_interval),
               "--save-every", "1", "--eval", "--eval-every", "1", "--lr-step-size", "0",  # fit(validation_data)
               # TensorBoard(log_dir=train_dir, histogram_freq=1) + model.summary()
               "--tensorboard-dir", a.train_dir, "--histogram-freq", "1", "--summary",
               # ModelCheckpoint(ckpt_{epoch}, weights only) + load latest before evaluate
               "--epoch-checkpoints"]
        if a.learning_rate is not None:
            out += ["--lr", str(a.learning_rate)]
        if multi:
            if a.job_name != "worker":  # tensorflow2/mnist_multi_worker_strategy.py:15-16
                raise ValueError("job_name must be 'worker' (parameter servers are not supported)")
            hosts = a.worker_hosts.split(",")
            out += ["--mode", "ddp", "--rank", str(a.task_index), "--world-size", str(len(hosts)),
                    "--init-method", f"tcp://{hosts[0]}", "--per-rank-batch", str(max(1, a.batch_size // len(hosts)))]
        elif mirror:
            out += ["--mode", "replica", "-b", str(a.batch_size), "-g", str(a.gpu_nums)]
        else:
            out += ["--mode", "single", "-b", str(a.batch_size)]
        return out + (["-sm"] if a.save_model else [])
    if script.startswith("chainer/"):
        kind = {"chainer/train_mnist": "single", "chainer/train_mnist_gpu": "gpu",
                "chainer/train_mnist_multi": "multi"}[script]
        a = _chainer_parser(kind).parse_args(argv)
        out = ["--model", "mlp", "--optimizer", "adam", "--mlp-units", str(a.unit), "-e", str(a.epoch),
               "-td", a.out, "-dd", a.dataset_dir, "--eval-every", "1", "--lr-step-size", "0",
               "--metrics-jsonl", f"{a.out}/log.jsonl", "-sm",
               # LogReport (<out>/log), PrintReport, dump_graph('main/loss') (<out>/cg.dot)
               "--chainer-out", a.out]
        if a.resume:
            out += ["--resume", a.resume]
        if kind == "single":
            freq = a.frequency if a.frequency > 0 else a.epoch  # default: snapshot at the end
            out += ["--mode", "single", "-b", str(a.batchsize), "--save-every", str(freq)]
            if a.gpu < 0:
                out += ["--cpu"]
        elif kind == "gpu":
            out += ["--mode", "replica", "-b", str(a.batchsize), "-g", str(a.gpu_number)]
            if not a.gpu:
                out += ["--cpu"]
        else:
            out += ["--mode", "ddp", "--per-rank-batch", str(a.batchsize)]
            if a.communicator == "naive" or not a.gpu:
                if a.gpu and a.communicator == "naive":  # chainer/train_mnist_multi.py:52-54
                    raise ValueError("naive communicator does not support GPU")
                out += ["--cpu", "--dist-backend", "gloo"]
        return out
    raise ValueError(f"unknown reference script {script!r}; one of {SCRIPTS}")


def main(script: str, argv: list[str] | None = None) -> int:
    return _train.main(translate(script, sys.argv[1:] if argv is None else argv))
