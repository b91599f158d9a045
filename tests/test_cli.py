"""T0: CLI / log-line / checkpoint compatibility with the reference DDP script.

The reference's argparse block is read as TEXT (never executed) from
/root/reference/pytorch/distributed_data_parallel.py:18-48 when it is available; a pinned copy
of its flag table keeps the test meaningful without the mount.
"""
import os
import re

import pytest
import torch

from mxddp.train import build_parser
from mxddp.utils import logging as L
from mxddp.utils.checkpoint import load_model_state, model_checkpoint_path, save_model, save_training_state, load_training_state

REF = "/root/reference/pytorch/distributed_data_parallel.py"
PINNED = {  # flag -> (short, default) from pytorch/distributed_data_parallel.py:20-48
    "--train-dir": ("-td", "./train_dir"), "--dataset-dir": ("-dd", "./data"), "--batch-size": ("-b", 64),
    "--num-workers": (None, 4), "--test-batch-size": ("-tb", 1000), "--epochs": ("-e", 10),
    "--gpu-nums": ("-g", 0), "--learning-rate": ("--lr", 0.1), "--momentum": (None, 0.9), "--seed": (None, 1),
    "--log-interval": (None, 20), "--save-model": ("-sm", False), "--weight-decay": ("--wd", 1e-4),
    "--init-method": (None, "tcp://127.0.0.1:13456"), "--dist-backend": (None, "nccl"), "--rank": (None, 0),
    "--world-size": (None, 1),
}


def _reference_flags():
    if not os.path.exists(REF):
        return PINNED
    text = open(REF).read()
    out = {}
    for m in re.finditer(r"add_argument\(([^)]*)\)", text, re.S):
        args = m.group(1)
        names = re.findall(r"'(-{1,2}[\w-]+)'", args)
        if not names:
            continue
        d = re.search(r"default=([^,\n]+)", args)
        default = d.group(1).strip() if d else None
        out[names[0]] = (names[1] if len(names) > 1 else None, default)
    return out


def test_reference_flags_accepted_with_same_short_forms():
    p = build_parser()
    opts = {o for a in p._actions for o in a.option_strings}
    for flag, (short, _) in _reference_flags().items():
        assert flag in opts, flag
        if short:
            assert short in opts, short


def test_reference_defaults():
    a = build_parser().parse_args([])
    assert a.train_dir == "./train_dir" and a.dataset_dir == "./data" and a.batch_size == 64
    assert a.num_workers == 4 and a.test_batch_size == 1000 and a.epochs == 10 and a.gpu_nums == 0
    assert a.seed == 1 and a.log_interval == 20 and a.save_model is False
    assert a.init_method == "tcp://127.0.0.1:13456" and a.dist_backend == "nccl" and a.rank == 0 and a.world_size == 1
    # lr / momentum / wd resolve to the reference values for the reference (SGD) model
    from mxddp.models import get_spec
    from mxddp.parallel.comm import DistInfo
    from mxddp.train import _resolve

    opt, lr, mom, wd, mode, bs = _resolve(a, get_spec(a.model), DistInfo())
    assert (opt, lr, mom, wd, mode, bs) == ("sgd", 0.1, 0.9, 1e-4, "ddp", 64)
    assert a.lr_step_size == 2  # StepLR(2, 0.1) in the DDP script


def test_reference_launch_line_parses():
    a = build_parser().parse_args("-td out -dd d -b 32 -e 3 -g 2 --lr 0.05 --momentum 0.8 --wd 5e-4 -sm "
                                  "--init-method tcp://c1:20201 --dist-backend nccl --rank 1 --world-size 4".split())
    assert (a.train_dir, a.batch_size, a.epochs, a.learning_rate, a.weight_decay, a.rank, a.world_size) == (
        "out", 32, 3, 0.05, 5e-4, 1, 4)


def test_log_formats_byte_for_byte():
    s = L.ddp_step_line(1, 2, 40, 391, 1.4861, 45.1734, 0.2741)
    assert s == "From Rank: 1, Epoch:[2][40/391]| loss: 1.486 | acc: 45.173 | batch time: 0.274s "
    assert L.ddp_epoch_line(0, 111.748) == "From Rank: 0, Training time 0:01:51.748000"
    assert L.single_step_line(0, 20, 782, 1.458, 46.49, 0.255) == \
        "Epoch[0]: [20/782]| loss: 1.458 | acc: 46.490 | batch time: 0.255s "
    assert L.single_epoch_line(200.438) == "Training time 0:03:20.438000"


def test_checkpoint_layouts(tmp_path):
    from mxddp.models import build_model

    m = build_model("mnist_cnn")
    p_ddp = save_model(m.state_dict(), str(tmp_path), "ddp", rank=3)
    assert os.path.basename(p_ddp) == "distributed_data_parallel_3.pth"
    sd = torch.load(p_ddp, weights_only=True)
    assert list(sd) == list(m.state_dict()) and not any(k.startswith("module.") for k in sd)
    p_rep = save_model(m.state_dict(), str(tmp_path), "replica")
    assert os.path.basename(p_rep) == "data_parallel_model.pth"
    assert all(k.startswith("module.") for k in torch.load(p_rep, weights_only=True))
    assert list(load_model_state(p_rep)) == list(m.state_dict())
    assert os.path.basename(model_checkpoint_path(str(tmp_path), "single")) == "single_gpu_model.pth"


def test_training_state_roundtrip(tmp_path):
    from mxddp.models import build_model

    m = build_model("mlp")
    p = save_training_state(str(tmp_path), 0, m.state_dict(), {"lr": 0.1, "momentum_buffer": torch.ones(3)},
                            {"last_epoch": 2}, epoch=2, step=100)
    st = load_training_state(p)  # weights_only=True inside
    assert st["epoch"] == 2 and st["step"] == 100 and st["scheduler"]["last_epoch"] == 2
    assert torch.equal(st["optimizer"]["momentum_buffer"], torch.ones(3))


def test_slurm_env_contract(monkeypatch):
    """srun-launched ranks (no torchrun env): rank layout from SLURM_* variables."""
    from mxddp.parallel import comm

    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("SLURM_PROCID", "11")
    monkeypatch.setenv("SLURM_NTASKS", "16")
    monkeypatch.setenv("SLURM_LOCALID", "3")
    monkeypatch.setenv("SLURM_NTASKS_PER_NODE", "8(x2)")
    monkeypatch.setenv("SLURM_LAUNCH_NODE_IPADDR", "10.0.0.7")
    monkeypatch.setenv("SLURM_JOB_ID", "4242")
    e = comm.env_dist()
    assert e == {"rank": 11, "world_size": 16, "local_rank": 3, "local_world_size": 8}
    import os

    assert os.environ["MASTER_ADDR"] == "10.0.0.7" and os.environ["MASTER_PORT"] == str(29500 + 242)


def test_slurm_tasks_per_node_fallbacks(monkeypatch):
    """srun -N2 -n16 without --ntasks-per-node: SLURM_NTASKS_PER_NODE is unset; the per-node
    count must come from SLURM_TASKS_PER_NODE ("8(x2)") or SLURM_NTASKS / SLURM_NNODES, never
    the global world size (which would mark the ranks as sharing GPUs)."""
    from mxddp.parallel import comm

    for k in ("RANK", "WORLD_SIZE", "SLURM_NTASKS_PER_NODE", "SLURM_TASKS_PER_NODE", "SLURM_NNODES",
              "SLURM_JOB_NUM_NODES"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("SLURM_PROCID", "9")
    monkeypatch.setenv("SLURM_NTASKS", "16")
    monkeypatch.setenv("SLURM_LOCALID", "1")
    monkeypatch.setenv("SLURM_TASKS_PER_NODE", "8(x2)")
    assert comm.env_dist()["local_world_size"] == 8
    monkeypatch.delenv("SLURM_TASKS_PER_NODE")
    monkeypatch.setenv("SLURM_NNODES", "2")
    assert comm.env_dist()["local_world_size"] == 8
    monkeypatch.delenv("SLURM_NNODES")
    assert comm.env_dist()["local_world_size"] == 16  # single node: every task is local


def test_rccl_variant_names():
    from mxddp.parallel.comm import parse_variant, rccl_variants

    assert parse_variant("default") == {"ctas": 0, "algo": "", "proto": ""}
    assert parse_variant("Ring:c14") == {"ctas": 14, "algo": "Ring", "proto": ""}
    assert parse_variant("Ring/LL128:c28") == {"ctas": 28, "algo": "Ring", "proto": "LL128"}
    assert parse_variant("auto:c7") == {"ctas": 7, "algo": "", "proto": ""}
    assert "default" in rccl_variants() and "Ring:c7" in rccl_variants()
    import pytest

    with pytest.raises(ValueError):
        parse_variant("Ring:7")


def test_fused_engines_take_reference_batch_sizes():
    """The reference's own per-device batches route to the native fused engines: Chainer's 100 /
    200 / 400 (chainer/train_mnist.py:31, train_mnist_gpu.py:33) and the DDP CLI's -b 64 over 8
    local ranks = 8 per rank (pytorch/distributed_data_parallel.py:71)."""
    from mxddp.train import fused_batch_ok

    assert all(fused_batch_ok("mlp", b) for b in (100, 200, 400, 1, 512))
    assert not fused_batch_ok("mlp", 513)
    assert all(fused_batch_ok("mnist_cnn", b) for b in (8, 64, 1, 100, 128))
    assert not fused_batch_ok("mnist_cnn", 129)
    assert fused_batch_ok("keras_cnn", 64) and not fused_batch_ok("keras_cnn", 12)
