"""Checkpoints compatible with the reference layouts.

* DDP: ``{train_dir}/distributed_data_parallel_{rank}.pth`` = ``net.module.state_dict()``
  written by EVERY rank after the last epoch (pytorch/distributed_data_parallel.py:103-115),
  keys without a ``module.`` prefix, loadable by a plain nn.Module;
* single device: ``single_gpu_model.pth`` (pytorch/single_gpu.py:77-85);
* replica / DataParallel: ``data_parallel_model.pth`` with ``module.``-prefixed keys
  (pytorch/data_parallel.py:83-91).

Additionally (the Chainer ``snapshot`` + ``--resume`` capability, chainer/train_mnist.py:91-93,
120-122) a full training state file -- model, optimizer, scheduler, epoch, step and RNG
state -- is written atomically and can be resumed from.  All tensors are saved as plain CPU
tensors so ``torch.load(..., weights_only=True)`` reads every file.
"""
from __future__ import annotations

import os

import torch

FILENAMES = {
    "ddp": "distributed_data_parallel_{rank}.pth",
    "single": "single_gpu_model.pth",
    "replica": "data_parallel_model.pth",
}


def _cpu(sd: dict) -> dict:
    return {k: (v.detach().cpu().clone() if torch.is_tensor(v) else v) for k, v in sd.items()}


def _atomic_save(obj, path: str):
    tmp = f"{path}.tmp.{os.getpid()}"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def model_checkpoint_path(train_dir: str, mode: str, rank: int = 0) -> str:
    return os.path.join(train_dir, FILENAMES[mode].format(rank=rank))


def save_model(state_dict: dict, train_dir: str, mode: str, rank: int = 0) -> str:
    os.makedirs(train_dir, exist_ok=True)  # race-free across ranks (fixes SURVEY §2.9 Q6)
    sd = _cpu(state_dict)
    if mode == "replica":
        sd = {f"module.{k}": v for k, v in sd.items()}
    path = model_checkpoint_path(train_dir, mode, rank)
    _atomic_save(sd, path)
    return path


def load_model_state(path: str) -> dict:
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if sd and all(k.startswith("module.") for k in sd):
        sd = {k[len("module."):]: v for k, v in sd.items()}
    return sd


def state_path(train_dir: str, rank: int = 0) -> str:
    return os.path.join(train_dir, f"mxddp_state_{rank}.pt")


def save_training_state(train_dir: str, rank: int, model_sd: dict, opt_sd: dict | None, sched_sd: dict | None,
                        epoch: int, step: int, extra: dict | None = None) -> str:
    os.makedirs(train_dir, exist_ok=True)
    state = {
        "model": _cpu(model_sd),
        "optimizer": {k: (v.cpu() if torch.is_tensor(v) else v) for k, v in (opt_sd or {}).items()},
        "scheduler": sched_sd or {},
        "epoch": int(epoch),
        "step": int(step),
        "torch_rng": torch.get_rng_state(),
        "extra": extra or {},
    }
    path = state_path(train_dir, rank)
    _atomic_save(state, path)
    return path


def load_training_state(path: str) -> dict:
    return torch.load(path, map_location="cpu", weights_only=True)


# ----------------------------------------------------------------------------- Keras ModelCheckpoint
# tensorflow2/mnist_single.py:67-76: ModelCheckpoint(filepath=train_dir/ckpt_{epoch},
# save_weights_only=True) every epoch, then load_weights(tf.train.latest_checkpoint(train_dir))
# and evaluate (:88-92).
def save_epoch_weights(model_sd: dict, train_dir: str, epoch: int) -> str:
    os.makedirs(train_dir, exist_ok=True)
    path = os.path.join(train_dir, f"ckpt_{epoch}.pth")
    _atomic_save(_cpu(model_sd), path)
    return path


def latest_checkpoint(train_dir: str) -> str | None:
    """Path of the highest-epoch ``ckpt_{epoch}.pth`` in train_dir (None if there is none)."""
    best, best_ep = None, -1
    if not os.path.isdir(train_dir):
        return None
    for f in os.listdir(train_dir):
        if f.startswith("ckpt_") and f.endswith(".pth") and f[5:-4].isdigit() and int(f[5:-4]) > best_ep:
            best, best_ep = os.path.join(train_dir, f), int(f[5:-4])
    return best
