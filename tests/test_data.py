"""Data loaders and sharding vs the reference semantics."""
import gzip
import os

import numpy as np
import torch
from torch.utils.data.distributed import DistributedSampler

from mxddp.data import ShardSampler, SyntheticLoader, TensorLoader, build_loader, load_cifar10, load_mnist, read_idx


def _write_idx(path, arr):
    arr = np.asarray(arr, dtype=np.uint8)
    magic = (0x08 << 8) | arr.ndim
    with (gzip.open(path, "wb") if path.endswith(".gz") else open(path, "wb")) as f:
        f.write(magic.to_bytes(4, "big"))
        for d in arr.shape:
            f.write(int(d).to_bytes(4, "big"))
        f.write(arr.tobytes())


def test_idx_roundtrip(tmp_path):
    img = np.random.randint(0, 256, (7, 28, 28)).astype(np.uint8)
    lab = np.random.randint(0, 10, (7,)).astype(np.uint8)
    _write_idx(str(tmp_path / "train-images-idx3-ubyte.gz"), img)
    _write_idx(str(tmp_path / "train-labels-idx1-ubyte"), lab)
    assert np.array_equal(read_idx(str(tmp_path / "train-images-idx3-ubyte.gz")), img)
    x, y = load_mnist(str(tmp_path), train=True)
    assert np.array_equal(x, img) and np.array_equal(y, lab.astype(np.int64))


def test_mnist_npz_keras_format(tmp_path):
    xtr = np.random.randint(0, 256, (5, 28, 28)).astype(np.uint8)
    np.savez(tmp_path / "mnist.npz", x_train=xtr, y_train=np.arange(5) % 10, x_test=xtr[:2], y_test=np.arange(2))
    x, y = load_mnist(str(tmp_path), train=False)
    assert x.shape == (2, 28, 28) and list(y) == [0, 1]


def test_cifar_binary(tmp_path):
    d = tmp_path / "cifar-10-batches-bin"
    d.mkdir()
    for i in range(1, 6):
        raw = np.zeros((3, 3073), dtype=np.uint8)
        raw[:, 0] = [i % 10, 1, 2]
        raw[:, 1:] = i
        raw.tofile(d / f"data_batch_{i}.bin")
    x, y = load_cifar10(str(tmp_path), train=True)
    assert x.shape == (15, 3, 32, 32) and y[0] == 1 and x[3, 0, 0, 0] == 2


def test_shard_sampler_matches_torch_distributed_sampler():
    class DS:
        def __len__(self):
            return 10

    for shuffle in (False, True):
        for ws in (1, 3, 4):
            for rank in range(ws):
                ref = DistributedSampler(DS(), num_replicas=ws, rank=rank, shuffle=shuffle, seed=7)
                ref.set_epoch(3)
                mine = ShardSampler(10, ws, rank, shuffle=shuffle, seed=7)
                mine.set_epoch(3)
                assert list(ref) == list(mine.indices()), (shuffle, ws, rank)
                assert len(mine) == len(ref)


def test_shard_sampler_padding_and_epoch_reshuffle():
    s = ShardSampler(10, 4, 0, shuffle=True, seed=0)  # 10 samples / 4 ranks -> 3 each (padded)
    assert len(s) == 3
    a = s.indices().tolist()
    s.set_epoch(1)
    assert s.indices().tolist() != a  # set_epoch reshuffles (reference bug Q3 fixed)


def test_tensor_loader_cpu_normalises():
    x = np.full((6, 28, 28), 255, dtype=np.uint8)
    y = np.arange(6)
    ld = TensorLoader(x, y, 4, "cpu", ShardSampler(6, 1, 0, shuffle=False), 0.5, 0.5)
    batches = list(ld)
    assert len(batches) == 2 and batches[0][0].shape == (4, 1, 28, 28)
    assert torch.allclose(batches[0][0], torch.ones(4, 1, 28, 28))


def test_synthetic_loader_cpu_learnable_shape():
    ld = SyntheticLoader((1, 28, 28), 10, 8, 3, "cpu", seed=1)
    xs = list(ld)
    assert len(xs) == 3 and xs[0][0].shape == (8, 1, 28, 28) and xs[0][1].dtype == torch.int64
    assert float(xs[0][0].min()) >= 0.0 and float(xs[0][0].max()) <= 1.0


def test_synthetic_heldout_set_shares_training_templates():
    """The held-out synthetic set (another sample seed) keeps the training run's class templates:
    a nearest-template classifier fit on the train templates labels it correctly."""
    train = SyntheticLoader((1, 28, 28), 10, 64, 1, "cpu", seed=1)
    test = SyntheticLoader((1, 28, 28), 10, 64, 1, "cpu", seed=100, template_seed=1)
    other = SyntheticLoader((1, 28, 28), 10, 64, 1, "cpu", seed=100)
    assert torch.equal(train.tmpl, test.tmpl) and not torch.equal(train.tmpl, other.tmpl)
    x, y = next(iter(test))
    pred = torch.cdist(x.flatten(1), train.tmpl).argmin(1)
    assert (pred == y).float().mean() > 0.9


def test_build_loader_auto_falls_back_to_synthetic(tmp_path):
    ld, kind = build_loader("mnist", "auto", str(tmp_path), 16, "cpu", 2, 0, 1, (1, 28, 28), 10)
    assert kind == "synthetic" and len(ld) == 30000 // 16 + 1 - (1 if 30000 % 16 == 0 else 0)
