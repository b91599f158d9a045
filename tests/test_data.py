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


def _write_cifar_py(d, n_per=4, extra=None, protocol=2):
    """torchvision's cifar-10-batches-py layout: pickled dicts with bytes keys (the Python-2 files
    load with encoding='bytes'), a uint8 [n, 3072] 'data' array and a 'labels' int list."""
    import pickle

    d.mkdir(parents=True, exist_ok=True)
    for name, v in [(f"data_batch_{i}", i) for i in range(1, 6)] + [("test_batch", 9)]:
        data = np.full((n_per, 3072), v, dtype=np.uint8)
        data[:, 1024:2048] = 100 + v  # channel 1
        b = {b"batch_label": b"x", b"labels": [(v + j) % 10 for j in range(n_per)], b"data": data,
             b"filenames": [b"f%d.png" % j for j in range(n_per)]}
        if extra is not None and name == "data_batch_3":
            b[b"extra"] = extra
        with open(d / name, "wb") as f:
            pickle.dump(b, f, protocol=protocol)


class _NamesAnotherGlobal:
    """Pickles as a call of collections.OrderedDict: harmless, but not a numpy array global."""

    def __reduce__(self):
        import collections

        return (collections.OrderedDict, ())


import pytest  # noqa: E402


@pytest.mark.parametrize("protocol", [2, 4, 5])
def test_cifar_python_layout_accepted(tmp_path, protocol):
    from mxddp.data import load_cifar10_python

    _write_cifar_py(tmp_path / "cifar-10-batches-py", protocol=protocol)
    x, y = load_cifar10_python(str(tmp_path), train=True)
    assert x.shape == (20, 3, 32, 32) and x.dtype == np.uint8
    assert x[0, 0, 0, 0] == 1 and x[0, 1, 5, 5] == 101 and x[4, 0, 0, 0] == 2
    assert y.tolist()[:5] == [1, 2, 3, 4, 2]
    xt, yt = load_cifar10_python(str(tmp_path), train=False)
    assert xt.shape == (4, 3, 32, 32) and yt.tolist() == [9, 0, 1, 2]
    # --data auto reads it (never synthetic when the reference's layout is on disk)
    ld, kind = build_loader("cifar10", "auto", str(tmp_path), 8, "cpu", 1, 0, 1, (3, 32, 32), 10)
    assert kind == "real" and len(ld) == 3


def test_cifar_python_archive_read_in_place(tmp_path):
    """The cifar-10-python.tar.gz torchvision downloads, read without extracting."""
    import tarfile

    from mxddp.data import load_cifar10_python

    _write_cifar_py(tmp_path / "src" / "cifar-10-batches-py")
    root = tmp_path / "root"
    root.mkdir()
    with tarfile.open(root / "cifar-10-python.tar.gz", "w:gz") as t:
        t.add(tmp_path / "src" / "cifar-10-batches-py", arcname="cifar-10-batches-py")
    x, y = load_cifar10_python(str(root), train=True)
    assert x.shape == (20, 3, 32, 32) and not (root / "cifar-10-batches-py").exists()


def test_cifar_python_extra_global_refused(tmp_path):
    """A batch whose pickle names any global beyond numpy's array reconstructors is refused before
    that global is called, and --data auto raises instead of training on synthetic data."""
    from mxddp.data import UnsafePickleError, load_cifar10_python

    _write_cifar_py(tmp_path / "cifar-10-batches-py", extra=_NamesAnotherGlobal())
    with pytest.raises(UnsafePickleError, match="collections.OrderedDict"):
        load_cifar10_python(str(tmp_path), train=True)
    with pytest.raises(UnsafePickleError):
        build_loader("cifar10", "auto", str(tmp_path), 8, "cpu", 1, 0, 1, (3, 32, 32), 10)


def test_cifar_python_array_subclass_refused(tmp_path):
    """numpy's _reconstruct is admitted only for numpy.ndarray itself."""
    import pickle

    from mxddp.data import UnsafePickleError, load_cifar10_python

    d = tmp_path / "cifar-10-batches-py"
    _write_cifar_py(d)
    with open(d / "data_batch_1", "wb") as f:
        pickle.dump({b"data": np.ma.masked_array(np.zeros((1, 3072), np.uint8)), b"labels": [0]}, f, protocol=2)
    with pytest.raises(UnsafePickleError):
        load_cifar10_python(str(tmp_path), train=True)


def test_cifar_layout_present_but_incomplete_is_an_error(tmp_path):
    _write_cifar_py(tmp_path / "cifar-10-batches-py")
    os.remove(tmp_path / "cifar-10-batches-py" / "data_batch_4")
    with pytest.raises(RuntimeError, match="incomplete"):
        build_loader("cifar10", "auto", str(tmp_path), 8, "cpu", 1, 0, 1, (3, 32, 32), 10)
