"""Datasets, sharding and device-resident batch loaders.

Reference data paths replaced:

* torchvision CIFAR10 + DataLoader(num_workers=4) + RandomCrop/Flip/Normalize
  (pytorch/single_gpu.py:51-61) -> CIFAR-10 batches kept resident in HBM, augmented on device
  by ``mxddp._C.augment_crop_flip_norm``.  Both on-disk layouts are read: the *binary* batches
  (``cifar-10-batches-bin``) with numpy, and the *python* batches torchvision's
  ``CIFAR10(root, download=True)`` leaves (``cifar-10-batches-py``, or the
  ``cifar-10-python.tar.gz`` it downloads, read in place) with an allowlisted unpickler;
* Keras ``mnist.load_data(path=.../mnist.npz)`` (tensorflow2/mnist_single.py:34-47) and the
  Chainer IDX parser with its npz cache (chainer/mnist_helper.py:9-53,
  chainer/mnist_dataset.py:8-38) -> one loader for both formats, vectorised (the reference
  parses IDX byte by byte in Python);
* DistributedSampler / ChainerMN scatter_dataset sharding -> ``ShardSampler`` (padded to a
  multiple of world_size, per-epoch reshuffle -- fixes the reference's missing set_epoch);
* no dataset on disk (this environment has no network) -> class-conditional synthetic data
  generated on device by a Philox kernel, identical in shape to the real dataset.

Only loaders that execute nothing from the file are used: numpy.load with allow_pickle=False,
raw byte parsing, and for the pickled CIFAR "python" batches ``_CifarUnpickler``, which resolves
only numpy's array / dtype reconstructors (and the latin-1 bytes codec a protocol-2 pickle
uses) and refuses every other global, so a pickle that names anything else is rejected before
any of it runs.  ``--data auto`` never swaps in synthetic data for a dataset that is on disk
but unreadable: it raises.
"""
from __future__ import annotations

import gzip
import io
import math
import os
import pickle
import sys
import tarfile

import numpy as np
import torch

from .. import native

MNIST_MEAN, MNIST_STD = 0.1307, 0.3081
CIFAR_MEAN = (0.4914, 0.4822, 0.4465)  # pytorch/distributed_data_parallel.py:83
CIFAR_STD = (0.2023, 0.1994, 0.2010)


# ----------------------------------------------------------------------------- file formats
def _open(path):
    return gzip.open(path, "rb") if path.endswith(".gz") else open(path, "rb")


def read_idx(path: str) -> np.ndarray:
    """IDX (MNIST) file -> ndarray, vectorised (no per-byte Python loop)."""
    with _open(path) as f:
        data = f.read()
    magic = int.from_bytes(data[0:4], "big")
    ndim = magic & 0xFF
    dtype_code = (magic >> 8) & 0xFF
    if dtype_code != 0x08:
        raise ValueError(f"{path}: only ubyte IDX files are supported (type 0x{dtype_code:02x})")
    dims = [int.from_bytes(data[4 + 4 * i:8 + 4 * i], "big") for i in range(ndim)]
    off = 4 + 4 * ndim
    arr = np.frombuffer(data, dtype=np.uint8, count=int(np.prod(dims)), offset=off)
    return arr.reshape(dims)


def _find(root: str, names):
    for n in names:
        for cand in (n, n + ".gz"):
            p = os.path.join(root, cand)
            if os.path.exists(p):
                return p
    return None


def load_mnist(root: str, train: bool = True):
    """(images uint8 [N,28,28], labels int64 [N]) from IDX files or a Keras-style mnist.npz."""
    npz = _find(root, ["mnist.npz"])
    if npz is not None:
        with np.load(npz, allow_pickle=False) as d:
            return (d["x_train"], d["y_train"].astype(np.int64)) if train else (d["x_test"], d["y_test"].astype(np.int64))
    pre = "train" if train else "t10k"
    img = _find(root, [f"{pre}-images-idx3-ubyte", f"{pre}-images.idx3-ubyte"])
    lab = _find(root, [f"{pre}-labels-idx1-ubyte", f"{pre}-labels.idx1-ubyte"])
    if img is None or lab is None:
        raise FileNotFoundError(f"MNIST not found under {root} (IDX files or mnist.npz)")
    x, y = read_idx(img), read_idx(lab).astype(np.int64)
    if len(x) != len(y):  # chainer/mnist_helper.py:14-18
        raise ValueError("MNIST image/label count mismatch")
    return x, y


def load_cifar10(root: str, train: bool = True):
    """(images uint8 [N,3,32,32], labels int64 [N]) from the CIFAR-10 binary version."""
    base = os.path.join(root, "cifar-10-batches-bin") if os.path.isdir(os.path.join(root, "cifar-10-batches-bin")) else root
    files = [f"data_batch_{i}.bin" for i in range(1, 6)] if train else ["test_batch.bin"]
    xs, ys = [], []
    for fn in files:
        p = os.path.join(base, fn)
        if not os.path.exists(p):
            raise FileNotFoundError(f"CIFAR-10 binary batch {p} not found")
        raw = np.fromfile(p, dtype=np.uint8).reshape(-1, 3073)
        ys.append(raw[:, 0].astype(np.int64))
        xs.append(raw[:, 1:].reshape(-1, 3, 32, 32))
    return np.concatenate(xs), np.concatenate(ys)


class UnsafePickleError(pickle.UnpicklingError):
    """A CIFAR python batch named a global outside the numpy-array allowlist."""


def _np_reconstruct(subtype, shape, dtype):
    if subtype is not np.ndarray:
        raise UnsafePickleError(f"array reconstruction of {subtype!r} refused (only numpy.ndarray)")
    return np.ndarray.__new__(np.ndarray, shape, dtype)


def _np_frombuffer(buf, dtype, shape, order):
    return np.frombuffer(buf, dtype=dtype).reshape(shape, order=order).copy()


def _latin1_encode(obj, encoding="latin1"):
    if not isinstance(obj, str) or encoding not in ("latin1", "latin-1"):
        raise UnsafePickleError("_codecs.encode only for latin-1 str -> bytes")
    return obj.encode("latin1")


# (module, name) -> object; numpy 1.x pickles say numpy.core, numpy 2.x numpy._core
_PICKLE_ALLOW = {
    ("numpy", "ndarray"): np.ndarray,
    ("numpy", "dtype"): np.dtype,
    ("numpy.core.multiarray", "_reconstruct"): _np_reconstruct,
    ("numpy._core.multiarray", "_reconstruct"): _np_reconstruct,
    ("numpy.core.numeric", "_frombuffer"): _np_frombuffer,
    ("numpy._core.numeric", "_frombuffer"): _np_frombuffer,
    ("_codecs", "encode"): _latin1_encode,
}


class _CifarUnpickler(pickle.Unpickler):
    """Resolves only the numpy array / dtype reconstruction globals (a CIFAR batch is a dict of
    bytes keys, int lists and one uint8 array); any other global raises before it is called."""

    def find_class(self, module, name):
        obj = _PICKLE_ALLOW.get((module, name))
        if obj is None:
            raise UnsafePickleError(f"CIFAR batch pickle names {module}.{name}: refused (not a numpy array global)")
        return obj


def _cifar_batch(f) -> tuple:
    d = _CifarUnpickler(f, encoding="bytes").load()
    if not isinstance(d, dict):
        raise ValueError("CIFAR python batch: not a dict")
    d = {(k.decode("latin1") if isinstance(k, bytes) else k): v for k, v in d.items()}
    data, labels = d.get("data"), d.get("labels", d.get("fine_labels"))
    if not isinstance(data, np.ndarray) or labels is None:
        raise ValueError("CIFAR python batch: no 'data' array / 'labels' list")
    x = np.asarray(data, dtype=np.uint8).reshape(-1, 3, 32, 32)
    y = np.asarray(labels, dtype=np.int64)
    if len(x) != len(y):
        raise ValueError("CIFAR python batch: image / label count mismatch")
    return x, y


def load_cifar10_python(root: str, train: bool = True):
    """(images uint8 [N,3,32,32], labels int64 [N]) from torchvision's layout: the extracted
    ``cifar-10-batches-py`` directory, or the ``cifar-10-python.tar.gz`` archive (members read
    in memory, nothing is extracted).  pytorch/distributed_data_parallel.py:85-86"""
    names = [f"data_batch_{i}" for i in range(1, 6)] if train else ["test_batch"]
    d = os.path.join(root, "cifar-10-batches-py")
    if not os.path.isdir(d) and os.path.basename(os.path.normpath(root)) == "cifar-10-batches-py":
        d = root
    parts = []
    if os.path.isdir(d):
        for n in names:
            p = os.path.join(d, n)
            if not os.path.exists(p):
                raise FileNotFoundError(f"CIFAR-10 python batch {p} not found")
            with open(p, "rb") as f:
                parts.append(_cifar_batch(f))
    else:
        tgz = os.path.join(root, "cifar-10-python.tar.gz")
        if not os.path.exists(tgz):
            raise FileNotFoundError(f"no cifar-10-batches-py / cifar-10-python.tar.gz under {root}")
        with tarfile.open(tgz, "r:gz") as t:
            for n in names:
                m = t.getmember(f"cifar-10-batches-py/{n}")
                if not m.isfile():
                    raise ValueError(f"{tgz}: {m.name} is not a regular file")
                parts.append(_cifar_batch(io.BytesIO(t.extractfile(m).read())))
    return np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts])


def cifar10_layout(root: str) -> str | None:
    """Which CIFAR-10 layout is under ``root``: 'bin', 'python', or None."""
    if os.path.isdir(os.path.join(root, "cifar-10-batches-bin")) or os.path.exists(os.path.join(root, "data_batch_1.bin")):
        return "bin"
    if (os.path.isdir(os.path.join(root, "cifar-10-batches-py")) or os.path.exists(os.path.join(root, "cifar-10-python.tar.gz"))
            or os.path.exists(os.path.join(root, "data_batch_1"))):
        return "python"
    return None


def load_cifar10_any(root: str, train: bool = True):
    """The binary layout if present, else torchvision's python layout."""
    if cifar10_layout(root) == "python":
        return load_cifar10_python(root, train)
    return load_cifar10(root, train)


# ----------------------------------------------------------------------------- sharding
class ShardSampler:
    """DistributedSampler semantics (verified): pad the index list to a multiple
    of world_size by wrapping, rank r takes indices[r::world_size]; reshuffled every epoch
    from (seed, epoch) when shuffle=True."""

    def __init__(self, n: int, world_size: int = 1, rank: int = 0, shuffle: bool = True, seed: int = 0,
                 drop_last: bool = False):
        self.n, self.ws, self.rank, self.shuffle, self.seed = n, world_size, rank, shuffle, seed
        self.drop_last = drop_last
        self.num_samples = n // world_size if drop_last else math.ceil(n / world_size)
        self.total = self.num_samples * world_size
        self.epoch = 0

    def set_epoch(self, epoch: int):
        self.epoch = epoch

    def indices(self) -> np.ndarray:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g).numpy()
        else:
            idx = np.arange(self.n)
        if self.drop_last:
            idx = idx[:self.total]
        elif self.total > self.n:
            reps = math.ceil((self.total - self.n) / self.n)
            idx = np.concatenate([idx] + [idx] * reps)[:self.total]
        return idx[self.rank:self.total:self.ws]

    def __len__(self):
        return self.num_samples


# ----------------------------------------------------------------------------- loaders
class TensorLoader:
    """Whole dataset resident on the target device; each batch is one on-device gather.
    Yields (x float32 [B,C,H,W] normalised, y int64 [B])."""

    def __init__(self, images: np.ndarray, labels: np.ndarray, batch_size: int, device, sampler: ShardSampler,
                 mean, std, augment: bool = False, drop_last: bool = False, seed: int = 0):
        x = torch.from_numpy(np.ascontiguousarray(images))
        if x.dim() == 3:
            x = x.unsqueeze(1)
        self.device = torch.device(device)
        self.x = x.to(self.device)  # uint8 resident copy (MNIST 47 MB, CIFAR 154 MB)
        self.y = torch.from_numpy(labels).to(self.device)
        self.C = self.x.shape[1]
        self.mean = torch.tensor(mean if isinstance(mean, (tuple, list)) else [mean] * self.C, device=self.device)
        self.std = torch.tensor(std if isinstance(std, (tuple, list)) else [std] * self.C, device=self.device)
        self.batch_size, self.sampler, self.augment, self.drop_last = batch_size, sampler, augment, drop_last
        self.seed = seed
        self._ctr = torch.zeros(4, dtype=torch.int32, device=self.device)

    def __len__(self):
        n = len(self.sampler)
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)

    def state_dict(self) -> dict:
        """Stream position for resume: the sampler epoch (the shuffle of an epoch is a function
        of (seed, epoch)) and the augmentation Philox counter."""
        return {"sampler_epoch": self.sampler.epoch, "aug_counter": self._ctr.cpu().clone()}

    def load_state_dict(self, sd: dict):
        self.sampler.set_epoch(int(sd.get("sampler_epoch", self.sampler.epoch)))
        if "aug_counter" in sd:
            self._ctr.copy_(sd["aug_counter"].to(self._ctr.device))

    def __iter__(self):
        idx = torch.from_numpy(self.sampler.indices()).to(self.device)
        for i in range(len(self)):
            bi = idx[i * self.batch_size:(i + 1) * self.batch_size]
            xb = self.x.index_select(0, bi).float().div_(255.0)
            yb = self.y.index_select(0, bi)
            if self.augment and self.device.type == "cuda":
                out = torch.empty_like(xb)
                N, C, H, W = xb.shape
                native().augment_crop_flip_norm(xb.data_ptr(), out.data_ptr(), N, C, H, W, 4, self.mean.data_ptr(),
                                                self.std.data_ptr(), self.seed, self._ctr.data_ptr(),
                                                torch.cuda.current_stream(self.device).cuda_stream)
                self._ctr.add_(1)
                xb = out
            else:
                if self.augment:
                    xb = _cpu_augment(xb, 4)
                xb = (xb - self.mean.view(1, -1, 1, 1)) / self.std.view(1, -1, 1, 1)
            yield xb, yb


def _cpu_augment(x: torch.Tensor, pad: int) -> torch.Tensor:
    N, C, H, W = x.shape
    xp = torch.nn.functional.pad(x, (pad, pad, pad, pad))
    out = torch.empty_like(x)
    dy = torch.randint(0, 2 * pad + 1, (N,))
    dx = torch.randint(0, 2 * pad + 1, (N,))
    flip = torch.rand(N) < 0.5
    for i in range(N):
        v = xp[i, :, dy[i]:dy[i] + H, dx[i]:dx[i] + W]
        out[i] = v.flip(-1) if flip[i] else v
    return out


class SyntheticLoader:
    """Class-conditional synthetic images of the real dataset's shape, generated on the
    device each step (GPU: Philox kernel; CPU: torch generator).  ``steps`` batches/epoch."""

    def __init__(self, shape, num_classes: int, batch_size: int, steps: int, device, seed: int = 1, rank: int = 0,
                 template_seed: int | None = None):
        """``template_seed`` (default ``seed``) fixes the class templates: a held-out set drawn with
        another ``seed`` but the training run's template seed comes from the same distribution."""
        self.shape, self.nc, self.batch_size, self.steps = tuple(shape), num_classes, batch_size, steps
        self.device = torch.device(device)
        self.seed = seed + 7919 * rank
        if template_seed is not None:
            seed = template_seed
        D = int(np.prod(shape))
        self.D = D
        if self.device.type == "cuda":
            C = native()
            st = torch.cuda.current_stream(self.device).cuda_stream
            self.tmpl = torch.empty(num_classes * D, device=self.device)
            C.synth_templates(self.tmpl.data_ptr(), num_classes, D, seed ^ 0x5EED, st)
            self.ctr = torch.zeros(4, dtype=torch.int32, device=self.device)
        else:
            g = torch.Generator().manual_seed(seed ^ 0x5EED)
            self.tmpl = torch.rand(num_classes, D, generator=g)
            self.gen = torch.Generator().manual_seed(self.seed)

    def __len__(self):
        return self.steps

    def state_dict(self) -> dict:
        """Stream position for resume (GPU: the Philox counter; CPU: the generator state)."""
        if self.device.type == "cuda":
            return {"counter": self.ctr.cpu().clone()}
        return {"gen_state": self.gen.get_state()}

    def load_state_dict(self, sd: dict):
        if self.device.type == "cuda" and "counter" in sd:
            self.ctr.copy_(sd["counter"].to(self.ctr.device))
        elif "gen_state" in sd:
            self.gen.set_state(sd["gen_state"])

    def __iter__(self):
        for _ in range(self.steps):
            if self.device.type == "cuda":
                x = torch.empty((self.batch_size,) + self.shape, device=self.device)
                y = torch.empty(self.batch_size, dtype=torch.int32, device=self.device)
                native().synth_batch(x.data_ptr(), y.data_ptr(), self.tmpl.data_ptr(), self.batch_size, self.D, self.nc,
                                     self.seed, self.ctr.data_ptr(), torch.cuda.current_stream(self.device).cuda_stream)
                yield x, y.long()
            else:
                y = torch.randint(0, self.nc, (self.batch_size,), generator=self.gen)
                noise = torch.rand(self.batch_size, self.D, generator=self.gen)
                x = 0.5 * self.tmpl[y] + 0.5 * noise
                yield x.view((self.batch_size,) + self.shape), y


DATASET_SIZES = {"mnist": 60000, "cifar10": 50000, "imagenet": 1281167}


def build_loader(dataset: str, data: str, root: str, batch_size: int, device, world_size: int, rank: int,
                 seed: int, shape, num_classes: int, train: bool = True, steps: int | None = None,
                 template_seed: int | None = None):
    """data: 'synthetic' | 'real' | 'auto' (real if files exist, else synthetic)."""
    if data in ("real", "auto"):
        try:
            if dataset == "mnist":
                x, y = load_mnist(root, train)
                mean, std, aug = MNIST_MEAN, MNIST_STD, False
            elif dataset == "cifar10":
                if cifar10_layout(root) is None:
                    raise FileNotFoundError(f"no CIFAR-10 (binary or python batches) under {root}")
                try:  # the dataset is on disk: an unreadable or incomplete copy is an error
                    x, y = load_cifar10_any(root, train)
                except (FileNotFoundError, KeyError) as e:
                    raise RuntimeError(f"CIFAR-10 under {root} is incomplete: {e}") from e
                mean, std, aug = CIFAR_MEAN, CIFAR_STD, train
            else:
                raise FileNotFoundError(f"no on-disk loader for {dataset}")
            sampler = ShardSampler(len(x), world_size, rank, shuffle=train, seed=seed)
            return TensorLoader(x, y, batch_size, device, sampler, mean, std, augment=aug, seed=seed + rank), "real"
        except FileNotFoundError as e:
            if data == "real":
                raise
            # nothing of the dataset on disk: synthetic, said on stderr as well as in the log
            # line (a dataset that IS on disk but unreadable raises above, never falls back)
            if rank == 0:
                print(f"mxddp: --data auto: {e}; training on SYNTHETIC {dataset} data", file=sys.stderr, flush=True)
    n = DATASET_SIZES.get(dataset, 50000)
    if steps is None:
        steps = math.ceil(math.ceil(n / world_size) / batch_size)
    return SyntheticLoader(shape, num_classes, batch_size, steps, device, seed, rank, template_seed), "synthetic"
