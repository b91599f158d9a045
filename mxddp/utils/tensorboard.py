"""TensorBoard event files without TensorFlow (the TF2 scripts' ``TensorBoard(log_dir=train_dir,
histogram_freq=1)`` callback, tensorflow2/mnist_single.py:67-76, tensorflow2/mnist_multi_worker_strategy.py:75-83).

Writes ``events.out.tfevents.<time>.<host>.mxddp`` in the TFRecord framing (little-endian
length, masked CRC32C of the length, the serialized ``Event`` proto, masked CRC32C of it) with
``Event`` / ``Summary`` / ``HistogramProto`` encoded by hand (field numbers of
tensorflow/core/util/event.proto and summary.proto), so the files open in a stock TensorBoard.
Scalars go in as ``simple_value``; ``add_histogram`` uses TensorBoard's default exponential
bucket edges.  Only rank 0 writes (the reference let every MultiWorker rank write into the
same directory: SURVEY §2.9 Q10).
"""
from __future__ import annotations

import os
import socket
import struct
import time

import numpy as np

# ----------------------------------------------------------------------------- CRC32C
_POLY = 0x82F63B78
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c = _TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def masked_crc32c(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ----------------------------------------------------------------------------- protobuf wire format
def _varint(v: int) -> bytes:
    out = bytearray()
    v &= (1 << 64) - 1
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wire: int) -> bytes:
    return _varint((field << 3) | wire)


def _f_double(field: int, v: float) -> bytes:
    return _key(field, 1) + struct.pack("<d", v)


def _f_float(field: int, v: float) -> bytes:
    return _key(field, 5) + struct.pack("<f", v)


def _f_int(field: int, v: int) -> bytes:
    return _key(field, 0) + _varint(v)


def _f_bytes(field: int, b: bytes) -> bytes:
    return _key(field, 2) + _varint(len(b)) + b


def _f_packed_doubles(field: int, vals) -> bytes:
    return _f_bytes(field, struct.pack(f"<{len(vals)}d", *vals))


def _default_edges() -> list[float]:
    """TensorBoard's default histogram bucket limits: +-1e-12 * 1.1^k up to 1e20."""
    pos, v = [], 1e-12
    while v < 1e20:
        pos.append(v)
        v *= 1.1
    return [-x for x in reversed(pos)] + [0.0] + pos + [float("inf")]


_EDGES = np.asarray(_default_edges())


def histogram_proto(values) -> bytes:
    v = np.asarray(values, dtype=np.float64).reshape(-1)
    # a diverged run (exactly when the histograms matter) has NaN / inf weights: NaNs are
    # dropped (TensorBoard has no bucket for them), +-inf land in the end buckets, and
    # min / max / sum are over the finite values so the proto stays well formed
    v = v[~np.isnan(v)]
    if v.size == 0:
        v = np.zeros(1)
    idx = np.minimum(np.searchsorted(_EDGES, v, side="left"), len(_EDGES) - 1)
    counts = np.bincount(idx, minlength=len(_EDGES)).astype(np.float64)
    fin = v[np.isfinite(v)]
    if fin.size == 0:
        fin = np.zeros(1)
    v_stats = fin
    nz = np.nonzero(counts)[0]
    lo, hi = (int(nz[0]), int(nz[-1]) + 1) if nz.size else (0, 1)
    return (_f_double(1, float(v_stats.min())) + _f_double(2, float(v_stats.max())) + _f_double(3, float(v.size)) +
            _f_double(4, float(v_stats.sum())) + _f_double(5, float((v_stats * v_stats).sum())) +
            _f_packed_doubles(6, _EDGES[lo:hi].tolist()) + _f_packed_doubles(7, counts[lo:hi].tolist()))


def _event(step: int, summary_values: list[bytes] | None = None, file_version: str | None = None,
           wall_time: float | None = None) -> bytes:
    ev = _f_double(1, time.time() if wall_time is None else wall_time) + _f_int(2, step)
    if file_version is not None:
        ev += _f_bytes(3, file_version.encode())
    if summary_values:
        ev += _f_bytes(5, b"".join(_f_bytes(1, v) for v in summary_values))
    return ev


def _record(data: bytes) -> bytes:
    hdr = struct.pack("<Q", len(data))
    return hdr + struct.pack("<I", masked_crc32c(hdr)) + data + struct.pack("<I", masked_crc32c(data))


class SummaryWriter:
    """Minimal ``tf.summary`` / ``torch.utils.tensorboard`` style writer (scalars + histograms)."""

    def __init__(self, logdir: str, enabled: bool = True):
        self.enabled = enabled
        self.path = None
        self._f = None
        if not enabled:
            return
        os.makedirs(logdir, exist_ok=True)
        self.path = os.path.join(logdir, f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}.mxddp")
        self._f = open(self.path, "wb")
        self._f.write(_record(_event(0, file_version="brain.Event:2")))
        self._f.flush()

    def add_scalar(self, tag: str, value: float, step: int):
        if self._f is None:
            return
        val = _f_bytes(1, tag.encode()) + _f_float(2, float(value))
        self._f.write(_record(_event(step, [val])))

    def add_histogram(self, tag: str, values, step: int):
        if self._f is None:
            return
        if hasattr(values, "detach"):
            values = values.detach().float().cpu().numpy()
        val = _f_bytes(1, tag.encode()) + _f_bytes(5, histogram_proto(values))
        self._f.write(_record(_event(step, [val])))

    def flush(self):
        if self._f is not None:
            self._f.flush()

    def close(self):
        if self._f is not None:
            self._f.close()
            self._f = None


class DeviceTrace:
    """The TF2 TensorBoard callback's ``profile_batch`` (tensorflow2/mnist_single.py:73 with TF's
    default profile_batch=2 [framework]): a host + device trace of one training batch, written where
    TensorBoard's profile plugin looks for it, ``<logdir>/plugins/profile/<run>/<host>.trace.json.gz``
    (Chrome trace format).  The device side comes from the ROCm tracer behind ``torch.profiler``:
    every HIP kernel of the step -- ours, RCCL's, graph replays included -- with its stream and
    duration.  ``batch`` counts from 1 in the first epoch, as in Keras; 0 = off."""

    def __init__(self, logdir: str, batch: int, enabled: bool = True):
        self.logdir, self.batch, self.enabled = logdir, int(batch), enabled and bool(logdir) and int(batch) > 0
        self.path = None
        self._prof = None
        self._done = False

    def wants(self, first_epoch: bool, bi_lo: int, n: int = 1) -> bool:
        """True if the step call covering batch indices [bi_lo, bi_lo + n) holds the traced batch."""
        return self.enabled and not self._done and first_epoch and bi_lo <= self.batch - 1 < bi_lo + n

    def start(self):
        import torch
        from torch.profiler import ProfilerActivity, profile

        acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if torch.cuda.is_available() else [])
        self._prof = profile(activities=acts)
        self._prof.__enter__()

    def stop(self):
        import gzip
        import shutil
        import tempfile

        import torch

        if self._prof is None:
            return None
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        self._prof.__exit__(None, None, None)
        run = time.strftime("%Y_%m_%d_%H_%M_%S")
        d = os.path.join(self.logdir, "plugins", "profile", run)
        os.makedirs(d, exist_ok=True)
        with tempfile.TemporaryDirectory() as td:
            raw = os.path.join(td, "trace.json")
            self._prof.export_chrome_trace(raw)
            self.path = os.path.join(d, f"{socket.gethostname()}.trace.json.gz")
            with open(raw, "rb") as fi, gzip.open(self.path, "wb") as fo:
                shutil.copyfileobj(fi, fo)
        self._prof = None
        self._done = True
        return self.path

    def around(self, first_epoch: bool, bi_lo: int, n: int = 1):
        """Context manager for one step call: traces it if it holds the profiled batch."""
        tr = self

        class _Ctx:
            def __enter__(self):
                self.on = tr.wants(first_epoch, bi_lo, n)
                if self.on:
                    tr.start()

            def __exit__(self, *exc):
                if self.on:
                    tr.stop()
                return False

        return _Ctx()


# ----------------------------------------------------------------------------- reader (tests / tools)
def _read_varint(b: bytes, i: int) -> tuple[int, int]:
    v, s = 0, 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << s
        s += 7
        if not c & 0x80:
            return v, i


def _fields(b: bytes) -> list[tuple[int, int, object]]:
    out, i = [], 0
    while i < len(b):
        k, i = _read_varint(b, i)
        f, w = k >> 3, k & 7
        if w == 0:
            v, i = _read_varint(b, i)
        elif w == 1:
            v = struct.unpack_from("<d", b, i)[0]
            i += 8
        elif w == 5:
            v = struct.unpack_from("<f", b, i)[0]
            i += 4
        elif w == 2:
            n, i = _read_varint(b, i)
            v = b[i:i + n]
            i += n
        else:
            raise ValueError(f"unsupported wire type {w}")
        out.append((f, w, v))
    return out


def read_events(path: str) -> list[dict]:
    """Parse an event file written by SummaryWriter (verifies both CRCs of every record)."""
    out = []
    with open(path, "rb") as f:
        data = f.read()
    i = 0
    while i < len(data):
        hdr = data[i:i + 8]
        (n,) = struct.unpack("<Q", hdr)
        if struct.unpack_from("<I", data, i + 8)[0] != masked_crc32c(hdr):
            raise ValueError("bad length crc")
        body = data[i + 12:i + 12 + n]
        if struct.unpack_from("<I", data, i + 12 + n)[0] != masked_crc32c(body):
            raise ValueError("bad data crc")
        i += 16 + n
        ev = {"values": []}
        for f, _, v in _fields(body):
            if f == 1:
                ev["wall_time"] = v
            elif f == 2:
                ev["step"] = v
            elif f == 3:
                ev["file_version"] = v.decode()
            elif f == 5:
                for sf, _, sv in _fields(v):
                    if sf != 1:
                        continue
                    rec = {}
                    for vf, _, vv in _fields(sv):
                        if vf == 1:
                            rec["tag"] = vv.decode()
                        elif vf == 2:
                            rec["simple_value"] = vv
                        elif vf == 5:
                            h = {}
                            for hf, _, hv in _fields(vv):
                                name = {1: "min", 2: "max", 3: "num", 4: "sum", 5: "sum_squares"}.get(hf)
                                if name:
                                    h[name] = hv
                                elif hf in (6, 7):
                                    arr = list(struct.unpack(f"<{len(hv) // 8}d", hv))
                                    h["bucket_limit" if hf == 6 else "bucket"] = arr
                            rec["histo"] = h
                    ev["values"].append(rec)
        out.append(ev)
    return out
