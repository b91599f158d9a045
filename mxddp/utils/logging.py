"""Reference log-line formats (byte-for-byte) + a JSONL metrics stream (§5.5)."""
from __future__ import annotations

import datetime
import json
import os
import time


def ddp_step_line(rank, epoch, batch_idx, n_batches, loss, acc, batch_time) -> str:
    # pytorch/distributed_data_parallel.py:145-148
    return ('From Rank: {}, Epoch:[{}][{}/{}]| loss: {:.3f} | '
            'acc: {:.3f} | batch time: {:.3f}s '.format(rank, epoch, batch_idx, n_batches, loss, acc, batch_time))


def ddp_epoch_line(rank, seconds) -> str:
    # pytorch/distributed_data_parallel.py:150-152
    return "From Rank: {}, Training time {}".format(rank, datetime.timedelta(seconds=seconds))


def single_step_line(epoch, batch_idx, n_batches, loss, acc, batch_time) -> str:
    # pytorch/single_gpu.py:115-116
    return ('Epoch[{}]: [{}/{}]| loss: {:.3f} | acc: {:.3f} | batch time: {:.3f}s '
            .format(epoch, batch_idx, n_batches, loss, acc, batch_time))


def single_epoch_line(seconds) -> str:
    return "Training time {}".format(datetime.timedelta(seconds=seconds))


class MetricsWriter:
    """Append-only JSONL (one record per log interval / epoch) consumed by the benches."""

    def __init__(self, path: str | None):
        self.path = path
        if path and os.path.dirname(path):
            os.makedirs(os.path.dirname(path), exist_ok=True)
        self._f = open(path, "a") if path else None

    def write(self, **rec):
        if self._f is None:
            return
        rec.setdefault("ts", time.time())
        self._f.write(json.dumps(rec) + "\n")
        self._f.flush()

    def close(self):
        if self._f:
            self._f.close()
            self._f = None
