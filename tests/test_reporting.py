"""CPU: trainer-extension parity -- TensorBoard event files (TF2 TensorBoard callback), Chainer
LogReport / PrintReport / dump_graph, Keras model.summary() -- and their CLI wiring through the
reference scripts' compat entry points (tensorflow2/mnist_single.py, chainer/train_mnist.py)."""
import json
import os
import subprocess
import sys

import numpy as np
import torch

from mxddp.utils import report, tensorboard

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")


def test_crc32c_known_vectors():
    assert tensorboard.crc32c(b"123456789") == 0xE3069283
    assert tensorboard.crc32c(b"") == 0


def test_event_file_roundtrip(tmp_path):
    w = tensorboard.SummaryWriter(str(tmp_path))
    w.add_scalar("epoch_loss", 0.5, 1)
    w.add_scalar("epoch_loss", 0.25, 2)
    vals = np.random.default_rng(0).standard_normal(1000)
    w.add_histogram("fc1.weight", torch.from_numpy(vals), 2)
    w.close()
    ev = tensorboard.read_events(w.path)  # checks both CRCs of every record
    assert ev[0]["file_version"] == "brain.Event:2"
    scal = [(e["step"], v["simple_value"]) for e in ev for v in e["values"] if "simple_value" in v]
    assert scal == [(1, 0.5), (2, 0.25)]
    h = [v["histo"] for e in ev for v in e["values"] if "histo" in v][0]
    assert h["num"] == 1000 and sum(h["bucket"]) == 1000
    v32 = vals.astype(np.float32).astype(np.float64)  # tensors are histogrammed as float32
    assert abs(h["sum"] - v32.sum()) < 1e-9 and h["min"] == v32.min() and h["max"] == v32.max()
    assert len(h["bucket"]) == len(h["bucket_limit"])
    # every value lies under its bucket's upper limit and above the previous one
    lim = h["bucket_limit"]
    assert all(a < b for a, b in zip(lim, lim[1:]))


def test_log_and_print_report(tmp_path):
    lines = []
    lr = report.LogReport(str(tmp_path))
    pr = report.PrintReport(out=lines.append)
    for ep in (1, 2):
        e = {"epoch": ep, "iteration": 10 * ep, "main/loss": 1.0 / ep, "main/accuracy": 0.5,
             "validation/main/loss": 0.9 / ep, "validation/main/accuracy": 0.6, "elapsed_time": 1.5 * ep}
        lr.append(e)
        pr(e)
    log = json.load(open(tmp_path / "log"))
    assert [x["epoch"] for x in log] == [1, 2] and log[1]["main/loss"] == 0.5
    assert lines[0].split() == report.PRINT_COLUMNS and len(lines) == 3
    assert lines[2].split()[0] == "2"


def test_dump_graph_and_summary(tmp_path):
    from mxddp import ops
    from mxddp.models import build_model

    m = build_model("keras_cnn")
    loss = ops.cross_entropy(m(torch.rand(2, 1, 28, 28)), torch.tensor([1, 2]))
    n = report.dump_graph(loss, str(tmp_path / "cg.dot"), dict(m.named_parameters()))
    dot = open(tmp_path / "cg.dot").read()
    assert dot.startswith("digraph") and "main/loss" in dot and n > 10
    for name, _ in m.named_parameters():
        assert name in dot, name
    s = report.model_summary(m, (1, 28, 28), "keras_cnn")
    assert "Total params: 93,322" in s and "(None, 10)" in s


def _run(args, cwd):
    p = subprocess.run([sys.executable] + args, env=ENV, cwd=cwd, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout + p.stderr
    return p.stdout


def test_tf2_script_writes_tensorboard_and_summary(tmp_path):
    out = _run([os.path.join(ROOT, "examples/tensorflow2/mnist_single.py"), "-e", "1", "-b", "32",
                "--train_dir", str(tmp_path / "td"), "--dataset_dir", str(tmp_path / "none")], str(tmp_path))
    assert "Total params: 93,322" in out
    files = [f for f in os.listdir(tmp_path / "td") if f.startswith("events.out.tfevents")]
    assert len(files) == 1
    ev = tensorboard.read_events(str(tmp_path / "td" / files[0]))
    tags = {v["tag"] for e in ev for v in e["values"]}
    assert {"epoch_loss", "epoch_accuracy", "epoch_val_loss", "conv1.weight"} <= tags
    assert (tmp_path / "td" / "ckpt_1.pth").exists() and "restored ckpt_1.pth" in out
    sd = torch.load(tmp_path / "td" / "ckpt_1.pth", weights_only=True)
    assert sum(v.numel() for v in sd.values()) == 93_322
    # TensorBoard profile_batch=2: one trace of batch 2 where the profile plugin looks for it
    import glob
    import gzip

    traces = glob.glob(str(tmp_path / "td" / "plugins" / "profile" / "*" / "*.trace.json.gz"))
    assert len(traces) == 1, traces
    tr = json.loads(gzip.open(traces[0]).read())
    assert len(tr["traceEvents"]) > 0


def test_chainer_script_writes_log_report_and_graph(tmp_path):
    out = _run([os.path.join(ROOT, "examples/chainer/train_mnist.py"), "--gpu", "-1", "-e", "2", "-b", "100",
                "--unit", "50", "--out", str(tmp_path / "result"), "--dataset-dir", str(tmp_path / "none")],
               str(tmp_path))
    log = json.load(open(tmp_path / "result" / "log"))
    assert [e["epoch"] for e in log] == [1, 2] and "validation/main/accuracy" in log[0]
    assert (tmp_path / "result" / "cg.dot").exists()
    assert "main/loss" in out and "validation/main/accuracy" in out  # PrintReport header


def test_histogram_proto_nonfinite_values():
    """A diverged run's weights (NaN / inf) still give a well-formed HistogramProto: as many
    bucket limits as counts, finite min / max / sum."""
    import math
    import struct

    import numpy as np

    from mxddp.utils.tensorboard import histogram_proto

    raw = histogram_proto(np.array([1.0, float("nan"), -2.0, float("inf"), float("-inf"), 0.5]))
    fields, i = {}, 0
    while i < len(raw):  # minimal protobuf walk: field 1-5 doubles, 6-7 packed doubles
        key = raw[i]
        i += 1
        f, wt = key >> 3, key & 7
        if wt == 1:
            fields[f] = struct.unpack("<d", raw[i:i + 8])[0]
            i += 8
        else:
            n, shift = 0, 0
            while True:
                b = raw[i]
                i += 1
                n |= (b & 0x7F) << shift
                shift += 7
                if not b & 0x80:
                    break
            fields[f] = struct.unpack(f"<{n // 8}d", raw[i:i + n])
            i += n
    assert len(fields[6]) == len(fields[7])
    assert fields[1] == -2.0 and fields[2] == 1.0 and math.isfinite(fields[4])
    assert sum(fields[7]) == 5  # the NaN is dropped, both infinities counted
