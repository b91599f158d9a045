"""Launcher failure propagation + end-to-end CPU training through the CLI (BASELINE config 1,
and multi-process gloo DDP through the torchrun-style spawner)."""
import os
import re
import subprocess
import sys
import textwrap
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")


def test_launcher_propagates_first_failure(tmp_path):
    script = tmp_path / "w.py"
    script.write_text(textwrap.dedent("""
        import os, sys, time
        r = int(os.environ["RANK"])
        assert os.environ["WORLD_SIZE"] == "3" and os.environ["LOCAL_RANK"] == str(r)
        if r == 1:
            sys.exit(3)
        time.sleep(60)
    """))
    t0 = time.time()
    p = subprocess.run([sys.executable, "-m", "mxddp.launch", "--nproc-per-node", "3", str(script)], env=ENV,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 3, p.stderr
    assert time.time() - t0 < 40  # siblings were torn down, not waited for
    assert "a rank failed" in p.stderr


def test_launcher_success_and_ranks(tmp_path):
    script = tmp_path / "ok.py"
    out = tmp_path / "ranks"
    out.mkdir()
    script.write_text(textwrap.dedent(f"""
        import os
        open(os.path.join({str(out)!r}, os.environ["RANK"]), "w").write(os.environ["MASTER_PORT"])
    """))
    p = subprocess.run([sys.executable, "-m", "mxddp.launch", "--nproc-per-node", "4", str(script)], env=ENV,
                       timeout=120)
    assert p.returncode == 0
    assert sorted(os.listdir(out)) == ["0", "1", "2", "3"]
    assert len({open(out / f).read() for f in os.listdir(out)}) == 1


LINE = re.compile(r"^From Rank: (\d+), Epoch:\[(\d+)\]\[(\d+)/(\d+)\]\| loss: [\d.]+ \| acc: [\d.]+ \| batch time: [\d.]+s $")


def _train(args, tmp_path, timeout=600):
    cmd = [sys.executable, "-m", "mxddp.train", "--cpu", "--data", "synthetic", "-td", str(tmp_path / "td")] + args
    p = subprocess.run(cmd, env=ENV, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout + p.stderr
    return p.stdout


def test_train_cli_single_process_cpu(tmp_path):
    out = _train(["--model", "mnist_cnn", "--steps-per-epoch", "6", "-e", "2", "--log-interval", "3", "-sm",
                  "--lr", "0.01"], tmp_path)
    lines = [l for l in out.splitlines() if l.startswith("From Rank")]
    assert any(LINE.match(l) for l in lines), out
    assert "From Rank: 0, Training time" in out
    ck = tmp_path / "td" / "distributed_data_parallel_0.pth"
    sd = torch.load(ck, weights_only=True)
    assert "fc2.bias" in sd and sd["conv1.weight"].shape == (32, 1, 3, 3)


def test_train_cli_ddp_two_ranks_gloo(tmp_path):
    out = _train(["--model", "mlp", "--steps-per-epoch", "4", "-e", "1", "--log-interval", "2", "-sm",
                  "--nproc-per-node", "2", "-b", "32"], tmp_path)
    for r in (0, 1):
        assert os.path.exists(tmp_path / "td" / f"distributed_data_parallel_{r}.pth")
    a = torch.load(tmp_path / "td" / "distributed_data_parallel_0.pth", weights_only=True)
    b = torch.load(tmp_path / "td" / "distributed_data_parallel_1.pth", weights_only=True)
    for k in a:  # replicas stay bit-identical under DDP
        assert torch.equal(a[k], b[k]), k


def test_train_cli_replica_and_resume_cpu(tmp_path):
    _train(["--model", "keras_cnn", "--mode", "replica", "--steps-per-epoch", "3", "-e", "1", "-sm",
            "--save-every", "1"], tmp_path)
    assert os.path.exists(tmp_path / "td" / "data_parallel_model.pth")


def test_train_cli_resume(tmp_path):
    _train(["--model", "mnist_cnn", "--mode", "single", "--steps-per-epoch", "2", "-e", "1", "--save-every", "1"],
           tmp_path)
    st = tmp_path / "td" / "mxddp_state_0.pt"
    assert st.exists()
    out = _train(["--model", "mnist_cnn", "--mode", "single", "--steps-per-epoch", "2", "-e", "2", "--resume",
                  str(st), "-sm", "--eval"], tmp_path)
    assert "Epoch[2]" in out and "Test (synthetic)" in out
    assert (tmp_path / "td" / "single_gpu_model.pth").exists()
