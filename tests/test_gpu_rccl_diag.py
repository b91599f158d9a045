"""Self-diagnosis of the multi-GPU path on one GPU: the bench JSON names
RCCL's version, ncclCommCount, the variant and each rank's device and the exposed comm time
(collectives forced at one rank, so the RCCL path runs), an RCCL init whose peer never joins
ends the process with the deadline's exit code instead of hanging, and the reducer's dry mode
issues no collective.  Reference: pytorch/distributed_data_parallel.py:61-62,74,132."""
import json
import os
import subprocess
import sys
import time

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=240, env=None):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


def test_bench_reports_rccl_and_exposed_comm_forced_ws1(cuda):
    out = _bench("--steps", "20", "--warmup", "5", "--force-collectives")
    rc = out["rccl"]
    from mxddp import native
    from mxddp.parallel.comm import rccl_version_str

    assert rc["rccl_version"] == rccl_version_str(native().Comm.version())
    assert rc["rccl_nranks"] == out["n_gpus"] == 1
    assert rc["variant"] and rc["channels"]
    assert [r["rank"] for r in rc["ranks"]] == [0] and rc["ranks"][0]["device"] == 0
    assert rc["ranks"][0]["rccl_device"] == 0
    assert rc["init_timeout_s"] > 0
    dry, exp = out["compute_only_ms_per_step"], out["exposed_comm_ms_per_step"]
    assert 0 < dry and abs(dry + exp - out["ms_per_step"]) < 1e-3 * max(1.0, out["ms_per_step"])
    # a 1-rank all-reduce is cheap but never negative by much (same graph, collectives removed)
    assert exp > -0.25 * out["ms_per_step"], out
    # the training metrics are read before the diagnosis pass, whose steps are not training steps
    # (read after it, train_acc came out above 1 in the 2-rank runs)
    assert 0.0 <= out["train_acc"] <= 1.0 and out["train_images"] > 0, out


def test_bench_headline_has_no_rccl_fields(cuda):
    """ws = 1 without forced collectives: no communicator, no diagnosis pass (the headline's
    timed region and JSON are unchanged)."""
    out = _bench("--steps", "20", "--warmup", "5")
    assert "rccl" not in out and "exposed_comm_ms_per_step" not in out


def test_rccl_init_with_absent_peer_exits_within_deadline(cuda):
    """Rank 0 of a 2-rank communicator whose rank 1 never joins: the init deadline ends the
    process with Comm.INIT_TIMEOUT_EXIT and names the rank / variant, instead of blocking."""
    from mxddp import native

    code = ("import mxddp; C = mxddp.native(); uid = C.Comm.new_unique_id(); "
            "C.Comm(uid, 0, 2, 0); print('init returned')")
    env = dict(os.environ, MXDDP_RCCL_INIT_TIMEOUT_S="6")
    t0 = time.perf_counter()
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=90, cwd=ROOT, env=env)
    dt = time.perf_counter() - t0
    assert r.returncode == native().Comm.INIT_TIMEOUT_EXIT, (r.returncode, r.stderr[-2000:])
    assert "did not complete within 6 s" in r.stderr and "rank 0 of 2" in r.stderr and "variant 'default'" in r.stderr
    assert "init returned" not in r.stdout
    assert dt < 60, dt


def test_dry_collectives_issue_no_collective(cuda):
    """compute_only_ms (the bench's dry pass) leaves the trainer as it found it: the flag is
    off again and the recaptured step still trains exactly like an engine that never ran a dry
    pass (over one rank the exchange is the identity, so the dry steps are ordinary steps)."""
    from mxddp import native
    from mxddp.engine import FusedMnistTrainer

    C = native()
    comm = C.Comm(C.Comm.new_unique_id(), 0, 1, cuda.index or 0)
    a = FusedMnistTrainer(batch=32, device=cuda, lr=0.01, comm=comm, force_collectives=True, graph_mode=1)
    b = FusedMnistTrainer(batch=32, device=cuda, lr=0.01, comm=comm, force_collectives=True, graph_mode=1)
    a.step(3)
    b.step(3)
    ms = b.compute_only_ms(5)  # dry pass: its graphs' warm launches + 2 + 5 steps, then recaptured
    assert ms is not None and ms > 0 and not C.dry_collectives()
    n = b.discarded_steps
    assert n >= 7
    a.step(n)
    torch.cuda.synchronize()
    for k, v in a.state_dict().items():
        assert torch.equal(v, b.state_dict()[k]), k  # 1 rank: identical with or without the exchange
