"""Single-node torchrun-style spawner.

Replaces the reference's process fan-out -- ``mp.spawn(main_worker, nprocs=device_count)``
with every child passing the SAME ``--rank`` (pytorch/distributed_data_parallel.py:54-62,
SURVEY §2.9 Q1: deadlocks / duplicate ranks with >1 visible GPU), the manual
one-shell-per-rank recipe (pytorch/README.md:71-113), ``TF_CONFIG`` and ``mpiexec`` -- with one
launcher that:

* computes correct global ranks ``node_rank * nproc_per_node + local_rank``;
* exports the torchrun env contract (RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE,
  MASTER_ADDR, MASTER_PORT, plus HSA_ENABLE_IPC_MODE_LEGACY=0 for dmabuf IPC);
* starts each rank as a child process (never exec from a GPU-initialised process);
* monitors the children, and on the first non-zero exit terminates the others and
  returns that exit code (failure propagation); an optional wall-clock timeout bounds
  hung jobs.

Usage::

    python -m mxddp.launch --nproc-per-node 8 [--nnodes 1 --node-rank 0
        --master-addr 127.0.0.1 --master-port 29500] (-m module | script.py) [args...]
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time


def free_port(addr: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((addr, 0))
        return s.getsockname()[1]


def launch(cmd: list[str], nproc_per_node: int, nnodes: int = 1, node_rank: int = 0,
           master_addr: str = "127.0.0.1", master_port: int | None = None, timeout_s: float | None = None,
           grace_s: float = 10.0, extra_env: dict | None = None) -> int:
    master_port = master_port or free_port(master_addr)
    world = nnodes * nproc_per_node
    procs: list[subprocess.Popen] = []
    for lr in range(nproc_per_node):
        env = dict(os.environ)
        env.update({
            "RANK": str(node_rank * nproc_per_node + lr),
            "LOCAL_RANK": str(lr),
            "WORLD_SIZE": str(world),
            "LOCAL_WORLD_SIZE": str(nproc_per_node),
            "GROUP_RANK": str(node_rank),
            "MASTER_ADDR": master_addr,
            "MASTER_PORT": str(master_port),
            "HSA_ENABLE_IPC_MODE_LEGACY": "0",
        })
        if extra_env:
            env.update(extra_env)
        procs.append(subprocess.Popen(cmd, env=env, start_new_session=True))
    t0 = time.time()
    rc = 0
    try:
        while True:
            alive = 0
            for p in procs:
                r = p.poll()
                if r is None:
                    alive += 1
                elif r != 0 and rc == 0:
                    rc = r
            if rc != 0 or alive == 0:
                break
            if timeout_s and time.time() - t0 > timeout_s:
                print(f"[mxddp.launch] timeout after {timeout_s}s; terminating ranks", file=sys.stderr)
                rc = 124
                break
            time.sleep(0.05)
    except KeyboardInterrupt:
        rc = 130
    if rc != 0:
        _terminate(procs, grace_s)
        print(f"[mxddp.launch] a rank failed (exit {rc}); all ranks stopped", file=sys.stderr)
    else:
        for p in procs:
            p.wait()
    return rc


def _terminate(procs, grace_s):
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)  # each child leads its own process group
            except ProcessLookupError:
                pass
    deadline = time.time() + grace_s
    for p in procs:
        while p.poll() is None and time.time() < deadline:
            time.sleep(0.05)
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait()


def spawn_self(nproc: int, argv: list[str], module: str) -> int:
    """Used by ``mxddp.train --nproc-per-node N``: re-launch this module N times."""
    args = [a for a in argv]
    # strip --nproc-per-node from the children's argv
    out, skip = [], False
    for a in args:
        if skip:
            skip = False
            continue
        if a == "--nproc-per-node":
            skip = True
            continue
        if a.startswith("--nproc-per-node="):
            continue
        out.append(a)
    return launch([sys.executable, "-m", module] + out, nproc)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="mxddp single-node multi-rank launcher")
    ap.add_argument("--nproc-per-node", "--nproc_per_node", type=int, default=1)
    ap.add_argument("--nnodes", type=int, default=1)
    ap.add_argument("--node-rank", "--node_rank", type=int, default=0)
    ap.add_argument("--master-addr", "--master_addr", default="127.0.0.1")
    ap.add_argument("--master-port", "--master_port", type=int, default=None)
    ap.add_argument("--timeout", type=float, default=None, help="kill the job after this many seconds")
    ap.add_argument("-m", dest="module", default=None, help="run a module (like python -m)")
    ap.add_argument("script_and_args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    rest = a.script_and_args
    if a.module:
        cmd = [sys.executable, "-m", a.module] + rest
    else:
        if not rest:
            ap.error("need a script or -m module")
        cmd = [sys.executable] + rest
    return launch(cmd, a.nproc_per_node, a.nnodes, a.node_rank, a.master_addr, a.master_port, a.timeout)


if __name__ == "__main__":
    sys.exit(main())
