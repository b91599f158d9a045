"""Process-group bootstrap + the mxddp RCCL communicator.

Rendezvous (reference: ``dist.init_process_group(backend, init_method, world_size, rank)``
at pytorch/distributed_data_parallel.py:61-62):

* the torchrun env contract (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT)
  when set, otherwise the reference's explicit ``--init-method tcp://h:p --rank r
  --world-size w`` manual mode;
* the torch c10d ``TCPStore`` created by ``init_process_group`` is the control plane
  (barriers, object exchange, the ncclUniqueId hand-off);
* the data plane on GPU is OUR RCCL communicator (``mxddp._C.Comm``): rank 0 creates the
  ncclUniqueId, publishes it in the store, every rank calls ncclCommInitRank.  Collectives
  are issued from C++ on streams we own (reducer side stream, graph capture).
* on CPU the data plane is gloo through torch.distributed.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist

from .. import native


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    local_world_size: int = 1
    backend: str = "gloo"
    device: torch.device = torch.device("cpu")

    @property
    def is_main(self) -> bool:
        return self.rank == 0


_INFO: DistInfo | None = None
_COMM = None
_VARIANT_COMMS: dict = {}

# RCCL communicator variants sized for the 8x MI355X xGMI mesh: RCCL's own
# tuning, and the ring algorithm pinned with 7 / 14 / 28 channels (1 / 2 / 4 ring permutations
# per point-to-point link).  The autotuners time them against each other and against the direct
# peer transport on the machine they run on.  MXDDP_RCCL_VARIANTS overrides the list.
DEFAULT_RCCL_VARIANTS = "default,Ring:c7,Ring:c14,Ring:c28"


def parse_variant(name: str) -> dict:
    """'default' | '<algo>[/<proto>][:c<channels>]' -> Comm kwargs (ctas, algo, proto)."""
    if name in ("", "default"):
        return {"ctas": 0, "algo": "", "proto": ""}
    head, _, tail = name.partition(":")
    algo, _, proto = head.partition("/")
    ctas = 0
    if tail:
        if not (tail.startswith("c") and tail[1:].isdigit()):
            raise ValueError(f"RCCL variant {name!r}: channel spec must be c<N>")
        ctas = int(tail[1:])
    if algo.lower() in ("", "auto"):
        algo = ""
    return {"ctas": ctas, "algo": algo, "proto": proto}


def rccl_variants() -> list[str]:
    return [v.strip() for v in os.environ.get("MXDDP_RCCL_VARIANTS", DEFAULT_RCCL_VARIANTS).split(",") if v.strip()]


def env_dist() -> dict:
    """torchrun-style env contract (empty dict when not launched by a spawner).  Under SLURM
    (``srun python -m mxddp.train ...``, one task per GPU) the rank layout comes from
    SLURM_PROCID / SLURM_NTASKS / SLURM_LOCALID / SLURM_NTASKS_PER_NODE, and the rendezvous
    host from MASTER_ADDR or SLURM_LAUNCH_NODE_IPADDR (the reference claims SLURM support but
    ships none: README.md:11)."""
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        return {
            "rank": int(os.environ["RANK"]),
            "world_size": int(os.environ["WORLD_SIZE"]),
            "local_rank": int(os.environ.get("LOCAL_RANK", os.environ["RANK"])),
            "local_world_size": int(os.environ.get("LOCAL_WORLD_SIZE", os.environ["WORLD_SIZE"])),
        }
    if "SLURM_PROCID" in os.environ and "SLURM_NTASKS" in os.environ:
        ws = int(os.environ["SLURM_NTASKS"])
        if "MASTER_ADDR" not in os.environ and "SLURM_LAUNCH_NODE_IPADDR" in os.environ:
            os.environ["MASTER_ADDR"] = os.environ["SLURM_LAUNCH_NODE_IPADDR"]
        os.environ.setdefault("MASTER_PORT", str(29500 + int(os.environ.get("SLURM_JOB_ID", "0")) % 1000))
        return {
            "rank": int(os.environ["SLURM_PROCID"]),
            "world_size": ws,
            "local_rank": int(os.environ.get("SLURM_LOCALID", "0")),
            "local_world_size": slurm_tasks_per_node(ws),
        }
    return {}


def slurm_tasks_per_node(ws: int) -> int:
    """Ranks on THIS node under srun.  SLURM_NTASKS_PER_NODE exists only with --ntasks-per-node;
    SLURM_TASKS_PER_NODE is always set ("8(x2)" or "8,6" -- the first entry is this job's first
    node; nodes are normally filled evenly); else SLURM_NTASKS / SLURM_NNODES.  Never silently
    the global world size on a multi-node job (that would mark the ranks as sharing GPUs)."""
    for key in ("SLURM_NTASKS_PER_NODE", "SLURM_TASKS_PER_NODE"):
        v = os.environ.get(key, "").split("(")[0].split(",")[0].strip()
        if v.isdigit() and int(v) > 0:
            return int(v)
    nn = os.environ.get("SLURM_NNODES", os.environ.get("SLURM_JOB_NUM_NODES", ""))
    if nn.isdigit() and int(nn) > 0:
        return max(1, -(-ws // int(nn)))
    return ws


def init_distributed(backend: str | None = None, init_method: str | None = None, rank: int | None = None,
                     world_size: int | None = None, local_rank: int | None = None, use_gpu: bool | None = None,
                     timeout_s: float = 1800.0) -> DistInfo:
    """Initialise the process group (idempotent) and pick this rank's device."""
    global _INFO
    if _INFO is not None:
        return _INFO
    env = env_dist()
    rank = env.get("rank", rank if rank is not None else 0)
    world_size = env.get("world_size", world_size if world_size is not None else 1)
    local_rank = env.get("local_rank", local_rank if local_rank is not None else rank)
    lws = env.get("local_world_size", world_size)
    if use_gpu is None:
        use_gpu = torch.cuda.is_available()
    if backend is None:
        backend = "nccl" if use_gpu else "gloo"
    if backend not in ("nccl", "gloo"):
        raise RuntimeError(f"--dist-backend {backend!r}: nccl (= RCCL on MI355X) or gloo")
    if backend == "nccl" and not use_gpu:
        raise RuntimeError("--dist-backend nccl (RCCL) needs a GPU; use gloo for CPU runs")
    if use_gpu:
        ndev = torch.cuda.device_count()
        dev_index = local_rank % max(ndev, 1)
        torch.cuda.set_device(dev_index)
        device = torch.device("cuda", dev_index)
    else:
        device = torch.device("cpu")
    if world_size > 1 and not dist.is_initialized():
        if init_method is None and "MASTER_ADDR" in os.environ:
            init_method = "env://"
        if os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True" and init_method and init_method != "env://":
            # under torchrun every worker's tcp:// rendezvous becomes a CLIENT of the agent's store
            # at that address: a tcp:// URL other than the agent's (e.g. the reference default
            # tcp://127.0.0.1:13456) has no server and hangs; the agent's env contract is the truth
            init_method = "env://"
        # control plane always gloo (TCPStore + CPU collectives); RCCL data plane is ours.
        dist.init_process_group("gloo", init_method=init_method, world_size=world_size, rank=rank,
                                timeout=datetime.timedelta(seconds=timeout_s))
    _INFO = DistInfo(rank, world_size, local_rank, lws, backend, device)
    return _INFO


def info() -> DistInfo:
    return _INFO if _INFO is not None else DistInfo()


def rccl_comm(force: bool = False, variant: str = "default"):
    """This rank's RCCL communicator (created on first use; None when world_size == 1 unless
    ``force``: a 1-rank communicator exercises the full RCCL path for tests/benchmarks).
    ``variant`` (see parse_variant): another communicator over the same ranks built with a
    pinned algorithm / channel count; collective over all ranks, so every rank must ask for the
    same variants in the same order."""
    global _COMM
    if variant not in ("", "default"):
        base = rccl_comm(force)
        if base is None:
            return None
        if variant not in _VARIANT_COMMS:
            inf = info()
            C = native()
            kw = parse_variant(variant)
            if inf.world_size == 1:
                uid = C.Comm.new_unique_id()
            else:
                store = dist.distributed_c10d._get_default_store()
                key = f"mxddp/rccl_uid/{variant}"
                if inf.rank == 0:
                    store.set(key, C.Comm.new_unique_id())
                uid = store.get(key)
            _VARIANT_COMMS[variant] = C.Comm(uid, inf.rank, inf.world_size, inf.device.index, **kw)
        return _VARIANT_COMMS[variant]
    inf = info()
    if (inf.world_size == 1 and not force) or inf.device.type != "cuda":
        return None
    if inf.backend == "gloo" and not force:
        return None  # --dist-backend gloo: gradients go over gloo (parallel/ddp.py), not RCCL
    if inf.world_size > 1 and shared_devices():
        return None  # RCCL refuses several ranks on one GPU; such jobs use the peer transport
    if _COMM is None and inf.world_size == 1:
        C = native()
        _COMM = C.Comm(C.Comm.new_unique_id(), 0, 1, inf.device.index)
    if _COMM is None:
        C = native()
        store = dist.distributed_c10d._get_default_store()
        key = "mxddp/rccl_uid/0"
        if inf.rank == 0:
            store.set(key, C.Comm.new_unique_id())
        uid = store.get(key)
        _COMM = C.Comm(uid, inf.rank, inf.world_size, inf.device.index)
    return _COMM


def shared_devices() -> bool:
    """True when this node runs more ranks than it has GPUs (ranks share a device: a functional
    rehearsal of a multi-GPU job on a 1-GPU box).  RCCL cannot build a communicator then."""
    inf = info()
    n = torch.cuda.device_count()
    return inf.device.type == "cuda" and 0 < n < inf.local_world_size


def barrier():
    if dist.is_initialized():
        dist.barrier()


def rccl_version_str(code: int | None = None) -> str:
    """ncclGetVersion's code (major * 10000 + minor * 100 + patch) as 'major.minor.patch'."""
    if code is None:
        code = native().Comm.version()
    return f"{code // 10000}.{code // 100 % 100}.{code % 100}"


def rccl_diag(comm) -> dict:
    """What RCCL itself reports for `comm`, plus every rank's device (collective over the
    ranks when world_size > 1: a gloo all_gather).  The first multi-GPU run of a job names its
    own topology in the bench JSON: RCCL version, ncclCommCount (must equal the job's ranks),
    the variant / pinned channels, and which HIP device each rank drove."""
    inf = info()
    C = native()
    mine = {"rank": inf.rank, "device": inf.device.index if inf.device.type == "cuda" else None,
            "rccl_device": comm.hip_device if comm is not None else None,
            "host": os.uname().nodename}
    if inf.device.type == "cuda":
        props = torch.cuda.get_device_properties(inf.device)
        for k in ("pci_bus_id", "pci_device_id", "uuid"):
            v = getattr(props, k, None)
            if v is not None:
                mine[k] = str(v)
                break
    ranks = [mine]
    if dist.is_initialized() and inf.world_size > 1:
        ranks = [None] * inf.world_size
        dist.all_gather_object(ranks, mine)
    out = {"rccl_version": rccl_version_str(C.Comm.version()), "ranks": ranks}
    if comm is not None:
        out.update({"rccl_nranks": comm.nranks, "variant": comm.variant,
                    "channels": comm.ctas if comm.ctas > 0 else "rccl-tuned",
                    "init_timeout_s": C.Comm.init_timeout()})
    return out


def all_reduce_max(value: float) -> float:
    """Host-side max over ranks (used for timing: the bench takes the slowest rank)."""
    if not dist.is_initialized():
        return value
    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


_ALIGN_BUF: dict = {}


def device_align(stream, comm=None, peer=None) -> str:
    """Device-side start line of a timed region (bench.py): one tiny all-reduce enqueued on
    `stream` -- over `comm` (RCCL) when given, else over the peer transport -- so every rank's
    device leaves it at (nearly) the same moment, whatever the skew with which the ranks' hosts
    left the preceding host barrier.  A start event recorded on `stream` right after it is then
    a common start for all ranks.  Returns the transport used ("none" at world size 1)."""
    inf = info()
    if inf.world_size == 1 or inf.device.type != "cuda":
        return "none"
    buf = _ALIGN_BUF.get(inf.device)
    if buf is None:
        buf = _ALIGN_BUF[inf.device] = torch.zeros(64, dtype=torch.float32, device=inf.device)
    C = native()
    h = stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)
    if comm is not None:
        comm.all_reduce(buf.data_ptr(), buf.data_ptr(), buf.numel(), C.DType.f32, C.RedOp.sum, h)
        return "rccl"
    if peer is not None:
        peer.all_reduce(buf.data_ptr(), buf.numel(), C.DType.f32, h, C.RedOp.sum)
        return "peer"
    return "none"


def all_reduce_sum(values):
    if not dist.is_initialized():
        return list(values)
    t = torch.tensor(list(values), dtype=torch.float64)
    dist.all_reduce(t)
    return t.tolist()


def shutdown():
    global _INFO, _COMM
    from . import peer as _peer

    _peer.shutdown()
    _COMM = None
    _VARIANT_COMMS.clear()
    if dist.is_initialized():
        dist.destroy_process_group()
    _INFO = None
