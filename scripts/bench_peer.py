"""Peer all-reduce microbenchmark: W ranks (processes).  On a 1-GPU box the ranks share the GPU
(a rehearsal: the exchange is HBM-local, so this prices the kernel's synchronisation and
memory traffic, not xGMI); on a multi-GPU node each rank gets its own GPU and RCCL is timed
alongside.

    python scripts/bench_peer.py --ws 2 --sizes 18816,1181066,6553600 --iters 50
"""
import argparse
import json
import os
import socket
import sys
import time

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def worker(rank, ws, port, a, q):
    import torch.distributed as dist

    from mxddp import native

    C = native()
    ndev = torch.cuda.device_count()
    dev = rank % ndev
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=ws)
    rccl = None
    if ndev >= ws:
        uid = [C.Comm.new_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, 0)
        rccl = C.Comm(uid[0], rank, ws, dev)
    res = {}
    for blocks, fence, one in [(b_, f_, o_) for b_ in a.blocks for f_ in a.fences for o_ in a.oneshot]:
        if True:
            pc = C.PeerComm(rank, ws, dev, 64 << 20, blocks)
            allh = [None] * ws
            dist.all_gather_object(allh, pc.handles())
            pc.open(allh)
            pc.set_fence(fence)
            pc.set_oneshot_bytes(one)
            st = torch.cuda.current_stream().cuda_stream
            for n in a.sizes:
                x = torch.randn(n, device="cuda")
                for _ in range(3):
                    pc.all_reduce(x.data_ptr(), n, C.DType.f32, st)
                torch.cuda.synchronize()
                dist.barrier()
                t0 = time.perf_counter()
                for _ in range(a.iters):
                    pc.all_reduce(x.data_ptr(), n, C.DType.f32, st)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / a.iters * 1e6
                t = torch.tensor([dt], dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                res[f"peer b={blocks} fence={fence} oneshot<={one} n={n}"] = round(float(t), 2)
            if pc.error():
                res["peer_error"] = pc.error()
            dist.barrier()
            del pc
    if rccl is not None:
        st = torch.cuda.current_stream().cuda_stream
        for n in a.sizes:
            x = torch.randn(n, device="cuda")
            for _ in range(3):
                rccl.all_reduce(x.data_ptr(), x.data_ptr(), n, C.DType.f32, C.RedOp.sum, st)
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                rccl.all_reduce(x.data_ptr(), x.data_ptr(), n, C.DType.f32, C.RedOp.sum, st)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.iters * 1e6
            t = torch.tensor([dt], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            res[f"rccl n={n}"] = round(float(t), 2)
    if rank == 0:
        q.put(res)
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ws", type=int, default=2)
    ap.add_argument("--sizes", type=lambda s: [int(v) for v in s.split(",")], default=[18816, 1181066, 6553600])
    ap.add_argument("--blocks", type=lambda s: [int(v) for v in s.split(",")], default=[64])
    ap.add_argument("--fences", type=lambda s: [int(v) for v in s.split(",")], default=[3])
    ap.add_argument("--oneshot", type=lambda s: [int(v) for v in s.split(",")], default=[262144],
                    help="one-shot kernel threshold(s) in bytes (0 = always two-shot)")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=worker, args=(r, a.ws, port, a, q)) for r in range(a.ws)]
    for p in ps:
        p.start()
    res = q.get(timeout=600)
    for p in ps:
        p.join(60)
    shared = torch.cuda.device_count() < a.ws
    print(json.dumps({"ws": a.ws, "shared_gpu": shared, "us_per_call": res}, indent=1))


if __name__ == "__main__":
    main()
