"""Diagnostic: fused MNIST DDP step over the peer transport, 2 ranks on one GPU, against the
PyTorch CPU reference on the global batch.  Variants: overlap on/off, same / split batch."""
import os
import socket
import sys

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def ref_params(init, batches, lr):
    import torch.nn.functional as F

    from mxddp.models import MnistCNN

    m = MnistCNN()
    m.load_state_dict(init.state_dict())
    opt = torch.optim.SGD(m.parameters(), lr=lr, momentum=0.9, weight_decay=1e-4)
    for x, y in batches:
        opt.zero_grad()
        F.cross_entropy(m(x), y).backward()
        opt.step()
    return torch.cat([v.detach().reshape(-1) for v in m.state_dict().values()])


def worker(rank, ws, port, q):
    import torch.distributed as dist

    from mxddp import native
    from mxddp.engine import FusedMnistTrainer
    from mxddp.models import MnistCNN

    C = native()
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=ws)
    pc = C.PeerComm(rank, ws, 0, 8 << 20, 16)
    allh = [None] * ws
    dist.all_gather_object(allh, pc.handles())
    pc.open(allh)
    b, steps, lr = 16, 3, 0.05
    torch.manual_seed(0)
    init = MnistCNN()
    g = torch.Generator().manual_seed(5)
    batches = [(torch.rand(ws * b, 1, 28, 28, generator=g), torch.randint(0, 10, (ws * b,), generator=g))
               for _ in range(steps)]
    res = {}
    # calibration: one process, no transport, global batch
    solo = FusedMnistTrainer(batch=ws * b, device=0, comm=None, lr=lr, init_model=init, use_graph=False)
    for x, y in batches:
        solo.set_batch(x.cuda(), y.cuda())
        solo.step(1)
    solo.synchronize()
    w_ = ref_params(init, batches, lr)
    i0 = torch.cat([v.detach().reshape(-1) for v in init.state_dict().values()])
    res["solo"] = [round((solo.params.cpu() - w_).abs().max().item(), 7), solo.params.cpu()[18816:18819].tolist(),
                   w_[18816:18819].tolist(), i0[18816:18819].tolist()]
    solo2 = FusedMnistTrainer(batch=ws * b, device=0, comm=None, lr=lr, init_model=init, use_graph=False)
    for x, y in batches:
        solo2.set_batch(x.cuda(), y.cuda())
        solo2.step(1)
    solo2.synchronize()
    res["solo2"] = [round((solo2.params.cpu() - w_).abs().max().item(), 7), solo2.params.cpu()[18816:18819].tolist()]
    os.environ["MXDDP_POISON_WORKSPACE"] = "1"
    solo3 = FusedMnistTrainer(batch=ws * b, device=0, comm=None, lr=lr, init_model=init, use_graph=False)
    for x, y in batches:
        solo3.set_batch(x.cuda(), y.cuda())
        solo3.step(1)
    solo3.synchronize()
    del os.environ["MXDDP_POISON_WORKSPACE"]
    d3 = (solo3.params.cpu() - w_).abs()
    off, per = 0, {}
    for k, v in init.state_dict().items():
        per[k] = d3[off:off + v.numel()].max().item()
        off += v.numel()
    res["solo3_poisoned"] = per
    for same in (True, False):
        for ov in (True, False):
            tr = FusedMnistTrainer(batch=b, device=0, comm=None, peer=pc, lr=lr, init_model=init, use_graph=False)
            tr.eng.set_overlap(ov)
            used = []
            for x, y in batches:
                xs, ys = (x[:b], y[:b]) if same else (x[rank * b:(rank + 1) * b], y[rank * b:(rank + 1) * b])
                used.append((x[:b], y[:b]) if same else (x, y))
                tr.set_batch(xs.cuda(), ys.cuda())
                tr.step(1)
            tr.synchronize()
            want = ref_params(init, used, lr)
            got = tr.params.cpu()
            d = (got - want).abs()
            # per-tensor max error
            off, per = 0, {}
            for k, v in init.state_dict().items():
                n = v.numel()
                per[k] = round(d[off:off + n].max().item(), 7)
                off += n
            i0 = torch.cat([v.detach().reshape(-1) for v in init.state_dict().values()])
            per["|got-init|"] = round((got - i0).abs().max().item(), 6)
            per["|want-init|"] = round((want - i0).abs().max().item(), 6)
            res[f"same={same} ovl={ov}"] = per
            dist.barrier()
    q.put((rank, res, pc.error()))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    for _ in ps:
        r, res, err = q.get(timeout=300)
        print("rank", r, "peer err", err)
        for k, v in res.items():
            print("  ", k, v)
    for p in ps:
        p.join()
