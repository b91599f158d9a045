"""T2: distributed semantics on CPU with gloo, world_size 2.

Golden equivalence: DDP at world_size N with per-rank batch b must equal single-process
training on the concatenated batch N*b (gradients averaged over ranks), and rank 0's
weights must win at wrap time.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from mxddp.models import build_model
from mxddp.parallel.ddp import assign_buckets


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batches(steps, global_b, shape, seed=123):
    g = torch.Generator().manual_seed(seed)
    return [(torch.rand((global_b,) + shape, generator=g), torch.randint(0, 10, (global_b,), generator=g))
            for _ in range(steps)]


def _worker(rank, ws, port, model_name, steps, b, q, perturb, comm_dtype="fp32"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from mxddp import ops
    from mxddp.optim import SGD
    from mxddp.parallel import comm
    from mxddp.parallel.ddp import DistributedDataParallel as DDP

    comm.init_distributed(rank=rank, world_size=ws, use_gpu=False, init_method=f"tcp://127.0.0.1:{port}")
    torch.manual_seed(0)
    model = build_model(model_name)
    if perturb and rank == 1:
        with torch.no_grad():
            for p in model.parameters():
                p.add_(1.0)
    ddp = DDP(model, grad_comm_dtype=comm_dtype)
    opt = SGD(ddp.flat, lr=0.05, momentum=0.9, weight_decay=1e-4)
    shape = model.input_shape
    for x, y in _batches(steps, ws * b, shape):
        xs, ys = x[rank * b:(rank + 1) * b], y[rank * b:(rank + 1) * b]
        opt.zero_grad()
        loss = ops.cross_entropy(ddp(xs), ys)
        loss.backward()
        opt.step()
    q.put((rank, {k: v.detach().numpy().copy() for k, v in model.state_dict().items()}, len(ddp.buckets)))
    comm.shutdown()


def _run_ddp(model_name, ws=2, steps=3, b=4, perturb=False, comm_dtype="fp32"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, ws, port, model_name, steps, b, q, perturb, comm_dtype))
          for r in range(ws)]
    for p in ps:
        p.start()
    out = {}
    for _ in range(ws):
        r, sd, nb = q.get(timeout=240)
        out[r] = ({k: torch.from_numpy(v) for k, v in sd.items()}, nb)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


@pytest.mark.parametrize("model_name", ["mnist_cnn", "mlp"])
def test_ddp_matches_single_process_large_batch(model_name):
    ws, steps, b = 2, 3, 4
    out = _run_ddp(model_name, ws, steps, b, perturb=True)
    # reference: plain torch, global batch, torch.optim.SGD
    torch.manual_seed(0)
    ref = build_model(model_name)
    opt = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    for x, y in _batches(steps, ws * b, ref.input_shape):
        opt.zero_grad()
        torch.nn.functional.cross_entropy(ref(x), y).backward()
        opt.step()
    ref_sd = ref.state_dict()
    for r in range(ws):
        sd = out[r][0]
        for k, v in ref_sd.items():
            assert torch.allclose(sd[k], v, rtol=1e-4, atol=1e-5), (r, k, (sd[k] - v).abs().max())
    # ranks identical to each other (rank-0 broadcast beat the perturbation on rank 1)
    for k in out[0][0]:
        assert torch.equal(out[0][0][k], out[1][0][k]), k


def test_ddp_bf16_gradient_communication():
    """--grad-comm-dtype bf16: buckets travel as bf16 (gloo here, RCCL / peer on GPUs) and come
    back into the fp32 gradient: the ranks stay identical and training matches the fp32-comm run
    within bf16 rounding of the gradients."""
    ref = _run_ddp("mlp", 2, 3, 4, comm_dtype="fp32")
    out = _run_ddp("mlp", 2, 3, 4, comm_dtype="bf16")
    for k in out[0][0]:
        assert torch.equal(out[0][0][k], out[1][0][k]), k
        a, b = out[0][0][k], ref[0][0][k]
        # lr 0.05 x bf16 relative rounding (2^-8) of gradients of O(1e-2): far below 1e-3
        assert (a - b).abs().max() < 1e-3, (k, (a - b).abs().max())
    moved = max((ref[0][0][k] - out[0][0][k]).abs().max().item() for k in out[0][0])
    assert moved > 0  # the bf16 path really ran (fp32 and bf16 results differ in the last bits)


def test_bucket_assignment_mnist_two_buckets():
    m = build_model("mnist_cnn")
    numels = [p.numel() for p in m.parameters()]
    offs, o = [], 0
    for n in numels:
        offs.append(o)
        o += (n + 15) // 16 * 16
    buckets, pb = assign_buckets(numels, offs, o)
    assert len(buckets) == 2  # 4.72 MB + 0.075 MB
    assert abs(buckets[0][1] * 4 / 1e6 - 4.72) < 0.01
    assert abs(buckets[1][1] * 4 / 1e6 - 0.075) < 0.002
    assert pb == [1, 1, 1, 1, 0, 0, 0, 0]
    # buckets tile the flat buffer contiguously from the end
    assert buckets[0][0] + buckets[0][1] == o and buckets[1][0] == 0 and buckets[1][1] == buckets[0][0]


def test_bucket_assignment_pyramidnet_five_buckets():
    m = build_model("pyramidnet110")
    numels = [p.numel() for p in m.parameters()]
    offs, o = [], 0
    for n in numels:
        offs.append(o)
        o += (n + 15) // 16 * 16
    buckets, _ = assign_buckets(numels, offs, o)
    mb = [n * 4 / 1e6 for _, n in buckets]
    # SURVEY §2.6 N4 (torch's own _compute_bucket_assignment_by_size): 2.66/28.10/26.47/26.66/13.12 MB
    expect = [2.66, 28.10, 26.47, 26.66, 13.12]
    assert len(mb) == 5
    for a, e in zip(mb, expect):
        assert abs(a - e) / e < 0.01, (mb, expect)


def test_gloo_reducer_rejects_double_mark():
    from mxddp.parallel.ddp import _GlooReducer

    r = _GlooReducer(torch.zeros(32), [(16, 16), (0, 16)], [1, 0], True, 1)
    r.mark_ready(0)
    with pytest.raises(RuntimeError):
        r.mark_ready(0)


def _uid_worker(rank, ws, port, q):
    """rccl_comm()'s rendezvous with the native communicator faked: every rank must receive rank
    0's ncclUniqueId bytes through the TCPStore and build its Comm with (uid, rank, ws, device)."""
    from mxddp.parallel import comm

    comm.init_distributed(rank=rank, world_size=ws, use_gpu=False, init_method=f"tcp://127.0.0.1:{port}")

    class FakeComm:
        @staticmethod
        def new_unique_id():
            return bytes(range(128)) if rank == 0 else b"wrong-rank-generated-id"

        def __init__(self, uid, r, w, dev):
            self.args = (bytes(uid), r, w, dev)

    class FakeNative:
        Comm = FakeComm

    orig_native, orig_info = comm.native, comm._INFO
    comm.native = lambda: FakeNative
    comm._INFO = comm.DistInfo(rank, ws, rank, ws, "nccl", torch.device("cuda", rank))
    try:
        c = comm.rccl_comm()
        q.put((rank, c.args[0] == bytes(range(128)), c.args[1:]))
    finally:
        comm.native, comm._INFO = orig_native, orig_info
        comm._COMM = None
        comm.shutdown()


def test_rccl_uid_rendezvous_ws4():
    ws, port = 4, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_uid_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(ws))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for r, (rank, same_uid, rest) in enumerate(res):
        assert rank == r and same_uid and rest == (r, ws, r), res


def _tiny_pyramidnet():
    from mxddp.models.pyramidnet import PyramidNet

    return PyramidNet(num_layers=3, alpha=24)  # 2 blocks per stage: BN, identity + stride-2 shortcuts


def _bn_worker(rank, ws, port, steps, b, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from mxddp import ops
    from mxddp.optim import SGD
    from mxddp.parallel import comm
    from mxddp.parallel.ddp import DistributedDataParallel as DDP

    comm.init_distributed(rank=rank, world_size=ws, use_gpu=False, init_method=f"tcp://127.0.0.1:{port}")
    torch.manual_seed(0)
    model = _tiny_pyramidnet()
    if rank == 1:  # rank-divergent weights AND buffers: the wrap-time broadcast must win
        with torch.no_grad():
            for p in model.parameters():
                p.add_(0.5)
            for n, bf in model.named_buffers():
                if bf.is_floating_point():
                    bf.add_(3.0)
    ddp = DDP(model, bucket_cap_mb=0.02, first_bucket_cap_mb=0.01)  # several buckets
    opt = SGD(ddp.flat, lr=0.05, momentum=0.9, weight_decay=1e-4)
    for x, y in _batches(steps, ws * b, (3, 32, 32), seed=77):
        opt.zero_grad()
        ops.cross_entropy(ddp(x[rank * b:(rank + 1) * b]), y[rank * b:(rank + 1) * b]).backward()
        opt.step()
    q.put((rank, {k: v.detach().numpy().copy() for k, v in model.state_dict().items()}, len(ddp.buckets)))
    comm.shutdown()


def test_ddp_batchnorm_model_matches_simulated_ranks():
    """DDP semantics for a BatchNorm model (PyramidNet blocks): every rank normalises with its OWN
    shard's batch statistics, gradients are averaged, and rank 0's floating buffers (running
    mean / var) are broadcast before every forward (broadcast_buffers=True,
    pytorch/distributed_data_parallel.py:74).  Golden reference: one process, plain torch, one
    model copy per rank -- copy rank 0's buffers to the others, forward / backward every copy on
    its shard, average the gradients, identical torch.optim.SGD steps."""
    import copy

    import torch.nn.functional as F

    ws, steps, b = 2, 3, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_bn_worker, args=(r, ws, port, steps, b, q)) for r in range(ws)]
    for p in ps:
        p.start()
    out = {}
    for _ in range(ws):
        r, sd, nb = q.get(timeout=240)
        out[r] = {k: torch.from_numpy(v) for k, v in sd.items()}
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert nb >= 3

    torch.manual_seed(0)
    base = _tiny_pyramidnet()
    copies = [copy.deepcopy(base) for _ in range(ws)]
    params = [list(c.parameters()) for c in copies]
    opts = [torch.optim.SGD(c.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4) for c in copies]
    with torch.no_grad():
        for x, y in _batches(steps, ws * b, (3, 32, 32), seed=77):
            for c in copies[1:]:  # per-forward buffer broadcast from rank 0
                for (n, dst), src in zip(c.named_buffers(), copies[0].buffers()):
                    if dst.is_floating_point():
                        dst.copy_(src)
            grads = []
            for r, c in enumerate(copies):
                c.zero_grad()
                with torch.enable_grad():
                    F.cross_entropy(c(x[r * b:(r + 1) * b]), y[r * b:(r + 1) * b]).backward()
                grads.append([p.grad.clone() for p in c.parameters()])
            avg = [sum(gs) / ws for gs in zip(*grads)]
            for r in range(ws):
                for p, g in zip(params[r], avg):
                    p.grad.copy_(g)
                opts[r].step()
    for r in range(ws):
        ref = copies[r].state_dict()
        for k, v in ref.items():
            got = out[r][k]
            if v.is_floating_point():
                assert torch.allclose(got, v, rtol=1e-4, atol=1e-5), (r, k, (got - v).abs().max())
            else:
                assert torch.equal(got, v), (r, k, got, v)  # num_batches_tracked == steps
    assert int(out[0]["bn1.num_batches_tracked"]) == steps
    # parameters identical across ranks; running stats differ (each rank's own last shard)
    for k in out[0]:
        if k.endswith("weight") or k.endswith("bias"):
            assert torch.equal(out[0][k], out[1][k]), k
    assert not torch.equal(out[0]["bn1.running_mean"], out[1]["bn1.running_mean"])


def _abort_worker(rank, ws, port, fail, q):
    """Three DDP steps of the MNIST CNN; with `fail`, an extra step in the middle whose backward
    raises on every rank after the fc bucket's all-reduce was launched (a hook on conv2's output
    gradient runs after fc1 / fc2 have their gradients)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    from mxddp import ops
    from mxddp.optim import SGD
    from mxddp.parallel import comm
    from mxddp.parallel.ddp import DistributedDataParallel as DDP

    comm.init_distributed(rank=rank, world_size=ws, use_gpu=False, init_method=f"tcp://127.0.0.1:{port}")
    torch.manual_seed(0)
    model = build_model("mnist_cnn")
    ddp = DDP(model)
    opt = SGD(ddp.flat, lr=0.05, momentum=0.9, weight_decay=1e-4)
    b = 4
    batches = _batches(3, ws * b, model.input_shape)
    armed = {"on": False}

    def boom(g):
        if armed["on"]:
            raise RuntimeError("injected backward failure")
        return g

    def attach(_m, _i, o):  # (returns None: a forward hook's return value would replace the output)
        if o.requires_grad:
            o.register_hook(boom)

    handle = model.conv2.register_forward_hook(attach)
    launched = None
    for i, (x, y) in enumerate(batches):
        if fail and i == 1:
            armed["on"] = True
            opt.zero_grad()
            try:
                ops.cross_entropy(ddp(x[rank * b:(rank + 1) * b]), y[rank * b:(rank + 1) * b]).backward()
            except RuntimeError as e:
                assert "injected" in str(e)
                launched = len(ddp.reducer.works)
            armed["on"] = False
        opt.zero_grad()
        ops.cross_entropy(ddp(x[rank * b:(rank + 1) * b]), y[rank * b:(rank + 1) * b]).backward()
        opt.step()
    handle.remove()
    q.put((rank, launched, {k: v.detach().numpy().copy() for k, v in model.state_dict().items()}))
    comm.shutdown()


def test_ddp_recovers_from_backward_that_raised_on_every_rank():
    """Reducer.abort (ddp.py forward): a backward that raised after its first bucket's all-reduce
    was launched leaves that step's reducer state behind; the next forward joins the launched
    all-reduces (they write the gradient buffer in place) and drops the step, so training goes on
    exactly as if the failed step had never run -- on every rank."""
    ctx = mp.get_context("spawn")
    res = {}
    for fail in (False, True):
        q = ctx.Queue()
        port = _free_port()
        ps = [ctx.Process(target=_abort_worker, args=(r, 2, port, fail, q)) for r in range(2)]
        for p in ps:
            p.start()
        out = {}
        for _ in range(2):
            r, launched, sd = q.get(timeout=240)
            out[r] = (launched, sd)
        for p in ps:
            p.join(timeout=60)
            assert p.exitcode == 0
        res[fail] = out
    for r in range(2):
        assert res[True][r][0] == 1  # the fc bucket's all-reduce was in flight when it raised
        for k, v in res[False][r][1].items():
            assert (res[True][r][1][k] == v).all(), (r, k)
