"""Diagnostic: layer-path DDP at 2 ranks sharing one GPU (peer transport), eager vs whole-step graph.
Prints, per step, each rank's parameter checksum and the peer transport's error word; at the end
whether the ranks' weights are identical.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
        scripts/diag_ddp_graph.py --model keras_cnn --steps 20 [--graph] [--overlap 0|1] [--opt adam|sgd]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from mxddp import ops  # noqa: E402
from mxddp.data import SyntheticLoader  # noqa: E402
from mxddp.models import build_model, get_spec  # noqa: E402
from mxddp.optim import SGD, Adam  # noqa: E402
from mxddp.parallel import comm as PC  # noqa: E402
from mxddp.parallel import peer as PP  # noqa: E402
from mxddp.parallel.ddp import DistributedDataParallel as DDP  # noqa: E402
from mxddp.parallel.graphed import GraphedStep  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="keras_cnn")
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--graph", action="store_true")
ap.add_argument("--overlap", type=int, default=1)
ap.add_argument("--opt", default="adam")
ap.add_argument("--loader", default="synthetic", choices=["synthetic", "fixed"])
ap.add_argument("--mimic", action="store_true", help="step body as in mxddp.train (correct count, events, check)")
ap.add_argument("--parts", default="corr,ev,check", help="--mimic parts: corr (return_correct), ev (events), check")
a = ap.parse_args()
parts = set(a.parts.split(",")) if a.mimic else set()

inf = PC.init_distributed(use_gpu=True)
dev = inf.device
spec = get_spec(a.model)
torch.manual_seed(0)
ddp = DDP(build_model(a.model).to(dev))
ddp.reducer.set_overlap(bool(a.overlap))
opt = Adam(ddp.flat, lr=1e-3, eps=1e-7, eps_hat=True) if a.opt == "adam" else SGD(ddp.flat, lr=0.05, momentum=0.9)
acc = torch.zeros((), device=dev)


corr_acc = torch.zeros((), device=dev)


def step(x, y):
    opt.zero_grad()
    if "corr" in parts:
        loss, corr = ops.cross_entropy(ddp(x), y, return_correct=True)
    else:
        loss, corr = ops.cross_entropy(ddp(x), y), None
    loss.backward()
    opt.step()
    acc.add_(loss.detach())
    if corr is not None:
        corr_acc.add_(corr)
    return (loss.detach(),)


run = GraphedStep(step, dev, warmup=2, before_replay=opt._sync_lr, enabled=a.graph)
loader = SyntheticLoader(spec.input_shape, 10, a.batch, a.steps, dev, seed=1, rank=inf.rank)
g = torch.Generator().manual_seed(5 + inf.rank)
fixed = [(torch.rand((a.batch,) + tuple(spec.input_shape), generator=g).to(dev),
          torch.randint(0, 10, (a.batch,), generator=g).to(dev)) for _ in range(a.steps)]
pc = PP.peer_comm()
it = iter(loader) if a.loader == "synthetic" else iter(fixed)
for i in range(a.steps):
    x, y = next(it)
    if "ev" in parts:
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
    run(x, y)
    if "ev" in parts:
        ev[1].record()
    torch.cuda.synchronize()
    if "check" in parts:
        ddp.check()
    cs = ddp.flat.data.double().sum().item()
    allcs = [None] * inf.world_size
    dist.all_gather_object(allcs, (cs, pc.error() if pc is not None else -1, run.captured))
    if inf.rank == 0:
        print(f"step {i}: " + " | ".join(f"r{r} sum={c:.9f} err={e} graph={gr}" for r, (c, e, gr) in enumerate(allcs)),
              flush=True)
mine = ddp.flat.data.cpu()
allp = [None] * inf.world_size
dist.all_gather_object(allp, mine)
if inf.rank == 0:
    d = max((allp[0] - t).abs().max().item() for t in allp)
    print(f"RESULT graph={a.graph} overlap={a.overlap} opt={a.opt} loader={a.loader}: max |rank diff| = {d:.3g} "
          f"transport={ddp.transport}", flush=True)
PC.shutdown()
