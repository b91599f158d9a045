"""Replica-mode hipGraph divergence hunt: train the Keras CNN with ReplicaGroup(use_graph=True)
for one 'epoch', do ACTION (none | cpu_read: copy every parameter to the host | sleep: idle the
host 50 ms | sync: device synchronize), train another epoch; print the loss trajectory."""
import os
import sys
import time

import torch

from mxddp import ops
from mxddp.data import SyntheticLoader
from mxddp.models import build_model, get_spec
from mxddp.optim import Adam
from mxddp.parallel.replica import ReplicaGroup

action = sys.argv[1]
graph = sys.argv[2] == "graph" if len(sys.argv) > 2 else True
dev = torch.device("cuda", 0)
torch.manual_seed(1)
spec = get_spec("keras_cnn")
grp = ReplicaGroup(build_model("keras_cnn"), [dev], lambda f: Adam(f, lr=1e-3, eps=1e-7, eps_hat=True),
                   use_graph=graph)
epochs, steps = (1, 236) if action == "long" else (2, 118)
loader = SyntheticLoader(spec.input_shape, 10, 512, steps, dev, seed=1)
loss_fn = lambda o, t: ops.cross_entropy(o, t, return_correct=True)  # noqa: E731
traj = []
per_step = []
acc = torch.zeros((), device=dev)
for epoch in range(epochs):
    if action != "noalloc":
        acc = torch.zeros((), device=dev)
    for i, (x, y) in enumerate(loader):
        grp.step(x, y, loss_fn)
        ls = torch.tensor(grp.read_metrics()[0])
        acc += ls / 512
        if os.environ.get("DIAG_PER_STEP") and 95 <= epoch * steps + i <= 135:
            per_step.append(round(ls.item() / 512, 3))
        if i % 20 == 19:
            traj.append(round(acc.item() / 20, 4))
            acc.zero_()
    torch.cuda.synchronize()
    if epoch == 0:
        if action == "cpu_read":
            for n, p in grp.module.named_parameters():
                p.detach().float().cpu().numpy()
        elif action == "sleep":
            time.sleep(0.05)
        elif action == "sync":
            torch.cuda.synchronize()
print(action, "graph" if graph else "eager", traj, flush=True)
print("steps 95..135:", per_step, flush=True)
