"""Diagnose: does autotune change the training trajectory?"""
import torch
from mxddp import native
from mxddp.engine import FusedMnistTrainer

C = native()
dev = torch.device("cuda", 0)
comm = C.Comm(C.Comm.new_unique_id(), 0, 1, 0)
a = FusedMnistTrainer(batch=64, device=dev, lr=0.01, comm=comm, force_collectives=True)
b = FusedMnistTrainer(batch=64, device=dev, lr=0.01)


def cnt(t):
    off = (t.eng.y_ptr - t.workspace.data_ptr()) // 4
    return None


a.step(1)
b.step(1)
print("after 1", a.read_metrics(), b.read_metrics())
res = a.autotune(trial_steps=4, include_graphs=True)
print("tuned", a.tuned)
la = a.read_metrics()
b.step(24)
lb = b.read_metrics()
print("during autotune (a reset) / b", la, lb)
for i in range(5):
    a.step(10)
    b.step(10)
    la, lb = a.read_metrics(), b.read_metrics()
    d = max((a.state_dict()[k] - b.state_dict()[k]).abs().max().item() for k in a.state_dict())
    print(i, "loss a %.5f b %.5f  acc a %d b %d  max|dp| %.3g" % (la[0] / 640, lb[0] / 640, la[1], lb[1], d))
for mode, ov in [(0, True), (0, False), (1, True), (1, False)]:
    a.eng.uncapture(); a.eng.set_overlap(ov)
    if mode:
        a._capture(mode)
    a.step(16); b.step(16)
    la, lb = a.read_metrics(), b.read_metrics()
    d = max((a.state_dict()[k] - b.state_dict()[k]).abs().max().item() for k in a.state_dict())
    print(mode, ov, "loss a %.5f b %.5f  acc a %d b %d  max|dp| %.3g" % (la[0] / 1024, lb[0] / 1024, la[1], lb[1], d))
