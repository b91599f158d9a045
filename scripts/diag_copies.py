"""Which ops of the PyramidNet layers step launch device copies / elementwise adds (torch
profiler, eager step after warm-up; prints each op with its Python call site)."""
import sys

import torch

sys.path.insert(0, ".")
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from mxddp import native, ops  # noqa: E402
from mxddp.models import build_model  # noqa: E402
from mxddp.optim import SGD  # noqa: E402
from mxddp.parallel.ddp import DistributedDataParallel as DDP  # noqa: E402
from mxddp.parallel import comm  # noqa: E402

comm.init_distributed()
dev = torch.device("cuda", 0)
model = build_model(sys.argv[1] if len(sys.argv) > 1 else "pyramidnet110").to(dev)
net = DDP(model)
opt = SGD(net.flat, lr=0.1, momentum=0.9, weight_decay=1e-4)
x = torch.randn(64, 3, 32, 32, device=dev)
y = torch.randint(0, 10, (64,), device=dev)


def step():
    opt.zero_grad()
    loss = ops.cross_entropy(net(x), y)
    loss.backward()
    opt.step()


for _ in range(2):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
    step()
    torch.cuda.synchronize()
print(prof.key_averages(group_by_stack_n=6).table(sort_by="count", row_limit=25, max_name_column_width=40))
