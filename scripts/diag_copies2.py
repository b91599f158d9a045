"""Which Python-level ops issue device-to-device copies (hipMemcpyAsync -> __amd_rocclr_copyBuffer)
inside a PyramidNet / ResNet-50 layer-path training step?  torch.profiler with stacks."""
import sys

import torch

from mxddp import ops
from mxddp.models import build_model, get_spec
from mxddp.optim import SGD
from mxddp.parallel.ddp import DistributedDataParallel as DDP
from mxddp.parallel import comm as C

model_name = sys.argv[1] if len(sys.argv) > 1 else "pyramidnet110"
dtype = sys.argv[2] if len(sys.argv) > 2 else "fp32"
C.init_distributed(use_gpu=True)
if dtype != "fp32":
    ops.set_compute_dtype(dtype)
dev = torch.device("cuda", 0)
spec = get_spec(model_name)
net = DDP(build_model(model_name).to(dev))
opt = SGD(net.flat, lr=0.1, momentum=0.9, weight_decay=1e-4)
B = 8
x = torch.rand((B,) + tuple(spec.input_shape), device=dev)
y = torch.randint(0, spec.num_classes, (B,), device=dev, dtype=torch.int32)


def step():
    opt.zero_grad()
    ops.cross_entropy(net(x), y).backward()
    opt.step()


for _ in range(2):
    step()
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile

with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    step()
    torch.cuda.synchronize()
evs = [e for e in prof.events() if "Memcpy" in e.name or "copy_" in e.name or "clone" in e.name]
from collections import Counter

cnt = Counter()
for e in prof.events():
    if e.name in ("aten::copy_", "aten::clone", "aten::contiguous", "aten::add", "aten::add_", "aten::cat"):
        st = [s for s in (e.stack or []) if "mxddp" in s or "torch/autograd" in s][:3]
        cnt[(e.name, tuple(st))] += 1
for k, v in cnt.most_common(25):
    print(v, k)
print(prof.key_averages().table(sort_by="count", row_limit=25))
C.shutdown()
