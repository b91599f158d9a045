"""Per-parameter gradient cosine of the channels-last bf16 ResNet-50 vs the fp32 NCHW model."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from mxddp import ops  # noqa: E402
from mxddp.models import resnet50  # noqa: E402
from mxddp.models.resnet import Bottleneck  # noqa: E402

cuda = torch.device("cuda", 0)
torch.manual_seed(4)
S = int(sys.argv[1]) if len(sys.argv) > 1 else 128
ref = resnet50(num_classes=10)
m = resnet50(num_classes=10).to(cuda)
m.load_state_dict(ref.state_dict())
x = torch.randn(2, 3, S, S)
y = torch.tensor([3, 7])
F.cross_entropy(ref(x), y).backward()
ops.set_compute_dtype("bf16")
loss = ops.cross_entropy(m(x.to(cuda)), y.to(cuda))
loss.backward()
torch.cuda.synchronize()
gp = dict(m.named_parameters())
for n, p in ref.named_parameters():
    g = gp[n].grad.cpu().flatten()
    r = p.grad.flatten()
    cos = F.cosine_similarity(g, r, dim=0).item()
    ratio = (g.norm() / (r.norm() + 1e-30)).item()
    flag = "  <--" if cos < 0.95 else ""
    print(f"{n:40s} cos={cos:.4f} norm_ratio={ratio:.3f}{flag}")

# isolated last bottleneck at the same spatial size
torch.manual_seed(5)
bref = Bottleneck(2048, 512)
b = Bottleneck(2048, 512).to(cuda)
b.load_state_dict(bref.state_dict())
xi = torch.randn(2, 2048, 4, 4)
gi = torch.randn(2, 2048, 4, 4)
bref(xi).backward(gi)
from mxddp.ops import nhwc  # noqa: E402
xg = xi.to(cuda).permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
b.forward_nhwc(xg).backward(gi.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).to(cuda))
for n, p in bref.named_parameters():
    g = dict(b.named_parameters())[n].grad.cpu().flatten()
    print("block", n, F.cosine_similarity(g, p.grad.flatten(), dim=0).item())
