"""ResNet-50 training trajectories side by side on the same init and the same synthetic batches:
mxddp's channels-last bf16 path (the bench / test path), stock PyTorch-ROCm autocast(bf16)
channels_last on the same module parameters (F.conv2d / F.batch_norm = MIOpen / hipBLASLt), and
mxddp's fp32 path.  Prints the loss every 10 steps, so a training problem can be placed: in the
setup (every path does it) or in a kernel (only one does).

    python scripts/diag_resnet_train.py [steps] [lr] [classes] [batch] [hw]
"""
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from mxddp import native, ops  # noqa: E402
from mxddp.models import resnet50  # noqa: E402
from mxddp.optim import SGD  # noqa: E402
from mxddp.parallel.flat import FlatParams  # noqa: E402


def _bn(x, bn):
    return F.batch_norm(x, bn.running_mean, bn.running_var, bn.weight, bn.bias, training=True, momentum=0.1,
                        eps=bn.eps)


def stock_forward(m, x):
    """The mxddp ResNet-50 module's parameters through plain torch ops."""
    y = F.relu(_bn(F.conv2d(x, m.conv1.weight, stride=2, padding=3), m.bn1))
    y = F.max_pool2d(y, 3, 2, 1)
    for layer in (m.layer1, m.layer2, m.layer3, m.layer4):
        for b in layer:
            h = F.relu(_bn(F.conv2d(y, b.conv1.weight), b.bn1))
            h = F.relu(_bn(F.conv2d(h, b.conv2.weight, stride=b.conv2.stride, padding=1), b.bn2))
            h = _bn(F.conv2d(h, b.conv3.weight), b.bn3)
            sc = y
            if b.downsample is not None:
                sc = _bn(F.conv2d(y, b.downsample[0].weight, stride=b.downsample[0].stride), b.downsample[1])
            y = F.relu(h + sc)
    y = y.float().mean((2, 3))
    return F.linear(y, m.fc.weight, m.fc.bias)


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    lr = float(sys.argv[2]) if len(sys.argv) > 2 else 0.02
    nc = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 32
    hw = int(sys.argv[5]) if len(sys.argv) > 5 else 128
    cuda = torch.device("cuda")
    torch.manual_seed(2)
    m0 = resnet50(num_classes=nc).to(cuda)
    Cn = native()
    D = 3 * hw * hw
    tmpl = torch.empty(nc * D, device=cuda)
    ctr = torch.zeros(4, dtype=torch.int32, device=cuda)
    st = torch.cuda.current_stream().cuda_stream
    Cn.synth_templates(tmpl.data_ptr(), nc, D, 5, st)
    batches = []
    for _ in range(steps):
        x = torch.empty((B, 3, hw, hw), device=cuda)
        y = torch.empty(B, dtype=torch.int32, device=cuda)
        Cn.synth_batch(x.data_ptr(), y.data_ptr(), tmpl.data_ptr(), B, D, nc, 5, ctr.data_ptr(), st)
        batches.append((x, y.long()))
    torch.cuda.synchronize()
    xs = batches[0][0]
    print(f"input: mean {xs.mean().item():.3f} std {xs.std().item():.3f} min {xs.min().item():.3f} "
          f"max {xs.max().item():.3f}; labels {batches[0][1][:16].tolist()}", flush=True)

    runs = {}
    # stock autocast bf16, channels_last, torch.optim.SGD
    m = copy.deepcopy(m0)
    opt = torch.optim.SGD(m.parameters(), lr=lr, momentum=0.9, weight_decay=1e-4)
    ls = []
    for x, y in batches:
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = stock_forward(m, x.contiguous(memory_format=torch.channels_last))
        loss = F.cross_entropy(out.float(), y)
        loss.backward()
        opt.step()
        ls.append(loss.detach())
    runs["stock-bf16"] = torch.stack(ls).cpu()

    for name, dt in (("mxddp-bf16", "bf16"), ("mxddp-fp32", "fp32")):
        m = copy.deepcopy(m0)
        flat = FlatParams(m, cuda)
        opt = SGD(flat, lr=lr, momentum=0.9, weight_decay=1e-4)
        ops.set_compute_dtype(dt)
        ls = []
        try:
            for x, y in batches:
                opt.zero_grad()
                flat.attach_grads()
                loss = ops.cross_entropy(m(x), y.int())
                loss.backward()
                opt.step()
                ls.append(loss.detach())
            torch.cuda.synchronize()
        finally:
            ops.set_compute_dtype("fp32")
        runs[name] = torch.stack(ls).float().cpu()

    names = list(runs)
    print("step " + " ".join(f"{n:>12}" for n in names))
    for i in sorted(set(list(range(0, min(steps, 10))) + list(range(10, steps, 10)) + list(range(max(0, steps - 10), steps)))):
        print(f"{i:>4} " + " ".join(f"{runs[n][i].item():>12.4f}" for n in names))
    for n in names:
        r = runs[n]
        print(f"{n}: first10 {r[:10].mean().item():.3f} last10 {r[-10:].mean().item():.3f}")


if __name__ == "__main__":
    main()
