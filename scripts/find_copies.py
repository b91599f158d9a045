"""Which Python call sites issue device copies / small elementwise kernels in a layers-path step
(torch.profiler, CPU side with stacks).  Diagnostic only.

    python scripts/find_copies.py [model] [dtype] [batch]
"""
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    model = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    dtype = sys.argv[2] if len(sys.argv) > 2 else "bf16"
    batch = sys.argv[3] if len(sys.argv) > 3 else "32"
    sys.argv = ["bench.py", "--model", model, "--dtype", dtype, "--batch", batch, "--impl", "layers", "--no-graph"]
    import torch

    import bench
    from mxddp import ops
    from mxddp.parallel import comm as C

    a = bench.parse()
    inf = C.init_distributed(use_gpu=True)
    ops.set_compute_dtype(a.dtype)
    run = bench._layers_or_torch(a, torch, inf, inf.device, C.rccl_comm(), a.batch)
    run(2)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        run(1)
        torch.cuda.synchronize()
    # device-side events: memcpy / memset / copy kernels, with the CPU op that issued them
    dev = Counter()
    for ev in prof.events():
        n = ev.name.lower()
        if ("memcpy" in n or "memset" in n or "copy" in n) and ev.device_type.name == "CUDA":
            dev[ev.name] += 1
    print("device events:", dict(dev))
    print(prof.key_averages(group_by_stack_n=6).table(sort_by="count", row_limit=25, max_name_column_width=60))
    cnt = Counter()
    for ev in prof.events():
        if ev.name in ("aten::copy_", "aten::add", "aten::add_", "aten::zero_", "aten::fill_", "aten::clone",
                       "aten::to", "aten::_to_copy", "aten::mul", "aten::sum", "aten::cat"):
            stack = [f for f in (ev.stack or []) if "mxddp" in f or "bench" in f][:3]
            cnt[(ev.name, " <- ".join(stack))] += 1
    for (name, st), n in cnt.most_common(40):
        print(f"{n:5d} {name:16s} {st}")
    C.shutdown()


if __name__ == "__main__":
    main()
