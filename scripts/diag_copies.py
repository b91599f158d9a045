"""Census of the device-to-device copies (hipMemcpyAsync -> __amd_rocclr_copyBuffer) and other
small copy / fill kernels in one eager layer-path training step, each attributed to the CPU op
that issued it and that op's mxddp call site (torch.profiler with stacks).  Diagnostic only.

    python scripts/diag_copies.py [model] [dtype] [batch]
"""
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def _site(ev):
    """Innermost mxddp / bench frames of an op (walking up to the first op that has a stack)."""
    e = ev
    while e is not None and not e.stack:
        e = e.cpu_parent
    frames = [f for f in ((e.stack or []) if e is not None else []) if "mxddp" in f or "bench" in f]
    return " <- ".join(frames[:3])


def main():
    model = sys.argv[1] if len(sys.argv) > 1 else "pyramidnet110"
    dtype = sys.argv[2] if len(sys.argv) > 2 else "fp32"
    batch = sys.argv[3] if len(sys.argv) > 3 else "64"
    sys.argv = ["bench.py", "--model", model, "--dtype", dtype, "--batch", batch, "--impl", "layers", "--no-graph"]
    import torch

    import bench
    from mxddp import ops
    from mxddp.parallel import comm as C

    a = bench.parse()
    gpu = torch.cuda.is_available()
    inf = C.init_distributed(use_gpu=gpu)
    sync = torch.cuda.synchronize if gpu else (lambda: None)
    ops.set_compute_dtype(a.dtype)
    run = bench._layers_or_torch(a, torch, inf, inf.device, C.rccl_comm(), a.batch)
    run(3)
    sync()
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        run(1)
        sync()
    evs = prof.events()
    dev = Counter(ev.name for ev in evs if ev.device_type.name == "CUDA")
    keys = ("memcpy", "memset", "copy", "fill", "add")
    print("device events of one step (copy / fill / add like):")
    for name, n in sorted(dev.items(), key=lambda t: -t[1]):
        if any(k in name.lower() for k in keys):
            print(f"{n:6d}  {name[:110]}")
    print(f"total device events: {sum(dev.values())}")
    # attribute each copy-like device event to the CPU op that launched it
    by_site = Counter()
    for ev in evs:
        if ev.device_type.name == "CUDA":
            continue
        for k in getattr(ev, "kernels", []) or []:
            kn = k.name.lower()
            if any(t in kn for t in ("memcpy", "copybuffer", "copy", "fill", "memset")):
                by_site[(ev.name, k.name[:60], _site(ev))] += 1
    print("\nissuing op / device event / call site:")
    for (op, kn, site), n in by_site.most_common(40):
        print(f"{n:5d}  {op:22s} {kn:60s} {site}")
    C.shutdown()


if __name__ == "__main__":
    main()
