"""Fixed per-call overhead of the fused MNIST step at the driver's step counts: times replay(n)
for several n (median of repeats) and several steps-per-graph settings, and fits
t(n) = a + b n.  The intercept a is what a 20-step timed region pays on top of the steady
per-step time b.

    python scripts/diag_intercept.py
"""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mxddp  # noqa: E402
from mxddp.engine import FusedMnistTrainer  # noqa: E402


def timed(fn, reps=7):
    out = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        out.append((time.perf_counter() - t0) * 1e6)
    return statistics.median(out)


def main():
    mxddp.native()
    res = {"sync_only_us": timed(lambda: None, 21)}
    for spg in [int(s) for s in os.environ.get("SPG", "32,20,8,1").split(",")]:
        tr = FusedMnistTrainer(batch=64, device=0, use_graph=True, steps_per_graph=spg)
        tr.step(1)
        tr.warm_graphs()
        tr.step(50)
        torch.cuda.synchronize()
        pts = {}
        for n in (1, 2, 4, 5, 10, 20, 40, 80):
            pts[n] = timed(lambda: tr.step(n))
        xs, ys = list(pts), list(pts.values())
        mx_, my = sum(xs) / len(xs), sum(ys) / len(ys)
        b = sum((x - mx_) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx_) ** 2 for x in xs)
        a = my - b * mx_
        res[f"spg{spg}"] = {"t_us": {k: round(v, 1) for k, v in pts.items()}, "intercept_us": round(a, 1),
                            "per_step_us": round(b, 2), "img_s_at_20": round(64 * 20 / pts[20] * 1e6)}
        print(json.dumps({f"spg{spg}": res[f"spg{spg}"]}), flush=True)
        del tr
    print(json.dumps(res))


if __name__ == "__main__":
    main()
