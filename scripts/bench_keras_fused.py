"""Throughput of the fused Keras-CNN engine (one GPU, or in-process replicas): images/s."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mxddp.keras_engine import FusedKerasReplicas, FusedKerasTrainer  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--steps", type=int, default=500)
ap.add_argument("--warmup", type=int, default=50)
ap.add_argument("--replicas", type=int, default=0)
ap.add_argument("--no-graph", action="store_true")
a = ap.parse_args()
if a.replicas:
    t = FusedKerasReplicas([torch.device("cuda", 0)] * a.replicas, batch=a.batch, use_graph=not a.no_graph)
    sync = t.synchronize
    nimg = a.batch * a.replicas
else:
    t = FusedKerasTrainer(batch=a.batch, device=0, use_graph=not a.no_graph)
    sync = t.synchronize
    nimg = a.batch
t.step(a.warmup)
sync()
t0 = time.perf_counter()
t.step(a.steps)
sync()
dt = time.perf_counter() - t0
ls, cs = t.read_metrics()
n = (a.warmup + a.steps) * nimg
print(json.dumps({"impl": "keras-fused", "replicas": a.replicas, "batch": a.batch, "img_per_s": round(nimg * a.steps / dt, 1),
                  "ms_per_step": round(dt / a.steps * 1e3, 4), "loss_avg": ls / n, "acc": cs / n}), flush=True)
