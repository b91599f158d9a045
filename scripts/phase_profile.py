"""Print in-kernel phase timings (us from block start) of the fused MNIST step."""
import json
import sys

import torch

from mxddp.engine import FusedMnistTrainer

tr = FusedMnistTrainer(batch=int(sys.argv[1]) if len(sys.argv) > 1 else 64, device=0, lr=0.01, use_graph=False)
tr.step(20)
print(json.dumps(tr.phase_profile(30), indent=1))
