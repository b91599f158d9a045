"""Print in-kernel phase timings (us from block start) of the fused MNIST step."""
import json
import sys

import os

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from mxddp.engine import FusedMnistTrainer  # noqa: E402

tr = FusedMnistTrainer(batch=int(sys.argv[1]) if len(sys.argv) > 1 else 64, device=0, lr=0.01, use_graph=False)
tr.step(20)
print(json.dumps(tr.phase_profile(30), indent=1))
