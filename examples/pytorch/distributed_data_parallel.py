#!/usr/bin/env python3
"""Drop-in for the reference's pytorch/distributed_data_parallel.py: same flags, runs on mxddp (see mxddp/compat.py)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from mxddp.compat import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main("pytorch/distributed_data_parallel"))
