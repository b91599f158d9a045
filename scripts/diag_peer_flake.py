"""Repeat the 2-rank shared-GPU autotune-with-withheld-flags scenario of
tests/test_gpu_peer.py N times in one process and report every run whose validation rejected a
candidate other than 'co' (the autotune message names the disagreeing tensors)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))

import test_gpu_peer as T  # noqa: E402

if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    mode = sys.argv[2] if len(sys.argv) > 2 else "autotune_withhold"
    fails = 0
    for i in range(n):
        t0 = time.time()
        try:
            T._run(2, mode)
            print(f"run {i}: ok ({time.time() - t0:.1f} s)", flush=True)
        except AssertionError as e:
            fails += 1
            print(f"run {i}: FAILED ({time.time() - t0:.1f} s): {e}", flush=True)
    print(f"{fails} of {n} runs failed", flush=True)
