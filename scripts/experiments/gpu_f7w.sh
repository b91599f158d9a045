#!/bin/bash
# Winograd F7W check: engine numerics, bench (Winograd vs direct F7), kernel stats, phases.
source "$(dirname "$0")/../gpu_check.sh"
run pytest_engine 600 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread
run bench_wino 300 python bench.py --steps 2000 --warmup 100
MXDDP_MNIST_F7=direct run bench_direct 300 python bench.py --steps 2000 --warmup 100
run bench_wino2 300 python bench.py --steps 2000 --warmup 100
run prof_wino 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wino -o run --output-format csv -- python bench.py --steps 200 --warmup 20
run phases 300 python scripts/phase_profile.py 64
