#!/bin/bash
# Quick Winograd iteration: conv numerics + per-shape timings.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run wq_tests 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "conv or wino or filter"
run wq_conv 300 python scripts/bench_conv.py --only-wino
