#!/bin/bash
# Winograd conv: numerics, per-shape timings (occupancy 2 vs 3), then PyramidNet bench.
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
run pytest_conv 400 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -v --timeout 120 --timeout-method thread -k "conv or wino"
run bench_conv_occ2 300 env MXDDP_WINO_OCC=2 python scripts/bench_conv.py
run bench_conv_occ3 300 env MXDDP_WINO_OCC=3 python scripts/bench_conv.py
run bench_pyr_wino 300 python bench.py --model pyramidnet110 --impl layers --steps 10 --warmup 3
