#!/bin/bash
# Winograd conv: numerics, per-shape timings, then PyramidNet bench.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run pytest_conv 400 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or wino"
run bench_conv 300 python scripts/bench_conv.py
run bench_conv_v2 300 env MXDDP_WINO_FWD=2 python scripts/bench_conv.py
run bench_pyr 300 python bench.py --model pyramidnet110 --impl layers --steps 10 --warmup 3
