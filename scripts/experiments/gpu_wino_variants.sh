#!/bin/bash
# Winograd forward / data-gradient kernel variants per PyramidNet shape, plus numerics of variant 4.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run wino_v2 300 env MXDDP_WINO_FWD=2 python scripts/bench_conv.py --only-wino
run wino_v4 300 env MXDDP_WINO_FWD=4 python scripts/bench_conv.py --only-wino
run wino_v4_tests 300 env MXDDP_WINO_FWD=4 python -u -m pytest tests/test_gpu_ops.py -x -q -k "conv or winograd" --timeout 120 --timeout-method thread
