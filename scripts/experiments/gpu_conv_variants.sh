#!/bin/bash
# Per-shape Winograd timings: forward / data-gradient kernel variants (MXDDP_WINO_FWD) and the
# weight-gradient grid rounding (slots floor vs the old ceil), then the PyramidNet step.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run conv_default 300 python scripts/bench_conv.py --only-wino
run conv_wg_ceil 300 env MXDDP_WGRAD_CEIL=1 python scripts/bench_conv.py --only-wino
run conv_v2 300 env MXDDP_WINO_FWD=2 python scripts/bench_conv.py --only-wino
run conv_v3 300 env MXDDP_WINO_FWD=3 python scripts/bench_conv.py --only-wino
run conv_v4 300 env MXDDP_WINO_FWD=4 python scripts/bench_conv.py --only-wino
run wg_tests 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "conv or winograd" --timeout 120 --timeout-method thread
run bench_pyr 600 python bench.py --model pyramidnet110 --impl layers --steps 20 --warmup 3
