#!/bin/bash
# F5 slice width 36 (256 blocks) vs 48 (192 blocks): engine numerics, interleaved A/B, trace.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run eng 300 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread
run c36 300 python bench.py --steps 2000 --warmup 100
run c48 300 env MXDDP_F5_COLS=48 python bench.py --steps 2000 --warmup 100
run c36b 300 python bench.py --steps 2000 --warmup 100
run c48b 300 env MXDDP_F5_COLS=48 python bench.py --steps 2000 --warmup 100
run c36c 300 python bench.py --steps 2000 --warmup 100
run tr36 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_c36 -o run -- python bench.py --steps 400 --warmup 50
