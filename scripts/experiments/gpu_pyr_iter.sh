#!/bin/bash
# PyramidNet layer-path iteration: conv / BN numerics, per-shape conv timings, step + profile.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run ops_tests 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread
run bench_pyr 600 python bench.py --model pyramidnet110 --impl layers --steps 20 --warmup 3
run prof_pyr 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pyr -o run --output-format csv -- python bench.py --model pyramidnet110 --impl layers --steps 6 --warmup 2
