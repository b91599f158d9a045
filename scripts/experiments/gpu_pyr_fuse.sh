#!/bin/bash
# PyramidNet shortcut fusion check: BN / model numerics, the step, its profile, copy sources.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run pyr_tests 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parallel.py -x -q --timeout 120 --timeout-method thread
run bench_pyr 600 python bench.py --model pyramidnet110 --impl layers --steps 20 --warmup 3
run prof_pyr 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pyr -o run --output-format csv -- python bench.py --model pyramidnet110 --impl layers --steps 6 --warmup 2
run diag_copies 300 python scripts/diag_copies.py
