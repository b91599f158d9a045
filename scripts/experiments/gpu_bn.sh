#!/bin/bash
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run pytest_bn 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parallel.py -m gpu -q --timeout 120 --timeout-method thread
run bench_pyr 300 python bench.py --model pyramidnet110 --impl layers --steps 20 --warmup 3
run prof_pyr 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pyr -o run --output-format csv -- python bench.py --model pyramidnet110 --impl layers --steps 5 --warmup 2
