#!/bin/bash
# BN hiwater fix + direct 3x3 conv: op numerics, model numerics, PyramidNet bench/profile.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run pytest_ops 600 python -m pytest tests/test_gpu_ops.py -m gpu -q
run pytest_parallel 600 python -m pytest tests/test_gpu_parallel.py -m gpu -q
run bench_pyr_layers 600 python bench.py --model pyramidnet110 --impl layers --steps 10 --warmup 3
run prof_pyr 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pyr -o run --output-format csv -- python bench.py --model pyramidnet110 --impl layers --steps 5 --warmup 2
