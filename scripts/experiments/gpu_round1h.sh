#!/bin/bash
# Split-reduction BN + engine tests + PyramidNet bench/profile.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run pytest_ops 600 python -m pytest tests/test_gpu_ops.py tests/test_gpu_engine.py -m gpu -x -q
run pytest_parallel 600 python -m pytest tests/test_gpu_parallel.py -m gpu -x -q
run bench_pyr_layers 600 python bench.py --model pyramidnet110 --impl layers --steps 10 --warmup 3
run prof_pyr 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pyr -o run --output-format csv -- python bench.py --model pyramidnet110 --impl layers --steps 5 --warmup 2
