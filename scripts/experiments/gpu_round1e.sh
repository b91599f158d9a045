#!/bin/bash
# Restructured fused step (7 launches): numerics, bench, kernel profile, model numerics.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run pytest_engine 600 python -m pytest tests/test_gpu_engine.py tests/test_gpu_ops.py -m gpu -x -q
run bench_v1 300 python bench.py --steps 2000 --warmup 100
run prof_v1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v1 -o run --output-format csv -- python bench.py --steps 200 --warmup 20
run pytest_parallel 600 python -m pytest tests/test_gpu_parallel.py tests/test_gpu_bf16.py -m gpu -q
