#!/bin/bash
# Fused-engine check: numerics vs torch fp32, bench, kernel profile.
source "$(dirname "$0")/../gpu_check.sh"
run pytest_engine 600 python -m pytest tests/test_gpu_engine.py -m gpu -x -q
run bench_v1 300 python bench.py --variant 1 --steps 1000 --warmup 50
run prof_v1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v1 -o run --output-format csv -- python bench.py --variant 1 --steps 100 --warmup 10
