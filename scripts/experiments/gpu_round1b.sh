#!/bin/bash
source "$(dirname "$0")/../gpu_check.sh"
run pytest_engine 600 python -m pytest tests/test_gpu_engine.py -m gpu -x -q
run bench_v1 300 python bench.py --variant 1 --steps 500 --warmup 50
run bench_v0 300 python bench.py --variant 0 --steps 200 --warmup 20
run prof_v1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v1 -o run --output-format csv -- python bench.py --variant 1 --steps 100 --warmup 10
