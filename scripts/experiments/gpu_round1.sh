#!/bin/bash
source "$(dirname "$0")/../gpu_check.sh"
run pytest_gpu 900 python -m pytest tests/test_gpu_ops.py tests/test_gpu_engine.py -m gpu -x -q
run bench_v0 300 python bench.py --variant 0 --steps 200 --warmup 20
run bench_torch 300 python bench.py --impl torch --steps 100 --warmup 10
run bench_layers 300 python bench.py --impl layers --steps 100 --warmup 10
run prof_v0 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v0 -o run --output-format csv -- python bench.py --variant 0 --steps 50 --warmup 5
run prof_torch 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_torch -o run --output-format csv -- python bench.py --impl torch --steps 50 --warmup 5
