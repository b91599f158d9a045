#!/bin/bash
source "$(dirname "$0")/../gpu_check.sh"
run pytest_engine 900 python -m pytest tests/test_gpu_engine.py -m gpu -x -q
run pytest_parallel 900 python -m pytest tests/test_gpu_parallel.py tests/test_gpu_bf16.py -m gpu -x -q
run bench_spg8 300 python bench.py --steps 1000 --warmup 50
run bench_spg1 300 env MXDDP_STEPS_PER_GRAPH=1 python bench.py --steps 1000 --warmup 50
run bench_resnet_bf16 600 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 5 --warmup 2
run bench_resnet_torch 600 python bench.py --model resnet50 --impl torch --batch 32 --steps 5 --warmup 2
