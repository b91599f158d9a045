#!/bin/bash
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run pytest_ops 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_bf16.py -m gpu -x -q --timeout 120 --timeout-method thread
run bench_rn 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 6 --warmup 3
run prof_rn 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn -o run --output-format csv -- python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 4 --warmup 2
