#!/bin/bash
# Layer path after direct-grad / in-place shortcut / on-device nbt: GPU tests, PyramidNet bench + profile.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run bench_pyr 300 python bench.py --model pyramidnet110 --impl layers --steps 10 --warmup 3
run prof_pyr 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pyr -o run --output-format csv -- python bench.py --model pyramidnet110 --impl layers --steps 5 --warmup 2
