#!/bin/bash
# Fused MNIST engine: full engine tests + bench + graph-mode kernel timeline.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run pytest_engine 600 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread
run bench 300 python bench.py --steps 2000 --warmup 100
run prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mprof -o run --output-format csv -- python bench.py --steps 200 --warmup 20
