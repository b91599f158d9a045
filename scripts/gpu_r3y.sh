#!/bin/bash
# Round-3: fixed per-call overhead of the fused MNIST step at the driver's step counts
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
run intercept 300 python -u scripts/diag_intercept.py
run b_drv 200 python bench.py --steps 20 --warmup 5
run b_drv2 200 python bench.py --steps 20 --warmup 5
run prof_drv 300 rocprofv3 --kernel-trace -d gpurun_out/prof_drv -o run --output-format csv -- python bench.py --steps 20 --warmup 5
