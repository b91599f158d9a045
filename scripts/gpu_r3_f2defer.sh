#!/bin/bash
# Round-3: F2 global stores deferred to the kernel end (no store ahead of the stage-2 loads)
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
run t_engine 600 $PT tests/test_gpu_engine.py tests/test_gpu_parallel.py
for i in 1 2 3; do run b_$i 200 python bench.py --steps 2000 --warmup 100; done
run b_drv 200 python bench.py --steps 20 --warmup 5
run ph 200 python bench.py --phase-profile 30
