#!/bin/bash
# Round-3: F2 publishes conv1's output from the accumulators; full GPU suite at HEAD
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
run t_engine 600 $PT tests/test_gpu_engine.py
run ph 200 python bench.py --phase-profile 30
for i in 1 2 3; do
  run b_$i 300 python bench.py --steps 2000 --warmup 100
done
run b_drv 300 python bench.py --steps 20 --warmup 5
run prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 200 --warmup 20
run pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
