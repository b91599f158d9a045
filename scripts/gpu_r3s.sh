#!/bin/bash
# Round-3: F2 LDS-only barriers + B fragments requested in stage 2; conv1-grad slab count retest
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
run t_engine 600 $PT tests/test_gpu_engine.py
run ph 200 python bench.py --phase-profile 30
for i in 1 2 3; do
  run b_$i 300 python bench.py --steps 2000 --warmup 100
  MXDDP_G1_SLABS=64 run b_g64_$i 300 python bench.py --steps 2000 --warmup 100
done
MXDDP_G1_SLABS=64 run ph_g64 200 python bench.py --phase-profile 30
