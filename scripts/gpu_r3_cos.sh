#!/bin/bash
# Round-3: co-split Winograd weight-gradient blocks with the slab epilogue (MXDDP_F6W_COS=2)
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
run t_engine_cos2 600 env MXDDP_F6W_COS=2 $PT tests/test_gpu_engine.py
for i in 1 2 3; do
  run b_def_$i 200 python bench.py --steps 2000 --warmup 100
  run b_cos2_$i 200 env MXDDP_F6W_COS=2 python bench.py --steps 2000 --warmup 100
done
run ph_cos2 200 env MXDDP_F6W_COS=2 python bench.py --phase-profile 30
run b_drv_cos2 200 env MXDDP_F6W_COS=2 python bench.py --steps 20 --warmup 5
