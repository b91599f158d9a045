#!/bin/bash
# Round-3: F7W operand prefetch A/B, then the same-run stock PyTorch comparison
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
run t_engine 600 $PT tests/test_gpu_engine.py
MXDDP_F7W_VQ=1 run t_engine_vq 600 $PT tests/test_gpu_engine.py -k "fused"
run ph_f5 200 python bench.py --phase-profile 30
MXDDP_F7W_VQ=1 run ph_vq 200 python bench.py --phase-profile 30
for i in 1 2 3; do
  run b_def_$i 300 python bench.py --steps 2000 --warmup 100
  MXDDP_F7W_VQ=1 run b_vq_$i 300 python bench.py --steps 2000 --warmup 100
done
KEEP_STEPS=1 bash scripts/gpu_compare.sh
