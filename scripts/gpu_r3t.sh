#!/bin/bash
# Round-3: F2 conv1-stage priority A/B; Keras fused-engine kernel stats + phase baseline
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
MXDDP_F2_PRIO=1 run ph_prio 200 python bench.py --phase-profile 30
for i in 1 2 3; do
  run b_$i 300 python bench.py --steps 2000 --warmup 100
  MXDDP_F2_PRIO=1 run b_prio_$i 300 python bench.py --steps 2000 --warmup 100
done
run b_keras 300 python bench.py --model keras_cnn --steps 1000 --warmup 50
run prof_keras 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_keras -o run --output-format csv -- python bench.py --model keras_cnn --steps 300 --warmup 30
