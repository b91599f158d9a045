#!/bin/bash
# Round-3: repeated A/B of the F3 tiling (tile vs tile8) and the weight-gradient wave priority
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
for i in 1 2 3; do
  run b_def_$i 300 python bench.py --steps 2000 --warmup 100
  MXDDP_F3=tile8 run b_t8_$i 300 python bench.py --steps 2000 --warmup 100
  MXDDP_F6W_PRIO=2 run b_p2_$i 300 python bench.py --steps 2000 --warmup 100
  MXDDP_F6W_PRIO=2 MXDDP_F3=tile8 run b_p2t8_$i 300 python bench.py --steps 2000 --warmup 100
done
MXDDP_F3=tile8 run prof_t8 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_t8 -o run --output-format csv -- python bench.py --steps 200 --warmup 20
