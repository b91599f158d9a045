#!/bin/bash
# Round-3: F2 occupancy cap (MXDDP_F2_PAD dynamic LDS bytes: 6400 -> 3 blocks per CU, 20480 -> 2)
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
for i in 1 2; do
  run b_pad0_$i 200 python bench.py --steps 2000 --warmup 100
  run b_pad6k_$i 200 env MXDDP_F2_PAD=6400 python bench.py --steps 2000 --warmup 100
  run b_pad20k_$i 200 env MXDDP_F2_PAD=20480 python bench.py --steps 2000 --warmup 100
done
run ph_pad0 200 python bench.py --phase-profile 30
run ph_pad6k 200 env MXDDP_F2_PAD=6400 python bench.py --phase-profile 30
