#!/bin/bash
# the driver's short bench (20 timed steps, 5 warm-up) at 8 / 16 / 32 steps per graph
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
for rep in 1 2 3; do
for s in 8 16 32; do
run short_${s}_$rep 300 env MXDDP_STEPS_PER_GRAPH=$s python bench.py --steps 20 --warmup 5
done
done
