#!/bin/bash
# steps unrolled per graph (MXDDP_STEPS_PER_GRAPH) for the default MNIST bench
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
for s in 8 16 32 64 8 32; do
run spg_$s 300 env MXDDP_STEPS_PER_GRAPH=$s python bench.py --steps 2048 --warmup 128
done
