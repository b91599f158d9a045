#!/bin/bash
# weight-gradient split target sweep (blocks per launch) on the per-layer benchmark, batch 32
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
for t in ${TARGETS:-512 384 256 192}; do
  MXDDP_WGRAD_BLOCKS=$t run wg_$t 300 python scripts/bench_nhwc_layers.py 32 20
done
