#!/bin/bash
# LDS / issue counters of every PyramidNet layer-path kernel (eager step, per dispatch).
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run pmc_pyr 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_pyr -o run -- python bench.py --model pyramidnet110 --impl layers --steps 3 --warmup 1 --no-graph
