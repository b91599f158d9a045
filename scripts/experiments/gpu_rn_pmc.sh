#!/bin/bash
# LDS / issue counters + kernel times of the ResNet-50 bf16 channels-last step (eager, per dispatch).
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run pmc_rn 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_rn -o run -- python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 2 --warmup 1 --no-graph
run bench_rn256 300 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3
