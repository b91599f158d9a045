#!/bin/bash
# LDS counters of the fused MNIST kernels (eager launches so every dispatch is attributed).
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run pmc_mnist 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_mnist -o run -- python bench.py --steps 40 --warmup 5 --graph-mode 0
