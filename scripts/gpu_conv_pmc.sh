#!/bin/bash
# Counter passes over the per-layer NHWC conv benchmark (counters with --kernel-trace only).
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
run pmcA 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmcA -o run -- python scripts/bench_nhwc_layers.py 32 3
run pmcB 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d gpurun_out/pmcB -o run -- python scripts/bench_nhwc_layers.py 32 3
