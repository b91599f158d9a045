#!/bin/bash
# Counter passes over the fused MNIST step (counters with --kernel-trace only, one pass per run).
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run mpmcA 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/mpmcA -o run -- python bench.py --steps 20 --warmup 2 --no-graph
run mpmcB 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d gpurun_out/mpmcB -o run -- python bench.py --steps 20 --warmup 2 --no-graph
