#!/bin/bash
# Round-end counter passes (one pass per run, --kernel-trace only): MNIST step and PyramidNet step.
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
A="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
B="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU"
run pmc_mA 120 rocprofv3 --pmc $A --kernel-trace --output-format csv -d gpurun_out/pmc_mA -o run -- python bench.py --steps 20 --warmup 2 --no-graph
run pmc_mB 120 rocprofv3 --pmc $B --kernel-trace --output-format csv -d gpurun_out/pmc_mB -o run -- python bench.py --steps 20 --warmup 2 --no-graph
run pmc_pA 180 rocprofv3 --pmc $A --kernel-trace --output-format csv -d gpurun_out/pmc_pA -o run -- python bench.py --model pyramidnet110 --steps 2 --warmup 1 --no-graph
run pmc_pB 180 rocprofv3 --pmc $B --kernel-trace --output-format csv -d gpurun_out/pmc_pB -o run -- python bench.py --model pyramidnet110 --steps 2 --warmup 1 --no-graph
