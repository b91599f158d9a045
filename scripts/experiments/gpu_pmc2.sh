#!/bin/bash
# Per-kernel PMC counters of the fused step (counters with --kernel-trace only).
source "$(dirname "$0")/../gpu_check.sh"
B="python bench.py --steps 20 --warmup 2 --no-graph"
run pmcA 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d gpurun_out/pmcA -o run -- $B
run pmcB 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_SALU --kernel-trace --output-format csv -d gpurun_out/pmcB -o run -- $B
