#!/bin/bash
# PMC counters for the fused kernels (counters only with --kernel-trace, never with sys/runtime traces).
source "$(dirname "$0")/../gpu_check.sh"
run counters_list 120 rocprofv3 -L
run pmc1 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d gpurun_out/pmc1 -o run -- python bench.py --variant 1 --steps 20 --warmup 2
run pmc2 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM --kernel-trace --output-format csv -d gpurun_out/pmc2 -o run -- python bench.py --variant 1 --steps 20 --warmup 2
