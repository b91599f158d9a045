#!/bin/bash
# Counter passes on single Winograd conv shapes (counters with --kernel-trace only).
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
for shp in "146 151 16" "266 271 8" "56 61 32"; do
  tag=$(echo $shp | tr ' ' '_')
  run pmcA_$tag 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d gpurun_out/pmcA_$tag -o run -- python scripts/conv_one.py $shp 10
  run pmcB_$tag 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d gpurun_out/pmcB_$tag -o run -- python scripts/conv_one.py $shp 10
done
