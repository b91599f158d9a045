# counter passes of the ResNet-50 batch-256 step: the default two-stage kernel vs gk2 (32x32x16)
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
SQ_A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
SQ_B="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU"
for g in 0 2; do
  i=0
  for set in "$SQ_A" "$SQ_B" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i + 1))
    run pmc_g${g}_$i 90 timeout -s KILL 80 rocprofv3 --pmc $set --kernel-trace --output-format csv \
      -d "gpurun_out/pmc_g${g}_$i" -o run -- python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 1 --warmup 1 --no-graph --min-warmup-ms 0 --ab gk2=$g
  done
  python scripts/pmc_summary.py $(find gpurun_out/pmc_g${g}_[1-4] -name '*counter_collection.csv') > gpurun_out/pmc_rn_g$g.txt || true
done
