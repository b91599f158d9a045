# MNIST headline step at HEAD: counter passes (eager launches: one dispatch per kernel) + graphed kernel trace
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
SQ_A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
SQ_B="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU"
i=0
for set in "$SQ_A" "$SQ_B" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  run pmc_$i 90 timeout -s KILL 80 rocprofv3 --pmc $set --kernel-trace --output-format csv \
    -d "gpurun_out/pmc_$i" -o run -- python bench.py --steps 20 --warmup 2 --no-graph --min-warmup-ms 0
done
python scripts/pmc_summary.py $(find gpurun_out/pmc_[1-4] -name '*counter_collection.csv') > gpurun_out/pmc_mnist.txt || true
run trace 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace -o run -- python bench.py --steps 200 --warmup 20
python scripts/kstats.py "$(find gpurun_out/trace -name '*kernel_stats.csv' | head -1)" > gpurun_out/summary_prof_mnist.txt || true
