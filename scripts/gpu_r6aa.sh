# wgrad_c3 patch swizzle + stem weight-gradient patch pitch: numerics, ResNet-50 runs, LDS counters
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
run nhwc 600 python -u -m pytest tests/test_gpu_nhwc.py -x -q --timeout 120 --timeout-method thread
run rn256 300 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3
run rn32 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 3
SQ_A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
SQ_B="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU"
i=0
for set in "$SQ_A" "$SQ_B"; do
  i=$((i + 1))
  run pmc_$i 90 timeout -s KILL 80 rocprofv3 --pmc $set --kernel-trace --output-format csv \
    -d "gpurun_out/pmc_$i" -o run -- python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 1 --warmup 1 --no-graph --min-warmup-ms 0
done
python scripts/pmc_summary.py $(find gpurun_out/pmc_[1-2] -name '*counter_collection.csv') > gpurun_out/pmc_rn.txt || true
