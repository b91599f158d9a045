# MNIST F2: Winograd V in [xi][ci][12] (conflict-free stores) -- tests, bench, kernel times, LDS counters
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
run t_eng 600 $T tests/test_gpu_engine.py
for i in 1 2 3; do run mn$i 300 python bench.py; done
run mnl 300 python bench.py --steps 2000 --warmup 100
run prof_mn 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mn -o run --output-format csv -- python bench.py --steps 200 --warmup 20 --min-warmup-ms 0
run pmc_mn 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES -d gpurun_out/pmc_mn -o run --output-format csv -- python bench.py --steps 20 --warmup 2 --no-graph --min-warmup-ms 0
