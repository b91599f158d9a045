source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
run t_e 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine.py -k deferred
for i in 1 2; do for d in 0 2; do run mn_d${d}_$i 300 python bench.py --steps 20 --warmup 5 --ab fc1_defer=$d; done; done
for d in 0 2; do run mnl_d$d 300 python bench.py --steps 2000 --warmup 100 --ab fc1_defer=$d; done
run prof_defer2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_defer2 -o run --output-format csv -- python bench.py --steps 200 --warmup 20 --min-warmup-ms 0 --ab fc1_defer=2
python scripts/kstats.py "$(find gpurun_out/prof_defer2 -name '*kernel_stats.csv' | head -1)" 200 > gpurun_out/summary_prof_defer2.txt || true
