source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
run t_b 600 $T tests/test_gpu_wgrad_defer.py tests/test_gpu_engine.py tests/test_gpu_rccl_diag.py
for i in 1 2; do for d in 0 1; do run mn_d${d}_$i 300 python bench.py --steps 20 --warmup 5 --ab fc1_defer=$d; done; done
for d in 0 1; do run mnl_d$d 300 python bench.py --steps 2000 --warmup 100 --ab fc1_defer=$d; done
for i in 1 2; do for d in 0 1; do run pyr_w${d}_$i 300 python bench.py --model pyramidnet110 --steps 20 --warmup 3 --ab wgrad_defer=$d; done; done
for d in 0 1; do run rn32_w$d 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 3 --ab wgrad_defer=$d; done
for d in 0 1; do run rn256_w$d 300 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3 --ab wgrad_defer=$d; done
run prof_defer 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_defer -o run --output-format csv -- python bench.py --steps 200 --warmup 20 --min-warmup-ms 0 --ab fc1_defer=1
python scripts/kstats.py "$(find gpurun_out/prof_defer -name '*kernel_stats.csv' | head -1)" 200 > gpurun_out/summary_prof_defer.txt || true
