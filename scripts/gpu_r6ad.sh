# coalesced 3x3 weight-gradient reduction: numerics (per-conv and deferred), ResNet-50 runs, b32 kernel stats
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
run tests 900 python -u -m pytest tests/test_gpu_nhwc.py tests/test_gpu_wgrad_defer.py -x -q --timeout 120 --timeout-method thread
run rn32 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 3
run rn256 300 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3
run prof32 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof32 -o run -- python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 10 --warmup 3
python scripts/kstats.py "$(find gpurun_out/prof32 -name "*kernel_stats.csv" | head -1)" > gpurun_out/summary_prof_rn32.txt || true
