source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
run eng_tests 400 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread
run bench_20 300 python bench.py --gpus 1 --steps 20 --warmup 5
run bench_def 300 python bench.py
