#!/bin/bash
# Round-3 gate at HEAD: full GPU suite, smoke, driver-length bench, ResNet-50 both batches, CPU bench
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_driver 300 python bench.py --steps 20 --warmup 5
run bench_default 300 python bench.py
run bench_rn32 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 5
run bench_rn256 400 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3
run prof_rn 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn -o run --output-format csv -- python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 5 --warmup 2
