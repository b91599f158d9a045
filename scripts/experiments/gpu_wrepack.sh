#!/bin/bash
# Batched weight repack with 16-byte stores: NHWC tests, ResNet-50 benches, kernel-trace stats.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run build 900 python -c "import __graft_entry__ as g; g.build()"
run pytest_nhwc 300 python -u -m pytest tests/test_gpu_nhwc.py -x -q --timeout 120 --timeout-method thread
run bench_rn256 300 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3
run bench_rn32 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 10 --warmup 3
run prof_rn 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn -o run --output-format csv -- python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 5 --warmup 2
