#!/bin/bash
# ResNet-50 input path: vectorised NCHW -> NHWC conversion, synthetic images split over more
# blocks; full GPU suite, ResNet-50 benches and kernel-trace stats.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run build 900 python -c "import __graft_entry__ as g; g.build()"
run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
run bench_rn256 300 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3
run bench_rn32 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 10 --warmup 3
run bench_driver 300 python bench.py --steps 20 --warmup 5
run prof_rn 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn -o run --output-format csv -- python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 3 --warmup 2
