#!/bin/bash
# Round-3 re-entry check at HEAD: full GPU suite, smoke, driver bench, MNIST kernel stats
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
run pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_driver 300 python bench.py --steps 20 --warmup 5
run bench_long 300 python bench.py --steps 2000 --warmup 100
run prof_mnist 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mnist -o run --output-format csv -- python bench.py --steps 200 --warmup 20
run bench_rn256 300 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3
run prof_rn 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn -o run --output-format csv -- python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 3 --warmup 2
