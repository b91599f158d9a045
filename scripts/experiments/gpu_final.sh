#!/bin/bash
# Round-end verification on a fresh box: full GPU suite, smoke, headline bench (driver defaults
# and a long run), per-kernel profile of the headline step, layer-path benches.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_default 300 python bench.py
run bench_long 300 python bench.py --steps 2000 --warmup 100
run prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 200 --warmup 20
run bench_pyr 300 python bench.py --model pyramidnet110 --impl layers --steps 20 --warmup 3
run bench_rn 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 3
