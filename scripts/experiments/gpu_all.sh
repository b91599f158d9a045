#!/bin/bash
# Full GPU suite + headline bench + layer-path benches.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_default 300 python bench.py
run bench_pyr 300 python bench.py --model pyramidnet110 --impl layers --steps 20 --warmup 3
run bench_rn 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 3
run bench_rn_b256 300 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3
