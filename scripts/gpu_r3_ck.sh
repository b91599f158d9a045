#!/bin/bash
# Round-3 checkpoint: full GPU suite, smoke, driver-length bench, ResNet-50 with the stem BN statistics
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_driver 300 python bench.py --steps 20 --warmup 5
run bench_rn32 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 5
run bench_rn256 400 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3
run diag_copies 300 env PYTHONPATH=. python scripts/diag_copies2.py pyramidnet110
