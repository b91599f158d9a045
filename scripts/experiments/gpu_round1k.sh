#!/bin/bash
# F5 48-col, merged F6+F7, a1 recompute: numerics, phase profile, bench, kernel profile.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run pytest_engine 600 python -m pytest tests/test_gpu_engine.py -m gpu -x -q
run phase 300 env PYTHONPATH=. python scripts/phase_profile.py
run bench_v1 300 python bench.py --steps 2000 --warmup 100
run prof_v1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v1 -o run --output-format csv -- python bench.py --steps 200 --warmup 20
run bn_rep 600 python -m pytest tests/test_gpu_ops.py -m gpu -q -k batchnorm
