#!/bin/bash
# F5 side-duty balance check: engine tests, bench, kernel stats, phases.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run pytest_engine 300 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread
run bench_f5 300 python bench.py --steps 2000 --warmup 100
run prof_f5 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f5 -o run --output-format csv -- python bench.py --steps 200 --warmup 20
run phases_f5 300 python scripts/phase_profile.py 64
