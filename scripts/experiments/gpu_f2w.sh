#!/bin/bash
# F2W (Winograd conv2 forward) check: engine tests, bench Winograd vs direct F2, kernel stats.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run pytest_engine 300 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread
run bench_f2w 300 python bench.py --steps 2000 --warmup 100
run bench_f2direct 300 env MXDDP_MNIST_F2=direct python bench.py --steps 2000 --warmup 100
run prof_f2w 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f2w -o run --output-format csv -- python bench.py --steps 200 --warmup 20
run phases_f2w 300 python scripts/phase_profile.py 64
