#!/bin/bash
# MNIST fused-engine iteration: engine numerics tests, phase timings, headline bench.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run engine_tests 300 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread
run phases 300 python scripts/phase_profile.py
run bench 300 python bench.py
run bench2 300 python bench.py --steps 2000 --warmup 100
