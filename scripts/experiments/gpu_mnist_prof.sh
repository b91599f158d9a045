#!/bin/bash
# Fused MNIST step: bench + kernel trace/stats (graph mode) + in-kernel phases.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run bench 300 python bench.py --steps 2000 --warmup 100
run prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mprof -o run --output-format csv -- python bench.py --steps 200 --warmup 20
run phases 300 python scripts/phase_profile.py 64
