#!/bin/bash
# Kernel trace of the default (graph) MNIST step: per-kernel durations and inter-kernel gaps.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run trace_mnist 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_mnist -o run -- python bench.py --steps 400 --warmup 50
