#!/bin/bash
# Current in-kernel phase timings of the fused MNIST step + the headline bench.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run phases 300 python scripts/phase_profile.py
run bench 300 python bench.py
