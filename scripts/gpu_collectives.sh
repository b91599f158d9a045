#!/bin/bash
# Headline step with the RCCL bucket all-reduces kept in at world size 1 (autotuned strategy),
# and its per-kernel profile (collective kernels included).
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
run bench_coll 300 python bench.py --steps 2000 --warmup 100 --force-collectives
run prof_coll 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_coll -o run --output-format csv -- python bench.py --steps 200 --warmup 20 --force-collectives
