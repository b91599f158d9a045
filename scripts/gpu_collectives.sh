#!/bin/bash
# Headline step with the RCCL bucket all-reduces kept in at world size 1, in the SAME launch mode
# as the default run (graph mode 1, 8 steps per graph) and autotuned, plus the default run for
# comparison.  At one rank RCCL runs each bucket all-reduce as a buffer copy, not a collective
# kernel, so the profile shows copyBuffer / fill calls rather than RCCL kernels.
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
run bench_plain 300 python bench.py --steps 2000 --warmup 100
run bench_coll_g1 300 python bench.py --steps 2000 --warmup 100 --force-collectives --graph-mode 1
run bench_coll_auto 300 python bench.py --steps 2000 --warmup 100 --force-collectives
run prof_coll 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_coll -o run --output-format csv -- python bench.py --steps 200 --warmup 20 --force-collectives --graph-mode 1
