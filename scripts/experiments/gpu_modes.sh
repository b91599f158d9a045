#!/bin/bash
# DDP-path cost at world size 1 with real RCCL collectives: eager vs segmented graphs vs one graph.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run m_eager_nocoll 300 python bench.py --steps 2000 --warmup 100 --no-graph
run m_eager_coll 300 python bench.py --steps 2000 --warmup 100 --no-graph --force-collectives
run m_g2_coll 300 python bench.py --steps 2000 --warmup 100 --graph-mode 2 --force-collectives
run m_g1_coll 300 python bench.py --steps 2000 --warmup 100 --graph-mode 1 --force-collectives
run m_g1_coll_spg1 300 python bench.py --steps 2000 --warmup 100 --graph-mode 1 --steps-per-graph 1 --force-collectives
run prof_g2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g2 -o run --output-format csv -- python bench.py --steps 200 --warmup 20 --graph-mode 2 --force-collectives
run prof_eager 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_eager -o run --output-format csv -- python bench.py --steps 200 --warmup 20 --no-graph --force-collectives
