#!/bin/bash
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run bench_rn_graph 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 3
run bench_rn_eager 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 3 --no-graph
run bench_rn_torch_cl 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 3 --impl torch --channels-last
run bench_pyr_graph 300 python bench.py --model pyramidnet110 --impl layers --steps 20 --warmup 3
run bench_pyr_eager 300 python bench.py --model pyramidnet110 --impl layers --steps 20 --warmup 3 --no-graph
run bench_pyr_torch 300 python bench.py --model pyramidnet110 --impl torch --steps 20 --warmup 3
