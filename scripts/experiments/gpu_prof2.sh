#!/bin/bash
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run bench_pyr 300 python bench.py --model pyramidnet110 --impl layers --steps 10 --warmup 3
run prof_pyr 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pyr -o run --output-format csv -- python bench.py --model pyramidnet110 --impl layers --steps 5 --warmup 2
run bench_rn 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 6 --warmup 3
run bench_rn_torch 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 6 --warmup 3 --impl torch
run prof_rn 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn -o run --output-format csv -- python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 4 --warmup 2
