#!/bin/bash
# Round-3: band kernel BN statistics kept in registers over all bands (one partial row per block)
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
run t_nhwc 600 $PT tests/test_gpu_nhwc.py tests/test_gpu_bf16.py
run b_rn256 400 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3
run b_rn32 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 5
run prof_rn 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn -o run --output-format csv -- python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 5 --warmup 2
