#!/bin/bash
# Round-3: branch-free 3x3/2 max-pool backward (ResNet stem pool)
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
run t_nhwc 600 $PT tests/test_gpu_nhwc.py
run b_rn256 400 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3
run prof_rn256 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn256 -o run --output-format csv -- python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 5 --warmup 2
