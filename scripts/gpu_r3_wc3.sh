#!/bin/bash
# Round-3: band weight-gradient kernel for the 3x3 / 64-channel layer (MXDDP_WGRAD_C3=1)
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
run t_nhwc_wc3 600 env MXDDP_WGRAD_C3=1 $PT tests/test_gpu_nhwc.py
run b_rn256_wc3 400 env MXDDP_WGRAD_C3=1 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3
run b_rn256 400 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3
run b_rn32_wc3 300 env MXDDP_WGRAD_C3=1 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 5
run b_rn32 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 5
run prof_wc3 400 env MXDDP_WGRAD_C3=1 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wc3 -o run --output-format csv -- python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 5 --warmup 2
