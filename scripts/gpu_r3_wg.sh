#!/bin/bash
# Round-3: weight-gradient block target sweep (split count of the NHWC wgrad) for ResNet-50 bf16
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
for nb in 512 256 1024 512; do
  run rn32_wg$nb 300 env MXDDP_WGRAD_BLOCKS=$nb python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 5
done
for nb in 512 256 1024; do
  run rn256_wg$nb 400 env MXDDP_WGRAD_BLOCKS=$nb python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3
done
