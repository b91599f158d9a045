#!/bin/bash
# ResNet-50 bf16 throughput vs per-GPU batch: mxddp (graph) and stock PyTorch channels_last
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
for b in 64 128 256; do
  run rn_b$b 300 python bench.py --model resnet50 --dtype bf16 --batch $b --steps 10 --warmup 3
  run rn_torch_b$b 300 python bench.py --model resnet50 --dtype bf16 --batch $b --steps 10 --warmup 3 --impl torch --channels-last
done
