#!/bin/bash
# ReLU mask applied on load in the linear backward vs a separate relu_bwd pass (same run,
# interleaved): MLP and Keras CNN.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
for i in 1 2; do
  run mlp_on_$i 120 python bench.py --model mlp --steps 300 --warmup 30
  run mlp_off_$i 120 env MXDDP_RELU_ON_LOAD=0 python bench.py --model mlp --steps 300 --warmup 30
  run keras_on_$i 120 python bench.py --model keras_cnn --steps 300 --warmup 30
  run keras_off_$i 120 env MXDDP_RELU_ON_LOAD=0 python bench.py --model keras_cnn --steps 300 --warmup 30
done
