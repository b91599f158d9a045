#!/bin/bash
# kernel-trace stats of the Keras CNN and MLP layer-path steps
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run prof_keras 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_keras -o run --output-format csv -- python bench.py --model keras_cnn --steps 200 --warmup 20
run prof_mlp 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mlp -o run --output-format csv -- python bench.py --model mlp --steps 200 --warmup 20
