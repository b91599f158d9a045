#!/bin/bash
# bias-gradient kernels without 64-bit divides (+ row path for linear layers): numerics + benches
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run t_ops 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_engine.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread
run b_keras 300 python bench.py --model keras_cnn --steps 500 --warmup 50
run b_mlp 300 python bench.py --model mlp --steps 500 --warmup 50
run b_mnist_layers 300 python bench.py --impl layers --steps 500 --warmup 50
run prof_keras 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_keras -o run --output-format csv -- python bench.py --model keras_cnn --steps 200 --warmup 20
