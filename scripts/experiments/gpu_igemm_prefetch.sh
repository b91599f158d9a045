#!/bin/bash
# generic implicit GEMM with two k-tiles of register prefetch: numerics, then the benches that
# run it (Keras CNN, MLP, MNIST layer path, PyramidNet stem / stride-2 convs, fused variant 0)
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run t_gemm 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fuzz.py tests/test_gpu_engine.py tests/test_gpu_parallel.py -m gpu -x -q --timeout 120 --timeout-method thread
run b_keras 300 python bench.py --model keras_cnn --steps 500 --warmup 50
run b_mlp 300 python bench.py --model mlp --steps 500 --warmup 50
run b_mnist_layers 300 python bench.py --impl layers --steps 500 --warmup 50
run b_v0 300 python bench.py --variant 0 --steps 500 --warmup 50
run b_pyr 300 python bench.py --model pyramidnet110 --steps 20 --warmup 3
run prof_keras 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_keras -o run --output-format csv -- python bench.py --model keras_cnn --steps 200 --warmup 20
