#!/bin/bash
# mxddp vs stock PyTorch-ROCm on the same GPU, same run: every model of the framework.
source "$(dirname "$0")/gpu_check.sh"
[ -n "${KEEP_STEPS:-}" ] || rm -f gpurun_out/steps.log
run cmp_mnist_mx 300 python bench.py --steps 2000 --warmup 100
run cmp_mnist_torch 300 python bench.py --impl torch --steps 500 --warmup 50
run cmp_keras_mx 300 python bench.py --model keras_cnn --steps 500 --warmup 50
run cmp_keras_torch 300 python bench.py --model keras_cnn --impl torch --steps 500 --warmup 50
run cmp_mlp_mx 300 python bench.py --model mlp --steps 500 --warmup 50
run cmp_mlp_torch 300 python bench.py --model mlp --impl torch --steps 500 --warmup 50
run cmp_pyr_mx 300 python bench.py --model pyramidnet110 --steps 20 --warmup 3
run cmp_pyr_torch 300 python bench.py --model pyramidnet110 --impl torch --steps 20 --warmup 3
run cmp_rn32_mx 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 10 --warmup 3
run cmp_rn32_torch 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --impl torch --channels-last --steps 10 --warmup 3
run cmp_rn256_mx 300 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3
run cmp_rn256_torch 300 python bench.py --model resnet50 --dtype bf16 --batch 256 --impl torch --channels-last --steps 10 --warmup 3
