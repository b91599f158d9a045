#!/bin/bash
# Pipelined F6 conv1 recompute, 1x1 conv GEMM ops: numerics, phase profile, bench, ResNet.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run pytest_engine 600 python -m pytest tests/test_gpu_engine.py tests/test_gpu_ops.py -m gpu -x -q
run phase 300 env PYTHONPATH=. python scripts/phase_profile.py
run bench_v1 300 python bench.py --steps 2000 --warmup 100
run prof_v1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v1 -o run --output-format csv -- python bench.py --steps 200 --warmup 20
run bench_rn_bf16 600 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 6 --warmup 3
run bench_rn_torch_bf16 600 python bench.py --model resnet50 --impl torch --dtype bf16 --batch 32 --steps 6 --warmup 6
run bench_pyr_torch 600 python bench.py --model pyramidnet110 --impl torch --steps 10 --warmup 5
run pytest_parallel 600 python -m pytest tests/test_gpu_parallel.py tests/test_gpu_bf16.py -m gpu -q
