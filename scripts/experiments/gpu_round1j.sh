#!/bin/bash
# BN order test, engine tests, phase profile, bench, ResNet-50 bf16 + torch profiles.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run bn1 300 python -m pytest tests/test_gpu_ops.py -m gpu -q -k batchnorm
run pytest_engine 600 python -m pytest tests/test_gpu_engine.py -m gpu -x -q
run phase 300 env PYTHONPATH=. python scripts/phase_profile.py
run bench_v1 300 python bench.py --steps 2000 --warmup 100
run prof_v1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v1 -o run --output-format csv -- python bench.py --steps 200 --warmup 20
run prof_rn_bf16 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn_bf16 -o run --output-format csv -- python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 3 --warmup 2
run prof_rn_torch 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn_torch -o run --output-format csv -- python bench.py --model resnet50 --impl torch --batch 32 --steps 3 --warmup 2
