#!/bin/bash
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run pytest_nhwc 300 python -u -m pytest tests/test_gpu_nhwc.py -m gpu -q --timeout 120 --timeout-method thread
run bench_rn 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 10 --warmup 3
run bench_rn_torch_cl 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 10 --warmup 3 --impl torch --channels-last
run bench_rn_b64 300 python bench.py --model resnet50 --dtype bf16 --batch 64 --steps 10 --warmup 3
run bench_rn_torch_b64 300 python bench.py --model resnet50 --dtype bf16 --batch 64 --steps 10 --warmup 3 --impl torch --channels-last
