#!/bin/bash
# NHWC BN LDS layout: numerics, counters, ResNet-50 steps at batch 32 and 256.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run nhwc_tests 300 python -u -m pytest tests/test_gpu_nhwc.py -x -q --timeout 120 --timeout-method thread
run pmc_rn 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_rn -o run -- python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 2 --warmup 1 --no-graph
run bench_rn256 300 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3
run bench_rn32 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 10 --warmup 3
