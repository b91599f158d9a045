#!/bin/bash
# Winograd weight-gradient LDS swizzle: numerics, per-shape timings, LDS counters, the step.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run ops_tests 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread
run conv 300 python scripts/bench_conv.py --only-wino
run pmc_lds 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_lds -o run -- python scripts/bench_conv.py --only-wino --shapes 146,151,16
run bench_pyr 600 python bench.py --model pyramidnet110 --impl layers --steps 20 --warmup 3
