#!/bin/bash
# Generic implicit-GEMM LDS swizzle: numerics (ops, fuzz, models), counters, PyramidNet step.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run ops_tests 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread
run model_tests 300 python -u -m pytest tests/test_gpu_parallel.py -x -q --timeout 120 --timeout-method thread -k "vs_torch or keras or mlp"
run pmc_pyr 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_pyr -o run -- python bench.py --model pyramidnet110 --impl layers --steps 3 --warmup 1 --no-graph
run bench_pyr 600 python bench.py --model pyramidnet110 --impl layers --steps 20 --warmup 3
run bench_keras 300 python bench.py --model keras_cnn --impl layers --steps 200 --warmup 20
