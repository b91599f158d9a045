#!/bin/bash
# One-block-per-channel BN (small channels) vs split BN: numerics, then PyramidNet A/B.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run build 900 python -c "import __graft_entry__ as g; g.build()"
run bn_tests 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fuzz.py -m gpu -x -q -k "batchnorm or batch_norm" --timeout 120 --timeout-method thread
run pyr_fused 300 python bench.py --model pyramidnet110 --impl layers --steps 20 --warmup 3
run pyr_split 300 env MXDDP_BN_FUSED_MAX=0 python bench.py --model pyramidnet110 --impl layers --steps 20 --warmup 3
run pyr_fused2 300 python bench.py --model pyramidnet110 --impl layers --steps 20 --warmup 3
run pyr_f4k 300 env MXDDP_BN_FUSED_MAX=4096 python bench.py --model pyramidnet110 --impl layers --steps 20 --warmup 3
