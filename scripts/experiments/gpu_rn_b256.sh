#!/bin/bash
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run pytest_glds 200 python -u -m pytest tests/test_gpu_nhwc.py -m gpu -q -k "glds or conv_nhwc or resnet" --timeout 120 --timeout-method thread
run rn_b256 300 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3
MXDDP_CONV_GLDS=0 run rn_b256_noglds 300 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3
run layers_b256 300 python scripts/bench_nhwc_layers.py 256 5
