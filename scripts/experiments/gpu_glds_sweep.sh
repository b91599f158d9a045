#!/bin/bash
# per-layer conv timings at batch 32 with the LDS-DMA kernel on large layers only (1) / everywhere (2)
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
MXDDP_CONV_GLDS=1 run layers_g1 300 python scripts/bench_nhwc_layers.py 32 20
MXDDP_CONV_GLDS=2 run layers_g2 300 python scripts/bench_nhwc_layers.py 32 20
MXDDP_CONV_GLDS=1 run layers64_g1 300 python scripts/bench_nhwc_layers.py 64 10
MXDDP_CONV_GLDS=2 run layers64_g2 300 python scripts/bench_nhwc_layers.py 64 10
