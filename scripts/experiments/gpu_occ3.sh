#!/bin/bash
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run conv_occ2 300 python scripts/bench_conv.py --only-wino --shapes 106,111,16:126,131,16:146,151,16:161,166,16:181,186,16
run conv_occ3 300 env MXDDP_WINO_OCC3=1 python scripts/bench_conv.py --only-wino --shapes 106,111,16:126,131,16:146,151,16:161,166,16:181,186,16
