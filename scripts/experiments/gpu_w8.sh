#!/bin/bash
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run bc_default 200 python scripts/bench_conv.py
run bc_nosplit 200 env MXDDP_WINO_SLOTS=0 python scripts/bench_conv.py
run bc_s256 200 env MXDDP_WINO_SLOTS=256 python scripts/bench_conv.py
run bc_s1536 200 env MXDDP_WINO_SLOTS=1536 python scripts/bench_conv.py
