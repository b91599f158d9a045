#!/bin/bash
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run debug_nhwc 300 python scripts/debug_nhwc.py 128
