#!/bin/bash
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run graphpar 120 python scripts/diag_graph_concurrency.py
