#!/bin/bash
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run diag_pyr 180 env PYTHONPATH=. python scripts/diag_copies2.py pyramidnet110 fp32
run diag_rn 180 env PYTHONPATH=. python scripts/diag_copies2.py resnet50 bf16
