#!/bin/bash
# Round-3: full GPU suite + smoke at HEAD
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
