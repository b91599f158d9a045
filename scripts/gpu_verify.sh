#!/bin/bash
# Round re-entry check: build (refreshes a stale in-tree .so), full GPU test suite, smoke(),
# default bench (driver contract).
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
run build 900 python -c "import __graft_entry__ as g; g.build()"
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_default 300 python bench.py
