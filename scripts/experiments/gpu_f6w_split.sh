#!/bin/bash
source "$(dirname "$0")/../gpu_check.sh"
run pytest_engine 600 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread -k matches_reference
for s in 1 2 3; do MXDDP_F6W_SPLIT=$s run bench_split$s 300 python bench.py --steps 2000 --warmup 100; done
MXDDP_F6W_SPLIT=2 run phases 300 python scripts/phase_profile.py 64
