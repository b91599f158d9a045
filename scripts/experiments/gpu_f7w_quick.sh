#!/bin/bash
source "$(dirname "$0")/../gpu_check.sh"
run pytest_engine 600 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread -k matches_reference
run bench_wino 300 python bench.py --steps 2000 --warmup 100
run phases 300 python scripts/phase_profile.py 64
