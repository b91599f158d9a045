#!/bin/bash
# Round-3 check j: output-tiled split-K F3 (default) vs the 144-chunk / 256x16 kernels
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
PT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
PS="rocprofv3 --kernel-trace --stats --output-format csv"
run t_engine 600 $PT tests/test_gpu_engine.py
run b_tile 200 python bench.py --steps 2000 --warmup 50
run b_144 200 env MXDDP_F3=144 python bench.py --steps 2000 --warmup 50
run b_256 200 env MXDDP_F3=256x16 python bench.py --steps 2000 --warmup 50
run b_tile2 200 python bench.py --steps 2000 --warmup 50
run b_drv 200 python bench.py --steps 20 --warmup 5
run p_tile 200 $PS -d gpurun_out/p_tile -o run -- python bench.py --steps 400 --warmup 20
run ph_tile 200 python scripts/phase_profile.py
