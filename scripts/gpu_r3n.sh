#!/bin/bash
# Round-3: conv1-grad slab count / F3 tiling A/B, phase profiles (ws 1 and the 2-rank co-scheduled exchange)
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
MXDDP_G1_SLABS=64 run t_engine64 600 $PT tests/test_gpu_engine.py
run ph_default 200 python bench.py --phase-profile 30
MXDDP_G1_SLABS=64 run ph_g64 200 python bench.py --phase-profile 30
run b_def 300 python bench.py --steps 2000 --warmup 100
MXDDP_G1_SLABS=32 run b_g32 300 python bench.py --steps 2000 --warmup 100
MXDDP_G1_SLABS=64 run b_g64 300 python bench.py --steps 2000 --warmup 100
MXDDP_G1_SLABS=64 MXDDP_F3=tile8 run b_g64_t8 300 python bench.py --steps 2000 --warmup 100
run b_def2 300 python bench.py --steps 2000 --warmup 100
MXDDP_G1_SLABS=64 run b_g64_2 300 python bench.py --steps 2000 --warmup 100
run ph_co_ws2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29593 bench.py --gpus 2 --buckets co --graph-mode 0 --phase-profile 20
MXDDP_F6W_PRIO=2 run ph_prio2 200 python bench.py --phase-profile 30
MXDDP_F6W_PRIO=2 run b_prio2 300 python bench.py --steps 2000 --warmup 100
MXDDP_F6W_PRIO=2 MXDDP_G1_SLABS=64 run b_prio2_g64 300 python bench.py --steps 2000 --warmup 100
MXDDP_F6W_PRIO=3 MXDDP_G1_SLABS=64 run b_prio3_g64 300 python bench.py --steps 2000 --warmup 100
