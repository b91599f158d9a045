#!/bin/bash
# Round-3: conv2 weight-gradient per-image slabs (no atomics) -- numerics, DDP path, A/B, phase trace
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
run t_engine 600 $PT tests/test_gpu_engine.py
run t_peer 600 $PT tests/test_gpu_peer.py
run ph_slab 200 python bench.py --phase-profile 30
MXDDP_WSLAB=0 run ph_atomic 200 python bench.py --phase-profile 30
for i in 1 2; do
  run b_slab_$i 300 python bench.py --steps 2000 --warmup 100
  MXDDP_WSLAB=0 run b_atomic_$i 300 python bench.py --steps 2000 --warmup 100
done
run b_drv 300 python bench.py --steps 20 --warmup 5
run prof_slab 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_slab -o run --output-format csv -- python bench.py --steps 200 --warmup 20
run ws2_auto 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29594 bench.py --gpus 2 --steps 200 --warmup 20
