#!/bin/bash
# Round-3 check g (re-entry): HEAD state -- smoke, engine tests, F6W co-split A/B (bench + in-kernel
# phase profile), Keras engine, layers-path CLI rank check at 2 ranks sharing the GPU, full suite.
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
PT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
run smoke 300 python __graft_entry__.py smoke
run t_engine 600 $PT tests/test_gpu_engine.py
run b_cos2 200 python bench.py --steps 2000 --warmup 50
run b_cos1 200 env MXDDP_F6W_COS=1 python bench.py --steps 2000 --warmup 50
run b_default 200 python bench.py
run ph_cos2 200 python scripts/phase_profile.py
run ph_cos1 200 env MXDDP_F6W_COS=1 python scripts/phase_profile.py
run b_keras 200 python bench.py --model keras_cnn --steps 1000 --warmup 50
run b_keras_rep 200 python bench.py --impl replica --model keras_cnn --steps 1000 --warmup 50
run cli_peer 300 env MXDDP_DEBUG_RANKSUM=1 python -m mxddp.train --model keras_cnn --engine layers --nproc-per-node 2 -e 1 --steps-per-epoch 12 --log-interval 4 --per-rank-batch 32 --transport peer
run t_all 900 $PT -m gpu tests
