#!/bin/bash
# Round-3 check i: the rank-divergence fix (non-differentiable correct count; DDP hook capture
# check) -- the train.py step body at 2 ranks sharing the GPU, torchrun and mxddp.launch.
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
PT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
CLI="-m mxddp.train --model keras_cnn --engine layers -e 1 --steps-per-epoch 8 --log-interval 1 --per-rank-batch 32"
run d_mimic 200 $TR --nproc-per-node 2 --master-port 29641 scripts/diag_ddp_graph.py --model keras_cnn --steps 8 --graph --mimic
run c_tr 200 env MXDDP_DEBUG_RANKSUM=1 $TR --nproc-per-node 2 --master-port 29644 $CLI
run c_launch 200 env MXDDP_DEBUG_RANKSUM=1 python $CLI --nproc-per-node 2
run c_pyr 300 env MXDDP_DEBUG_RANKSUM=1 python -m mxddp.train --model pyramidnet110 --engine layers -e 1 --steps-per-epoch 6 --log-interval 1 --per-rank-batch 8 --nproc-per-node 2
run t_multi 600 $PT tests/test_gpu_ddp_multi.py tests/test_gpu_parallel.py
