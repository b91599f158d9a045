#!/bin/bash
# Multi-rank rehearsal at the end of round 2 (ranks SHARE the one GPU: peer transport only):
# the fused engine (autotune + graph pre-launch) at 2 ranks with the driver's step counts and at
# 4 ranks, the layer-path DDP at 4 ranks.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
run ws2_driver 300 $TR --nproc-per-node 2 --master-port 29571 bench.py --gpus 2 --steps 20 --warmup 5
run ws4_fused 300 $TR --nproc-per-node 4 --master-port 29572 bench.py --gpus 4 --steps 200 --warmup 20
run ws4_keras 300 $TR --nproc-per-node 4 --master-port 29573 bench.py --model keras_cnn --gpus 4 --steps 50 --warmup 5
