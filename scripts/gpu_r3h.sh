#!/bin/bash
# Round-3 check h: layers-path rank divergence bisection (2 ranks sharing the GPU, keras_cnn, peer)
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
D="scripts/diag_ddp_graph.py --model keras_cnn --steps 8 --graph --mimic"
run d_corr 200 $TR --nproc-per-node 2 --master-port 29641 $D --parts corr
run d_ev 200 $TR --nproc-per-node 2 --master-port 29642 $D --parts ev
run d_check 200 $TR --nproc-per-node 2 --master-port 29643 $D --parts check
run c_tr 200 env MXDDP_DEBUG_RANKSUM=1 $TR --nproc-per-node 2 --master-port 29644 -m mxddp.train --model keras_cnn --engine layers -e 1 --steps-per-epoch 6 --log-interval 1 --per-rank-batch 32
