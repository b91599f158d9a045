#!/bin/bash
# Replica graphs with a host wait after each replay (before the eager optimizer): throughput and
# the TensorBoard run that diverged without it.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run keras_after 120 env MXDDP_REPLICA_SYNC=after python bench.py --impl replica --model keras_cnn --steps 300 --warmup 30
run keras_plain 120 python bench.py --impl replica --model keras_cnn --steps 300 --warmup 30
run mlp_after 120 env MXDDP_REPLICA_SYNC=after python bench.py --impl replica --model mlp --steps 300 --warmup 30
run mlp_plain 120 python bench.py --impl replica --model mlp --steps 300 --warmup 30
B="python -m mxddp.train --model keras_cnn --optimizer adam --mode replica -b 512 -e 2 --steps-per-epoch 118 --data synthetic --log-interval 40 --lr-step-size 0"
for i in 1 2; do
  run tb_after_$i 120 env MXDDP_REPLICA_GRAPH=1 MXDDP_REPLICA_SYNC=after $B -td gpurun_out/t$i --eval --eval-every 1 --tensorboard-dir gpurun_out/t$i --histogram-freq 1
done
