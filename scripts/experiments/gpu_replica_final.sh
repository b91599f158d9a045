#!/bin/bash
# Replica graphs on by default again (memset nodes removed): the TF2 MirroredStrategy example and
# the TensorBoard CLI runs that diverged before, plus the replica benches.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run tf2_mirror 300 python examples/tensorflow2/mnist_mirror_strategy.py --batch_size 512 --epochs 3 --train_dir gpurun_out/tf2_mirror
B="python -m mxddp.train --model keras_cnn --optimizer adam --mode replica -b 512 -e 3 --steps-per-epoch 118 --data synthetic --log-interval 40 --lr-step-size 0"
for i in 1 2; do
  run tb_$i 120 $B -td gpurun_out/t$i --eval --eval-every 1 --tensorboard-dir gpurun_out/t$i --histogram-freq 1
done
run replica_keras 120 python bench.py --impl replica --model keras_cnn --steps 300 --warmup 30
run replica_mlp 120 python bench.py --impl replica --model mlp --steps 300 --warmup 30
run bench_keras 120 python bench.py --model keras_cnn --steps 300 --warmup 30
