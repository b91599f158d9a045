#!/bin/bash
# Training CLI in replica mode (graph-captured ReplicaGroup) through the reference's TF2
# MirroredStrategy and Chainer ParallelUpdater entry points, synthetic data.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run build 900 python -c "import __graft_entry__ as g; g.build()"
run tf2_mirror 300 python examples/tensorflow2/mnist_mirror_strategy.py --batch_size 512 --epochs 2 --train_dir gpurun_out/tf2_mirror
run chainer_gpu 300 python examples/chainer/train_mnist_gpu.py --gpu 0 --epoch 1 --out gpurun_out/chainer_gpu
run cli_replica 300 python -m mxddp.train --model keras_cnn --mode replica -b 512 -e 2 --steps-per-epoch 100 --data synthetic -td gpurun_out/cli_replica
run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
