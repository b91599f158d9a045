#!/bin/bash
# Replica mode (one process, MirroredStrategy / ParallelUpdater parity) on the reference's own
# TF2 and Chainer models; the linear dy-mask kernel test.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run build 900 python -c "import __graft_entry__ as g; g.build()"
run pytest_mask 300 python -u -m pytest tests/test_gpu_ops.py -k "dy_mask or linear" -q --timeout 120 --timeout-method thread
run replica_keras 300 python bench.py --impl replica --model keras_cnn --steps 300 --warmup 30
run replica_mlp 300 python bench.py --impl replica --model mlp --steps 300 --warmup 30
