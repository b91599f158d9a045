#!/bin/bash
# ReplicaGroup per-device hipGraph capture: tests, then replica-mode benches of the reference's
# TF2 / Chainer models with and without graphs.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run build 900 python -c "import __graft_entry__ as g; g.build()"
run pytest_par 300 python -u -m pytest tests/test_gpu_parallel.py -x -q --timeout 120 --timeout-method thread
run replica_keras 300 python bench.py --impl replica --model keras_cnn --steps 300 --warmup 30
run replica_keras_eager 300 python bench.py --impl replica --model keras_cnn --steps 300 --warmup 30 --no-graph
run replica_mlp 300 python bench.py --impl replica --model mlp --steps 300 --warmup 30
run replica_mlp_eager 300 python bench.py --impl replica --model mlp --steps 300 --warmup 30 --no-graph
