#!/bin/bash
# Conv bias gradient as an extra GEMM column of the weight gradient: op tests, full suite,
# Keras / MNIST-layers / replica benches.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run build 900 python -c "import __graft_entry__ as g; g.build()"
run pytest_ops 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread
run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
run bench_keras 120 python bench.py --model keras_cnn --steps 300 --warmup 30
run bench_mnist_layers 120 python bench.py --impl layers --steps 300 --warmup 30
run bench_replica_keras 120 python bench.py --impl replica --model keras_cnn --steps 300 --warmup 30
run bench_pyr 300 python bench.py --model pyramidnet110 --steps 20 --warmup 3
