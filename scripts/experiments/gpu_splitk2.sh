#!/bin/bash
# Split-K partial planes, second pass (plane cap by output size, unrolled finish): GPU suite,
# the DDP-over-peer deviation with and without the partial planes, layer-path benches.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run build 900 python -c "import __graft_entry__ as g; g.build()"
run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
run ddp_dev_on 300 python -u -m pytest tests/test_gpu_peer.py -k ddp_layers -s -q --timeout 120 --timeout-method thread
run ddp_dev_off 300 env MXDDP_SPLITK_PARTIAL=0 python -u -m pytest tests/test_gpu_peer.py -k ddp_layers -s -q --timeout 120 --timeout-method thread
run bench_keras 300 python bench.py --model keras_cnn --steps 300 --warmup 30
run bench_mlp 300 python bench.py --model mlp --steps 300 --warmup 30
run bench_mnist_layers 300 python bench.py --impl layers --steps 300 --warmup 30
run bench_default 300 python bench.py --steps 20 --warmup 5
run prof_mnist_layers 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ml -o run --output-format csv -- python bench.py --impl layers --steps 100 --warmup 10
