#!/bin/bash
# Split-K partial planes for few-tile GEMMs (Keras / MLP layers): GPU suite, layer-path benches,
# kernel-trace stats of the Keras / MLP / MNIST-layers steps.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run build 900 python -c "import __graft_entry__ as g; g.build()"
run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
run bench_keras 300 python bench.py --model keras_cnn --steps 300 --warmup 30
run bench_mlp 300 python bench.py --model mlp --steps 300 --warmup 30
run bench_mnist_layers 300 python bench.py --impl layers --steps 300 --warmup 30
run bench_mnist_layers_off 300 env MXDDP_SPLITK_PARTIAL=0 python bench.py --impl layers --steps 300 --warmup 30
run bench_pyr 300 python bench.py --model pyramidnet110 --steps 20 --warmup 3
run prof_keras 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_keras -o run --output-format csv -- python bench.py --model keras_cnn --steps 100 --warmup 10
run prof_mlp 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mlp -o run --output-format csv -- python bench.py --model mlp --steps 100 --warmup 10
run prof_mnist_layers 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ml -o run --output-format csv -- python bench.py --impl layers --steps 100 --warmup 10
