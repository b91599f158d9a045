#!/bin/bash
source "$(dirname "$0")/../gpu_check.sh"
run pytest_gpu 900 python -m pytest tests/test_gpu_ops.py tests/test_gpu_engine.py -m gpu -x -q
run bench_v1 300 python bench.py --steps 1000 --warmup 50
run bench_mode2 300 env MXDDP_GRAPH_MODE=2 python bench.py --steps 1000 --warmup 50
run bench_pyr_layers 600 python bench.py --model pyramidnet110 --impl layers --steps 10 --warmup 3
run bench_pyr_torch 600 python bench.py --model pyramidnet110 --impl torch --steps 10 --warmup 3
run bench_keras_layers 300 python bench.py --model keras_cnn --impl layers --steps 50 --warmup 5
run bench_mlp_layers 300 python bench.py --model mlp --impl layers --steps 50 --warmup 5
run prof_pyr 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pyr -o run --output-format csv -- python bench.py --model pyramidnet110 --impl layers --steps 5 --warmup 2
run pytest_parallel 900 python -m pytest tests/test_gpu_parallel.py -m gpu -x -q
