#!/bin/bash
# Round-3: layer-path Adam without the arrival ticket (MLP / Keras layer path), full GPU suite
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
run b_mlp 300 python bench.py --model mlp --steps 500 --warmup 50
run b_keras_layers 300 python bench.py --model keras_cnn --impl layers --steps 500 --warmup 50
run b_mlp_rep 300 python bench.py --model mlp --impl replica --steps 500 --warmup 50
run prof_mlp 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mlp -o run --output-format csv -- python bench.py --model mlp --steps 200 --warmup 20
run pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
