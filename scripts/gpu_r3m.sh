#!/bin/bash
# Round-3: ResNet-50 / PyramidNet state at HEAD (benches + kernel stats at batch 32 and 256)
source "$(dirname "$0")/gpu_check.sh"
: > /dev/null
run bench_rn32 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 5
run bench_rn256 300 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3
run prof_rn32 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn32 -o run --output-format csv -- python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 10 --warmup 3
run prof_rn 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn -o run --output-format csv -- python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 3 --warmup 2
run bench_pyr 300 python bench.py --model pyramidnet110 --steps 20 --warmup 3
run bench_keras 300 python bench.py --model keras_cnn --steps 1000 --warmup 50
run bench_mlp 300 python bench.py --model mlp --steps 300 --warmup 30
