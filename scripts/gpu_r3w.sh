#!/bin/bash
# Round-3: Keras KF2 load schedule (no in-chain global loads, LDS-only barriers after stores)
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
run t_keras 900 $PT tests/test_gpu_keras_engine.py
for i in 1 2 3; do
  run b_keras_$i 300 python bench.py --model keras_cnn --steps 1000 --warmup 50
done
run prof_keras 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_keras -o run --output-format csv -- python bench.py --model keras_cnn --steps 300 --warmup 30
