#!/bin/bash
# Round-3: Winograd epilogue operands requested before use (PyramidNet)
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
run t_ops 900 $PT tests/test_gpu_ops.py tests/test_gpu_parallel.py tests/test_gpu_fuzz.py
for i in 1 2; do
  run b_pyr_$i 300 python bench.py --model pyramidnet110 --steps 20 --warmup 3
done
run prof_pyr 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pyr -o run --output-format csv -- python bench.py --model pyramidnet110 --steps 5 --warmup 2
