#!/bin/bash
# Round-2 re-entry: build + GPU suite + smoke, then the driver-length bench (20 timed / 5 warm-up)
# with and without graph pre-warming and small-first replay order.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run build 900 python -c "import __graft_entry__ as g; g.build()"
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
for i in 1 2; do
  run old_$i 120 env MXDDP_WARM_GRAPHS=0 MXDDP_SMALL_FIRST=0 python bench.py --steps 20 --warmup 5
  run small_$i 120 env MXDDP_WARM_GRAPHS=0 MXDDP_SMALL_FIRST=1 python bench.py --steps 20 --warmup 5
  run warm_$i 120 python bench.py --steps 20 --warmup 5
done
run long 120 python bench.py --steps 2000 --warmup 100
grep -h '"value"' gpurun_out/old_*.log gpurun_out/small_*.log gpurun_out/warm_*.log gpurun_out/long.log | python3 -c "
import sys, json
for l in sys.stdin: d = json.loads(l); print(d['value'], d['ms_per_step'], d['steps'], d['warmup'])" > gpurun_out/warm_summary.txt
run prof_keras 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_keras -o run --output-format csv -- python bench.py --model keras_cnn --steps 100 --warmup 10
run prof_mlp 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mlp -o run --output-format csv -- python bench.py --model mlp --steps 100 --warmup 10
run bench_rn32 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 10 --warmup 3
run bench_rn256 300 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3
