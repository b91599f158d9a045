#!/bin/bash
# Full GPU suite + smoke + default bench on the current tree, then the replica-graph divergence
# hunt, part 3: which extension triggers it, and whether the split-K planes are involved.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run build 900 python -c "import __graft_entry__ as g; g.build()"
run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_driver 300 python bench.py --steps 20 --warmup 5
B="python -m mxddp.train --model keras_cnn --optimizer adam --mode replica -b 512 -e 2 --steps-per-epoch 118 --data synthetic --log-interval 40 --lr-step-size 0"
for i in 1 2; do
  run tb_eval_$i 120 env MXDDP_REPLICA_GRAPH=1 $B -td gpurun_out/t$i --eval --eval-every 1 --tensorboard-dir gpurun_out/t$i --histogram-freq 1
  run tb_eval_nosplit_$i 120 env MXDDP_REPLICA_GRAPH=1 MXDDP_SPLITK_PARTIAL=0 $B -td gpurun_out/u$i --eval --eval-every 1 --tensorboard-dir gpurun_out/u$i --histogram-freq 1
  run tb_only_$i 120 env MXDDP_REPLICA_GRAPH=1 $B -td gpurun_out/v$i --tensorboard-dir gpurun_out/v$i --histogram-freq 1
  run eval_only_$i 120 env MXDDP_REPLICA_GRAPH=1 $B -td gpurun_out/w$i --eval --eval-every 1
done
