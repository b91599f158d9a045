#!/bin/bash
# Memsets replaced by a zero-fill kernel: does the replica-graph divergence go away?  Then the
# GPU suite.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run build 900 python -c "import __graft_entry__ as g; g.build()"
for i in 1 2 3; do
  run diag_none_$i 120 env PYTHONPATH=. python scripts/diag_replica_graph.py none graph
done
B="python -m mxddp.train --model keras_cnn --optimizer adam --mode replica -b 512 -e 2 --steps-per-epoch 118 --data synthetic --log-interval 40 --lr-step-size 0"
run tb_1 120 env MXDDP_REPLICA_GRAPH=1 $B -td gpurun_out/t1 --eval --eval-every 1 --tensorboard-dir gpurun_out/t1 --histogram-freq 1
run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
