#!/bin/bash
# Replica-mode divergence hunt: graph vs eager, with / without the per-epoch evaluation.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run build 900 python -c "import __graft_entry__ as g; g.build()"
A="python -m mxddp.train --model keras_cnn --optimizer adam --mode replica -b 512 -e 3 --steps-per-epoch 118 --data synthetic --log-interval 40"
run g_eval 120 $A --eval --eval-every 1 -td gpurun_out/a
run e_eval 120 $A --eval --eval-every 1 --no-graph -td gpurun_out/b
run g_noeval 120 $A -td gpurun_out/c
run e_noeval 120 $A --no-graph -td gpurun_out/d
