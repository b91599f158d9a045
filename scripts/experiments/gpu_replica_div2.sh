#!/bin/bash
# Replica-mode divergence hunt, part 2: the TF2 MirroredStrategy flag set, graph vs eager, and
# with the TensorBoard / checkpoint extensions removed one group at a time.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run build 900 python -c "import __graft_entry__ as g; g.build()"
B="python -m mxddp.train --model keras_cnn --optimizer adam --mode replica -b 512 -e 2 --steps-per-epoch 118 --data synthetic --log-interval 40 --eval --eval-every 1 --lr-step-size 0"
run full 120 $B -td gpurun_out/f1 --save-every 1 --tensorboard-dir gpurun_out/f1 --histogram-freq 1 --summary --epoch-checkpoints
run full_eager 120 $B -td gpurun_out/f2 --save-every 1 --tensorboard-dir gpurun_out/f2 --histogram-freq 1 --summary --epoch-checkpoints --no-graph
run no_tb 120 $B -td gpurun_out/f3 --save-every 1 --summary --epoch-checkpoints
run no_ckpt 120 $B -td gpurun_out/f4 --tensorboard-dir gpurun_out/f4 --histogram-freq 1 --summary
run no_summary 120 $B -td gpurun_out/f5 --save-every 1 --tensorboard-dir gpurun_out/f5 --histogram-freq 1 --epoch-checkpoints
