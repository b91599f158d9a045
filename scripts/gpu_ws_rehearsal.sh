#!/bin/bash
# Rank-count rehearsal on the one-GPU box: 4 and 8 ranks SHARE the GPU (peer transport only,
# RCCL refuses duplicate GPUs) -- exercises the ws=4/8 code paths of bench.py (fused engine
# autotune, layer-path DDP), not a scaling measurement.  Then the full GPU suite.
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
run ws4_fused 300 $TR --nproc-per-node 4 --master-port 29561 bench.py --gpus 4 --steps 200 --warmup 20
run ws8_fused 300 $TR --nproc-per-node 8 --master-port 29562 bench.py --gpus 8 --steps 200 --warmup 20
run ws4_keras 300 $TR --nproc-per-node 4 --master-port 29563 bench.py --model keras_cnn --gpus 4 --steps 50 --warmup 5
run ws4_pyr 300 $TR --nproc-per-node 4 --master-port 29564 bench.py --model pyramidnet110 --gpus 4 --steps 4 --warmup 2
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
