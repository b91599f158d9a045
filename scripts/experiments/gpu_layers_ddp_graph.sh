#!/bin/bash
# Layer-path DDP under hipGraph capture: 2 ranks sharing the GPU (peer transport), graph vs eager,
# and the 1-GPU eager / graph pair.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run pyr1_graph 300 python bench.py --model pyramidnet110 --impl layers --steps 20 --warmup 3
run pyr1_eager 300 python bench.py --model pyramidnet110 --impl layers --steps 20 --warmup 3 --no-graph
run pyr2_graph 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --model pyramidnet110 --impl layers --gpus 2 --steps 20 --warmup 3
run pyr2_eager 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29542 bench.py --model pyramidnet110 --impl layers --gpus 2 --steps 20 --warmup 3 --no-graph
run keras2_graph 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29543 bench.py --model keras_cnn --impl layers --gpus 2 --steps 200 --warmup 20
run ddp_tests 300 python -u -m pytest tests/test_gpu_parallel.py -x -q --timeout 120 --timeout-method thread
