#!/bin/bash
# Conv weight gradients on a side stream (eager steps; operands held until the join): the
# PyramidNet eager step first (it faulted with record_stream lifetimes), then numerics and A/B.
source "$(dirname "$0")/../gpu_check.sh"

run pyr_eager_side 300 python bench.py --model pyramidnet110 --impl layers --steps 20 --warmup 3 --no-graph
run pyr_eager_side_long 300 python bench.py --model pyramidnet110 --impl layers --steps 100 --warmup 3 --no-graph
run t_side 300 python -u -m pytest tests/test_gpu_parallel.py -m gpu -x -q --timeout 120 --timeout-method thread
run pyr_graph 300 python bench.py --model pyramidnet110 --impl layers --steps 20 --warmup 3
run pyr_eager_main 300 env MXDDP_SIDE_WGRAD=0 python bench.py --model pyramidnet110 --impl layers --steps 20 --warmup 3 --no-graph
run keras_eager_side 300 python bench.py --model keras_cnn --impl layers --steps 300 --warmup 30 --no-graph
run keras_graph 300 python bench.py --model keras_cnn --impl layers --steps 300 --warmup 30
run pyr2_side 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29571 bench.py --model pyramidnet110 --gpus 2 --steps 6 --warmup 2
run rn_eager_side 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 6 --warmup 3 --no-graph
run rn_graph 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 6 --warmup 3
run rn_eager_main 300 env MXDDP_SIDE_WGRAD=0 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 6 --warmup 3 --no-graph
run t_nhwc 300 python -u -m pytest tests/test_gpu_nhwc.py -m gpu -x -q --timeout 120 --timeout-method thread
