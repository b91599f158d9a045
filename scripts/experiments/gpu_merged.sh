#!/bin/bash
# One all-reduce over the whole MNIST gradient ("one") as a third bucket strategy: engine tests,
# DDP tests (2 ranks sharing the GPU, autotuned), default bench, 2-rank shared bench.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run eng 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_parallel.py tests/test_gpu_peer.py -m gpu -x -q --timeout 120 --timeout-method thread
run b_def 300 python bench.py --steps 2000 --warmup 100
run b_coll 300 python bench.py --steps 2000 --warmup 100 --force-collectives
run b_ws2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29581 bench.py --gpus 2 --steps 1000 --warmup 50
