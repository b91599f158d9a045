#!/bin/bash
# Round-3 check c: the fused Keras-CNN engine (numerics, graphs, replicas, throughput) and the
# two-rank CLI divergence diagnostic.
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
run t_keras 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_keras_engine.py
run b_keras 200 python scripts/bench_keras_fused.py
run b_keras_long 200 python scripts/bench_keras_fused.py --steps 2000 --warmup 100
run b_keras_eager 200 python scripts/bench_keras_fused.py --no-graph --steps 200
run p_keras 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_keras -o run --output-format csv -- python scripts/bench_keras_fused.py --steps 300
run cli_keras 300 env MXDDP_DEBUG_RANKSUM=1 python -m mxddp.train --model keras_cnn --nproc-per-node 2 -e 1 --steps-per-epoch 20 --log-interval 1 -td /tmp/tdk -sm --per-rank-batch 32
run cli_keras_ng 300 env MXDDP_DEBUG_RANKSUM=1 python -m mxddp.train --model keras_cnn --nproc-per-node 2 -e 1 --steps-per-epoch 20 --log-interval 1 -td /tmp/tdk2 -sm --per-rank-batch 32 --no-graph
run t_multi 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_ddp_multi.py -k bn_semantics
