#!/bin/bash
# Round-3 first GPU check: the changed / new GPU tests first, then the whole suite and benches.
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
PT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
run t_new 900 $PT tests/test_gpu_ops.py -k "scratch or sgd_adam" tests/test_gpu_parallel.py tests/test_gpu_engine.py -k "bench_json or replica or ddp_reducer or scratch or sgd_adam or variant or autotune"
run t_multi 900 $PT tests/test_gpu_ddp_multi.py
run t_all 1200 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
run bench_default 300 python bench.py --steps 20 --warmup 5
run bench_keras 300 python bench.py --model keras_cnn --steps 300 --warmup 30
run bench_keras_rep 300 python bench.py --impl replica --model keras_cnn --steps 300 --warmup 30
run bench_mlp_rep 300 python bench.py --impl replica --model mlp --steps 300 --warmup 30
run bench_rn_ws2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29593 bench.py --gpus 2 --model resnet50 --dtype bf16 --batch 32 --steps 10 --warmup 3
run bench_keras_ws2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29594 bench.py --gpus 2 --model keras_cnn --steps 200 --warmup 20
