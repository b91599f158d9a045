#!/bin/bash
# Round-3 check b: layer-path DDP at 2 shared-GPU ranks, eager vs whole-step graph (diagnostic),
# the multi-rank tests and the secondary benches after the capture-stream plane fix.
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
run d_eager 200 $TR --master-port 29611 scripts/diag_ddp_graph.py --steps 12
run d_graph 200 $TR --master-port 29612 scripts/diag_ddp_graph.py --steps 12 --graph
run d_graph_fixed 200 $TR --master-port 29613 scripts/diag_ddp_graph.py --steps 12 --graph --loader fixed
run d_graph_ovl0 200 $TR --master-port 29614 scripts/diag_ddp_graph.py --steps 12 --graph --overlap 0
run d_graph_sgd 200 $TR --master-port 29615 scripts/diag_ddp_graph.py --steps 12 --graph --opt sgd
PT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
run t_multi 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_ddp_multi.py tests/test_gpu_parallel.py -k "two_ranks or replica"
run bench_keras 300 python bench.py --model keras_cnn --steps 300 --warmup 30
run bench_mlp 300 python bench.py --model mlp --steps 300 --warmup 30
run bench_keras_rep 300 python bench.py --impl replica --model keras_cnn --steps 300 --warmup 30
run bench_mlp_rep 300 python bench.py --impl replica --model mlp --steps 300 --warmup 30
