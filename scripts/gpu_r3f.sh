#!/bin/bash
# Round-3 check f: KO with wave-split coalesced plane sums, KB1 per-role timing, MNIST F3
# tiling profiles, layers-path CLI divergence bisection (diag in train.py's step shape).
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
PT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
PS="rocprofv3 --kernel-trace --stats --output-format csv"
run t_keras 600 $PT tests/test_gpu_keras_engine.py
run b_keras 200 python bench.py --model keras_cnn --steps 1000 --warmup 50
run b_keras_rep 200 python bench.py --impl replica --model keras_cnn --steps 1000 --warmup 50
run p_keras 200 $PS -d gpurun_out/p_keras -o run -- python bench.py --model keras_cnn --steps 200 --warmup 20
for r in 1 2 4 8; do run p_kb1_$r 200 env MXDDP_KB1_ROLES=$r $PS -d gpurun_out/p_kb1_$r -o run -- python bench.py --model keras_cnn --steps 100 --warmup 10; done
run p_mnist_144 200 env MXDDP_F3=144 $PS -d gpurun_out/p_mnist_144 -o run -- python bench.py --steps 400 --warmup 20
run p_mnist_256 200 env MXDDP_F3=256x16 $PS -d gpurun_out/p_mnist_256 -o run -- python bench.py --steps 400 --warmup 20
run diag_mimic 300 $TR --nproc-per-node 2 --master-port 29636 scripts/diag_ddp_graph.py --model keras_cnn --steps 12 --graph --mimic
run diag_launch 300 python -m mxddp.launch --nproc-per-node 2 scripts/diag_ddp_graph.py --model keras_cnn --steps 12 --graph
run cli_peer 300 env MXDDP_DEBUG_RANKSUM=1 python -m mxddp.train --model keras_cnn --engine layers --nproc-per-node 2 -e 1 --steps-per-epoch 12 --log-interval 4 --per-rank-batch 32 --transport peer
run cli_tr 300 env MXDDP_DEBUG_RANKSUM=1 $TR --nproc-per-node 2 --master-port 29637 -m mxddp.train --model keras_cnn --engine layers -e 1 --steps-per-epoch 12 --log-interval 4 --per-rank-batch 32
