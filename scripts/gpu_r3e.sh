#!/bin/bash
# Round-3 check e: F67 LDS fix (co-scheduled peer block), optimized Keras kernels (KO plan,
# role-E LDS staging, 512-thread KF1/KF2), 2/4-rank rehearsal, ws=1 bucket-strategy traces,
# layers-path CLI divergence bisection.
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
PT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
run t_keras 600 $PT tests/test_gpu_keras_engine.py
run t_co 600 $PT tests/test_gpu_peer.py -k "trainer"
run b_keras 200 python bench.py --model keras_cnn --steps 1000 --warmup 50
run p_keras 200 rocprofv3 --kernel-trace --stats -d gpurun_out/p_keras -o run --output-format csv -- python bench.py --model keras_cnn --steps 200 --warmup 20
run b_mnist 200 python bench.py --steps 1000 --warmup 50
run ws2_auto 300 $TR --nproc-per-node 2 --master-port 29631 bench.py --gpus 2 --steps 200 --warmup 20
run ws2_co 300 $TR --nproc-per-node 2 --master-port 29632 bench.py --gpus 2 --steps 200 --warmup 20 --buckets co --graph-mode 1 --transport peer
run ws2_one 300 $TR --nproc-per-node 2 --master-port 29633 bench.py --gpus 2 --steps 200 --warmup 20 --buckets one --graph-mode 1 --transport peer
run ws4_auto 300 $TR --nproc-per-node 4 --master-port 29634 bench.py --gpus 4 --steps 100 --warmup 10
run tr_ovl 200 rocprofv3 --kernel-trace -d gpurun_out/tr_ovl -o run --output-format csv -- python bench.py --steps 64 --warmup 8 --force-collectives --graph-mode 1 --buckets ovl --steps-per-graph 8
run tr_inl 200 rocprofv3 --kernel-trace -d gpurun_out/tr_inl -o run --output-format csv -- python bench.py --steps 64 --warmup 8 --force-collectives --graph-mode 1 --buckets inl --steps-per-graph 8
run b_ovl 200 python bench.py --steps 1000 --warmup 50 --force-collectives --graph-mode 1 --buckets ovl
run b_inl 200 python bench.py --steps 1000 --warmup 50 --force-collectives --graph-mode 1 --buckets inl
run cli_ng 300 env MXDDP_DEBUG_RANKSUM=1 python -m mxddp.train --model keras_cnn --engine layers --nproc-per-node 2 -e 1 --steps-per-epoch 12 --log-interval 1 --per-rank-batch 32 --no-graph
run cli_g5 300 env MXDDP_DEBUG_RANKSUM=1 python -m mxddp.train --model keras_cnn --engine layers --nproc-per-node 2 -e 1 --steps-per-epoch 12 --log-interval 4 --per-rank-batch 32
run diag_g 300 $TR --nproc-per-node 2 --master-port 29636 scripts/diag_ddp_graph.py --model keras_cnn --steps 12 --graph
for v in 576x32 576x16 384x16 256x16; do run b_f3_$v 200 env MXDDP_F3=$v python bench.py --steps 2000 --warmup 50; done
run b_f3_144 200 env MXDDP_F3=144 python bench.py --steps 2000 --warmup 50
for s in 2 3; do run b_f6s$s 200 env MXDDP_F6W_SPLIT=$s python bench.py --steps 2000 --warmup 50; done
