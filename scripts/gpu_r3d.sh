#!/bin/bash
# Round-3 check d: co-scheduled fc-bucket exchange (tests + 2-rank rehearsal), Keras engine in
# bench.py, the cross-stream fence trace at world size 1, and the layers-path CLI divergence.
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
PT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
run t_co 600 $PT tests/test_gpu_peer.py -k "trainer"
run ws2_auto 300 $TR --nproc-per-node 2 --master-port 29631 bench.py --gpus 2 --steps 200 --warmup 20
run ws2_co 300 $TR --nproc-per-node 2 --master-port 29632 bench.py --gpus 2 --steps 200 --warmup 20 --buckets co --graph-mode 1 --transport peer
run ws2_one 300 $TR --nproc-per-node 2 --master-port 29633 bench.py --gpus 2 --steps 200 --warmup 20 --buckets one --graph-mode 1 --transport peer
run ws4_auto 300 $TR --nproc-per-node 4 --master-port 29634 bench.py --gpus 4 --steps 100 --warmup 10
run tr_ovl 200 rocprofv3 --kernel-trace -d gpurun_out/tr_ovl -o run --output-format csv -- python bench.py --steps 64 --warmup 8 --force-collectives --graph-mode 1 --buckets ovl --steps-per-graph 8
run tr_inl 200 rocprofv3 --kernel-trace -d gpurun_out/tr_inl -o run --output-format csv -- python bench.py --steps 64 --warmup 8 --force-collectives --graph-mode 1 --buckets inl --steps-per-graph 8
run b_ovl 200 python bench.py --steps 1000 --warmup 50 --force-collectives --graph-mode 1 --buckets ovl
run b_inl 200 python bench.py --steps 1000 --warmup 50 --force-collectives --graph-mode 1 --buckets inl
run b_ovl0 200 python bench.py --steps 1000 --warmup 50 --force-collectives --graph-mode 0 --buckets ovl
run b_inl0 200 python bench.py --steps 1000 --warmup 50 --force-collectives --graph-mode 0 --buckets inl
run b_keras 200 python bench.py --model keras_cnn --steps 1000 --warmup 50
run b_keras_rep 200 python bench.py --impl replica --model keras_cnn --steps 1000 --warmup 50
run b_keras_ws2 300 $TR --nproc-per-node 2 --master-port 29635 bench.py --gpus 2 --model keras_cnn --steps 300 --warmup 30
run cli_layers 300 env MXDDP_DEBUG_RANKSUM=1 python -m mxddp.train --model keras_cnn --engine layers --nproc-per-node 2 -e 1 --steps-per-epoch 20 --log-interval 1 -td /tmp/tdk -sm --per-rank-batch 32
run t_all 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
