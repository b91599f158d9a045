#!/bin/bash
# Round-2 check: full GPU suite, smoke, default bench, replica bench, 2-rank shared-GPU DDP bench,
# fused replica training through the CLI.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run build 900 python -c "import __graft_entry__ as g; g.build()"
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_default 300 python bench.py
run bench_replica1 300 python bench.py --impl replica --gpus 1 --steps 500 --warmup 50
run bench_ddp2_shared 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 200 --warmup 20
run train_replica 300 python -m mxddp.train --model mnist_cnn --mode replica -b 64 -e 1 --steps-per-epoch 40 --log-interval 20 -td gpurun_out/td_rep -sm
run train_ddp2_fused 300 python -m mxddp.train --model mnist_cnn --nproc-per-node 2 --per-rank-batch 64 -e 1 --steps-per-epoch 60 --log-interval 30 -td gpurun_out/td_ddp2 -sm
run train_ddp2_layers 300 python -m mxddp.train --model keras_cnn --nproc-per-node 2 --per-rank-batch 32 -e 1 --steps-per-epoch 20 --log-interval 10 -td gpurun_out/td_ddp2k -sm
run bench_peer_os 300 python -u scripts/bench_peer.py --ws 2 --sizes 4096,18816,65536,1181066 --blocks 64 --fences 1 --oneshot 0,262144,1048576
