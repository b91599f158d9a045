#!/bin/bash
# Round-end evidence: build, full GPU suite, smoke, the driver's default bench and a long run,
# kernel-trace stats of the MNIST / PyramidNet / ResNet-50 steps, the secondary benches and the
# 2-rank shared-GPU DDP rehearsal.  Logs under gpurun_out/ (copy to profiles/<round>_final/).
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
run build 900 python -c "import __graft_entry__ as g; g.build()"
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_default 300 python bench.py
run bench_driver 300 python bench.py --steps 20 --warmup 5
run bench_long 300 python bench.py --steps 2000 --warmup 100
run prof_mnist 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mnist -o run --output-format csv -- python bench.py --steps 200 --warmup 20
run bench_pyr 300 python bench.py --model pyramidnet110 --steps 20 --warmup 3
run prof_pyr 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pyr -o run --output-format csv -- python bench.py --model pyramidnet110 --steps 5 --warmup 2
run bench_rn32 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 10 --warmup 3
run bench_rn256 300 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3
run prof_rn 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn -o run --output-format csv -- python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 3 --warmup 2
run bench_keras 300 python bench.py --model keras_cnn --steps 300 --warmup 30
run bench_mlp 300 python bench.py --model mlp --steps 300 --warmup 30
run bench_mnist_layers 300 python bench.py --impl layers --steps 300 --warmup 30
run bench_cpu 300 python bench.py --cpu --steps 30 --warmup 3
run bench_replica 300 python bench.py --impl replica --steps 1000 --warmup 50
run bench_coll 300 python bench.py --steps 2000 --warmup 100 --force-collectives
run bench_ws2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29591 bench.py --gpus 2 --steps 1000 --warmup 50
run bench_keras_replica 300 python bench.py --model keras_cnn --impl replica --steps 300 --warmup 30
run bench_ws2_keras 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29592 bench.py --gpus 2 --model keras_cnn --steps 300 --warmup 30
