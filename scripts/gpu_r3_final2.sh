#!/bin/bash
# Round-3 closing check at HEAD: full GPU suite, smoke, driver-length and long MNIST benches, ResNet-50
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_driver 300 python bench.py --steps 20 --warmup 5
run bench_long 300 python bench.py --steps 2000 --warmup 100
run bench_rn32 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 5
run bench_rn256 400 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3
run bench_rn_ws2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29593 bench.py --gpus 2 --model resnet50 --dtype bf16 --batch 32 --steps 10 --warmup 3
