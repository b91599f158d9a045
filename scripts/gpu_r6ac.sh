# bench metrics read before the diagnosis pass: the diag tests and the 2-rank run
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
run diag 600 python -u -m pytest tests/test_gpu_rccl_diag.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread
run ws2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 400)) bench.py --gpus 2 --steps 20 --warmup 5
run driver 300 python bench.py --steps 20 --warmup 5
