# final gate at HEAD: every GPU test, smoke, the driver's 1-GPU run, a 2,000-step MNIST run, the 2-rank shared-GPU run
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
run suite 1500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run driver 300 python bench.py --steps 20 --warmup 5
run long 300 python bench.py --steps 2000 --warmup 50
run ws2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 400)) bench.py --gpus 2 --steps 20 --warmup 5
