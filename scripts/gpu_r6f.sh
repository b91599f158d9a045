source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
run t_f 900 $T tests/test_gpu_engine.py tests/test_gpu_peer.py tests/test_gpu_rccl_diag.py
for d in 0 2 0 2; do run coll_one_d$d 300 python bench.py --steps 200 --warmup 20 --force-collectives --buckets one --ab fc1_defer=$d; done
run ws2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 400)) bench.py --gpus 2 --steps 200 --warmup 20
bash scripts/gpu_r6_pmc.sh
