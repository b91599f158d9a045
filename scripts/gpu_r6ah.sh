# device-scope (agent) per-block peer epoch accesses: the peer GPU tests twice, the withheld-flags scenario x8, 2-rank bench x2
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
run peer1 600 python -u -m pytest tests/test_gpu_peer.py -x -q --timeout 120 --timeout-method thread
run peer2 600 python -u -m pytest tests/test_gpu_peer.py tests/test_gpu_replicas8.py -x -q --timeout 120 --timeout-method thread
run flake 600 python -u scripts/diag_peer_flake.py 8
run ws2a 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 400)) bench.py --gpus 2 --steps 20 --warmup 5
run ws2b 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 400)) bench.py --gpus 2 --steps 20 --warmup 5
