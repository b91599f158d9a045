#!/bin/bash
# Repeat the layers-DDP-over-peer vs global-batch test (one failure at d = 6.8e-5 in the
# round-end run) and the peer numerics tests, printing the deviation each time.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
for i in 1 2 3 4 5 6; do
run ddpl_$i 200 python -u -m pytest tests/test_gpu_peer.py -m gpu -q -s --timeout 120 --timeout-method thread -k ddp_layers
done
run peer_all 300 python -u -m pytest tests/test_gpu_peer.py -m gpu -q -s --timeout 120 --timeout-method thread
