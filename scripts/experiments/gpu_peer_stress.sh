#!/bin/bash
# Try to reproduce the rare layers-DDP-over-peer deviation: the test repeated, two instances at
# a time (4 processes on the GPU) so the ranks' timing is perturbed.  Prints the deviation.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 200 python -u -m pytest tests/test_gpu_peer.py -m gpu -q -s --timeout 120 --timeout-method thread -k ddp_layers > gpurun_out/stress_a$i.log 2>&1 &
  pa=$!
  timeout -k 10 200 python -u -m pytest tests/test_gpu_peer.py -m gpu -q -s --timeout 120 --timeout-method thread -k "ddp_layers or burst" > gpurun_out/stress_b$i.log 2>&1
  rb=$?
  wait $pa; ra=$?
  echo "iter $i: rc $ra $rb $(grep -ho 'max |ddp - global batch| = [0-9.e-]*' gpurun_out/stress_a$i.log gpurun_out/stress_b$i.log | tr '\n' ' ')" | tee -a gpurun_out/steps.log
  if [ $ra -gt 1 ] || [ $rb -gt 1 ]; then echo "stopping"; exit 1; fi
done
