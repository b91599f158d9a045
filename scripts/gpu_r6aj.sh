# the peer GPU tests with the Keras co-scheduled case at 4 shared-GPU ranks (within one GPU's residency)
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
run peer 600 python -u -m pytest tests/test_gpu_peer.py -x -v --timeout 120 --timeout-method thread
