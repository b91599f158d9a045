#!/bin/bash
# Round-3 check k: stalled-replica fast failure, TensorBoard profile_batch device trace
source "$(dirname "$0")/gpu_check.sh"
rm -f gpurun_out/steps.log
PT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
run t_new 600 $PT tests/test_gpu_peer.py -k "stalled or in_process" tests/test_gpu_keras_engine.py -k "stalled or in_process or profile_batch"
