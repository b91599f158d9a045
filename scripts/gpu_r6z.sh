# flaky-check of the withheld-flags autotune scenario (2 ranks sharing the GPU), 8 repetitions
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
run flake 600 python -u scripts/diag_peer_flake.py 8
