#!/bin/bash
source "$(dirname "$0")/../gpu_check.sh"
run phases 300 python scripts/phase_profile.py 64
MXDDP_MNIST_F7=direct run phases_direct 300 python scripts/phase_profile.py 64
