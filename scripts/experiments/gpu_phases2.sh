#!/bin/bash
source "$(dirname "$0")/../gpu_check.sh"
run phases2 300 python scripts/phase_profile.py 64
