#!/bin/bash
# fc1 SGD folded into F5 (world size 1): engine numerics + interleaved A/B + kernel trace.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
run eng 300 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread
run m_fold 300 python bench.py --steps 2000 --warmup 100
run m_nofold 300 env MXDDP_F5_SGD=0 python bench.py --steps 2000 --warmup 100
run m_fold2 300 python bench.py --steps 2000 --warmup 100
run m_nofold2 300 env MXDDP_F5_SGD=0 python bench.py --steps 2000 --warmup 100
run m_fold3 300 python bench.py --steps 2000 --warmup 100
run m_trace 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_fold -o run -- python bench.py --steps 400 --warmup 50
