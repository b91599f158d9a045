#!/bin/bash
# Latent out-of-bounds hunt: every tensor in its own allocation (no caching allocator), so a
# kernel reading past a buffer's end is more likely to touch unmapped memory.
source "$(dirname "$0")/../gpu_check.sh"
rm -f gpurun_out/steps.log
export PYTORCH_NO_CUDA_MEMORY_CACHING=1
run nc_pyr 300 python bench.py --model pyramidnet110 --steps 3 --warmup 2 --no-graph
run nc_ops 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_nhwc.py tests/test_gpu_parallel.py -m gpu -x -q --timeout 120 --timeout-method thread
run nc_rn 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 3 --warmup 2 --no-graph
run nc_mnist 300 python bench.py --steps 200 --warmup 20
