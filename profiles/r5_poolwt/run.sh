set -e
O=gpurun_out/wt7
mkdir -p $O
timeout -k 10 300 python -u -c "import sys, pytest; from mxddp import native; native().nhwc_pool_set_wt(1); sys.exit(pytest.main(['-x', '-q', '--timeout', '120', '--timeout-method', 'thread', 'tests/test_gpu_nhwc.py', '-m', 'gpu', '-k', 'pool']))" > $O/tests.log 2>&1
for r in 1 2 3; do
  for v in 0 1; do
    timeout -k 10 200 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 30 --warmup 5 --ab pool_wt=$v > $O/rn32_${v}_$r.log 2>&1
    timeout -k 10 200 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 20 --warmup 3 --ab pool_wt=$v > $O/rn256_${v}_$r.log 2>&1
  done
done
