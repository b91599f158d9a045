set -e
O=gpurun_out/wt3
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/ -m gpu -k "bn or pyramid" > $O/tests.log 2>&1
for r in 1 2 3; do
  for v in 0 1; do
    timeout -k 10 200 python bench.py --model pyramidnet110 --steps 20 --warmup 3 --ab bn32_wt=$v > $O/pyr_${v}_$r.log 2>&1
  done
done
