# MNIST: XCD-aware F67 block placement (mnist_set_f67_order) -- tests + interleaved A/B
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
run t_eng 600 $T tests/test_gpu_engine.py
for v in 1 0 1 0 1 0; do run mn_o$v 300 python bench.py --ab f67_order=$v; done
for v in 1 0 1 0; do run mnl_o$v 300 python bench.py --steps 2000 --warmup 100 --ab f67_order=$v; done
