# Keras kb1 role B: the pooled-conv1 tile staged in one round trip (clamped stores)
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
run t_kr 600 $T tests/test_gpu_keras_engine.py
for i in 1 2 3; do run kr$i 300 python bench.py --model keras_cnn --steps 2000 --warmup 50; done
run prof_kr 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kr -o run --output-format csv -- python bench.py --model keras_cnn --steps 200 --warmup 20 --min-warmup-ms 0
