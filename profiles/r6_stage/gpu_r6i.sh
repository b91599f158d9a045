# MNIST: fc1 resident blocks' staging in one round trip; tests + driver-length and long runs
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
run t_mn 600 $T tests/test_gpu_engine.py -k "deferred or fused"
for i in 1 2 3; do run mn_drv$i 300 python bench.py; done
run mn_long 300 python bench.py --steps 2000 --warmup 50
run mn_d0 300 python bench.py --ab fc1_defer=0
run prof_mn 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mn -o run --output-format csv -- python bench.py --steps 200 --warmup 20 --min-warmup-ms 0
run t_kr 600 $T tests/test_gpu_keras_engine.py
for i in 1 2; do run kr$i 300 python bench.py --model keras_cnn --steps 2000 --warmup 50; done
run prof_kr 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kr -o run --output-format csv -- python bench.py --model keras_cnn --steps 200 --warmup 20 --min-warmup-ms 0
