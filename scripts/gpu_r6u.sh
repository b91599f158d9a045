# ResNet-50: LDS-tiled 3x3 forward weight repack -- tests, bench, kernel time
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
run t_nhwc 600 $T tests/test_gpu_nhwc.py tests/test_gpu_bf16.py tests/test_gpu_bf16_numerics.py
for i in 1 2; do run rn32_$i 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 5; done
run rn256 300 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3
run prof_rn32 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn32 -o run --output-format csv -- python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 10 --warmup 2 --min-warmup-ms 0
