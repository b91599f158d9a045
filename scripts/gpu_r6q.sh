# ResNet-50 bf16: the small-layer rule (<= 25,088 pixels AND >= 32 planes), on / off, both batches
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
run t_nhwc 600 $T tests/test_gpu_nhwc.py tests/test_gpu_wgrad_defer.py
for v in 25088 0 25088 0; do run rn32_s$v 300 python scripts/ab_native.py nhwc_wgrad_set_small_npix=$v -- --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 5; done
for v in 25088 0 25088 0; do run rn256_s$v 300 python scripts/ab_native.py nhwc_wgrad_set_small_npix=$v -- --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3; done
