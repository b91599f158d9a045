# ResNet-50 bf16: half the weight-gradient block target on layers of <= 100,352 pixels (rule on / off)
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
for v in 100352 0 100352 0; do run rn32_s$v 300 python scripts/ab_native.py nhwc_wgrad_set_small_npix=$v -- --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 5; done
for v in 100352 0 100352 0; do run rn256_s$v 300 python scripts/ab_native.py nhwc_wgrad_set_small_npix=$v -- --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3; done
