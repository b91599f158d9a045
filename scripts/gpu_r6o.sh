# ResNet-50 bf16 batch 32: which layers gain from half the weight-gradient block target
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
for v in 6272 25088 100352 0 6272 25088 100352 0; do run rn32_s$v 300 python scripts/ab_native.py nhwc_wgrad_set_small_npix=$v -- --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 5; done
