# ResNet-50 bf16 batch 32 / 256: weight-gradient block target (split-K planes) with the batched flush
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
for t in 512 256 128 512 256 128; do run rn32_t$t 300 python scripts/ab_native.py nhwc_wgrad_set_target=$t -- --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 5; done
for t in 512 256 512 256; do run rn256_t$t 300 python scripts/ab_native.py nhwc_wgrad_set_target=$t -- --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3; done
