# ResNet-50 bf16 batch 256: the small-layer rule at 25,088 pixels (only the 7 x 7 stage qualifies)
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
for v in 25088 0 25088 0; do run rn256_s$v 300 python scripts/ab_native.py nhwc_wgrad_set_small_npix=$v -- --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3; done
