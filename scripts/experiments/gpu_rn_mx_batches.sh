source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
run rn_b256 300 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3
run rn_b128 300 python bench.py --model resnet50 --dtype bf16 --batch 128 --steps 10 --warmup 3
run rn_b64 300 python bench.py --model resnet50 --dtype bf16 --batch 64 --steps 10 --warmup 3
