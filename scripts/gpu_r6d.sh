source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
run t_d 600 $T tests/test_gpu_wgrad_defer.py
for mb in 0 16 64 256; do run rn32_f$mb 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 3 --ab wgrad_flush_mb=$mb; done
for mb in 0 16 64; do run rn256_f$mb 300 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3 --ab wgrad_flush_mb=$mb; done
for mb in 0 16 64; do run pyr_f$mb 300 python bench.py --model pyramidnet110 --steps 20 --warmup 3 --ab wgrad_flush_mb=$mb; done
run rn32_off 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 3 --ab wgrad_defer=0
