source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
run t_c 600 $T tests/test_gpu_wgrad_defer.py tests/test_gpu_engine.py tests/test_gpu_rccl_diag.py
for i in 1 2; do for d in 1 0; do run rn32_w${d}_$i 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 3 --ab wgrad_defer=$d; done; done
for d in 1 0; do run pyr_w${d}_3 300 python bench.py --model pyramidnet110 --steps 20 --warmup 3 --ab wgrad_defer=$d; done
