source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
run t_new 600 $T tests/test_gpu_nhwc.py -k "gk2 or half_resolution or glds_deep or bn_backward_statistics" tests/test_gpu_rccl_diag.py
for g in 0 1 2; do GK2=$g run layers_g$g 300 python scripts/bench_nhwc_layers.py 256 5; done
for g in 0 2 1 0; do run rn256_g$g 300 python bench.py --model resnet50 --dtype bf16 --batch 256 --steps 10 --warmup 3 --ab gk2=$g; done
for g in 0 2 1; do run rn32_g$g 300 python bench.py --model resnet50 --dtype bf16 --batch 32 --steps 20 --warmup 3 --ab gk2=$g; done
