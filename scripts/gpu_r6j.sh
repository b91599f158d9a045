# PyramidNet: BN normalise pass folded into the Winograd convs (ops.bn_conv): tests, A/B, profile
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
run t_fold 600 $T tests/test_gpu_bn_fold.py
run t_ops 600 $T tests/test_gpu_ops.py tests/test_gpu_wgrad_defer.py
for d in 1 0 1 0; do run pyr_f$d 300 python bench.py --model pyramidnet110 --steps 30 --warmup 5 --ab bn_fold=$d; done
run prof_pyr 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pyr -o run --output-format csv -- python bench.py --model pyramidnet110 --steps 10 --warmup 3
