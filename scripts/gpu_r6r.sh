# PyramidNet: Winograd weight-gradient blocks aimed at per CU (split planes vs parallelism)
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
for v in 3 2 4 3 2 4; do run pyr_slots$v 300 python scripts/ab_native.py wino_wgrad_set_slots=$v -- --model pyramidnet110 --steps 30 --warmup 5; done
