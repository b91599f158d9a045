# MLP after batching the backward kernels' staging loads: tests, A/B of the W2 deferral, profile
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
run t_mlp 600 $T tests/test_gpu_mlp_engine.py
for d in 1 0 1 0; do run mlp_d$d 300 python bench.py --model mlp --steps 2000 --warmup 50 --ab w2_defer=$d; done
run mlp_coll 300 python bench.py --model mlp --steps 1000 --warmup 50 --force-collectives
for d in 0 1; do run prof_mlp_d$d 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mlp_d$d -o run --output-format csv -- python bench.py --model mlp --steps 200 --warmup 20 --min-warmup-ms 0 --ab w2_defer=$d; done
