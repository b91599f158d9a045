# MLP: dW2 tile + Adam as resident blocks of K5 (mlp_set_w2_defer): tests, A/B, profile
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
run t_mlp 600 $T tests/test_gpu_mlp_engine.py
for d in 1 0 1 0; do run mlp_d$d 300 python bench.py --model mlp --steps 2000 --warmup 50 --ab w2_defer=$d; done
for d in 1 0; do run mlp_coll_d$d 300 python bench.py --model mlp --steps 1000 --warmup 50 --force-collectives --buckets one --ab w2_defer=$d; done
run prof_mlp 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mlp -o run --output-format csv -- python bench.py --model mlp --steps 200 --warmup 20 --min-warmup-ms 0
