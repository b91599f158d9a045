# round gate at HEAD + Winograd forward-variant A/B on PyramidNet's 16x16 / 8x8 shapes
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
run suite 1500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run driver 300 python bench.py --steps 20 --warmup 5
run ws2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 400)) bench.py --gpus 2 --steps 20 --warmup 5
S="106,111,16:126,131,16:146,151,16:161,166,16:181,186,16:191,196,8:211,216,8:231,236,8:251,256,8:266,271,8"
for v in 0 2 3 4; do
  run wino_v$v 300 env MXDDP_WINO_FWD=$v python scripts/bench_conv.py --only-wino --shapes $S
done
