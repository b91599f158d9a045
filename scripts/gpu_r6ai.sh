# final tree after the epoch experiments were reverted: smoke, driver run, the peer GPU tests
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run driver 300 python bench.py --steps 20 --warmup 5
run peer 600 python -u -m pytest tests/test_gpu_peer.py -x -q --timeout 120 --timeout-method thread
