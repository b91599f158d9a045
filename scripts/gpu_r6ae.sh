# final tree: smoke, driver run, the NHWC / engine / wgrad-defer GPU tests
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run driver 300 python bench.py --steps 20 --warmup 5
run tests 900 python -u -m pytest tests/test_gpu_nhwc.py tests/test_gpu_wgrad_defer.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread
