# final gate at HEAD: every GPU test, smoke, the driver's 1-GPU run
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
run suite 1500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run driver 300 python bench.py --steps 20 --warmup 5
