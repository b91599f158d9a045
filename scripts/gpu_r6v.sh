# re-entry check of the rebuilt tree: GPU suite, smoke, the driver's 1-GPU run
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
run suite 1200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run driver 300 python bench.py --steps 20 --warmup 5
