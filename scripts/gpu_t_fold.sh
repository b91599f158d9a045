source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
run t_fold 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bn_fold.py
