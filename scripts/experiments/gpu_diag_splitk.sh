source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
run diag 120 env PYTHONPATH=. python scripts/diag_splitk.py
run diag_off 120 env PYTHONPATH=. MXDDP_SPLITK_PARTIAL=0 python scripts/diag_splitk.py
