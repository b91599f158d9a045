source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
run phases 300 python scripts/phase_profile.py
