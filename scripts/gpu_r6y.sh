# Winograd forward at three blocks per CU (MXDDP_WINO_FWD=5, 17 VGPRs spilled) vs the default, per shape
source scripts/gpu_check.sh
rm -f gpurun_out/steps.log
S="16,21,32:56,61,32:96,101,32:106,111,16:126,131,16:146,151,16:161,166,16:181,186,16:191,196,8:211,216,8:231,236,8:251,256,8:266,271,8"
for v in 0 5; do
  run wino_v$v 300 env MXDDP_WINO_FWD=$v python scripts/bench_conv.py --only-wino --shapes $S
done
