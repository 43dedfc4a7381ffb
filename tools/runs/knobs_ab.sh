# default-knob re-check after round 2's fusions: each variant next to the default, same box
B="python bench.py --no-cpu-baseline --pcie-steps 0"
tools/gpu_steps.sh \
 "120 $B > gpurun_out/kn_def0.log 2>&1" \
 "120 env RN_BN_FUSION_MIN_COLS=64 $B > gpurun_out/kn_min64.log 2>&1" \
 "120 env RN_BN_BWD_FUSION=2 $B > gpurun_out/kn_bwd2.log 2>&1" \
 "120 env RN_BN_EPILOGUE_STATS=2 $B > gpurun_out/kn_st2.log 2>&1" \
 "120 env RN_TUNE=10=1024 $B > gpurun_out/kn_p1024.log 2>&1" \
 "120 $B > gpurun_out/kn_def1.log 2>&1"
