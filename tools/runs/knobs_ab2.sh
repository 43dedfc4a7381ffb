# BN fusion coverage knobs after the per-tile partials: each variant next to the default, same box
B="python bench.py --no-cpu-baseline --pcie-steps 0"
tools/gpu_steps.sh \
 "120 $B > gpurun_out/k2_def0.log 2>&1" \
 "120 env RN_BN_EPILOGUE_STATS=2 $B > gpurun_out/k2_st2.log 2>&1" \
 "120 env RN_BN_EPILOGUE_STATS=2 RN_BN_BWD_FUSION=2 RN_BN_FUSION_MIN_COLS=64 $B > gpurun_out/k2_all.log 2>&1" \
 "120 $B > gpurun_out/k2_def1.log 2>&1" \
 "120 env RN_BN_EPILOGUE_STATS=2 $B > gpurun_out/k2_st2b.log 2>&1" \
 "120 env RN_BN_EPILOGUE_STATS=2 RN_BN_BWD_FUSION=2 RN_BN_FUSION_MIN_COLS=64 $B > gpurun_out/k2_allb.log 2>&1"
