# C4 (ResNeXt-50) BN fusion coverage knobs, each next to the default
B="python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0"
tools/gpu_steps.sh \
 "150 $B > gpurun_out/c4k_def.log 2>&1" \
 "150 env RN_BN_FUSION_MIN_COLS=64 $B > gpurun_out/c4k_m64.log 2>&1" \
 "150 env RN_BN_FUSION_MIN_COLS=64 RN_BN_BWD_FUSION=2 RN_BN_EPILOGUE_STATS=2 $B > gpurun_out/c4k_all.log 2>&1" \
 "150 $B > gpurun_out/c4k_def2.log 2>&1"
