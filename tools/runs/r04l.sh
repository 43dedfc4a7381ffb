# re-check the opt-in knobs under the half-chip weight-gradient grids (C2 pairs against the default)
b() { echo "200 env $1 python bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04l_$2.log 2>&1"; }
tools/gpu_steps.sh \
 "$(b RN_X=0 d1)" "$(b RN_BN_FUSION_MIN_COLS=64 mc64)" "$(b RN_BN_APPLY_FUSION_3X3=1 act2)" "$(b RN_TUNE=19=2 band2)" \
 "$(b RN_X=0 d2)" "$(b RN_TUNE=19=1 band1)" "$(b RN_BN_BWD_RECOMPUTE=1 recomp)" "$(b RN_TUNE=10=0 nopersist)" \
 "$(b RN_X=0 d3)" "$(b RN_BN_FUSION_MIN_COLS=64 mc64b)" "$(b RN_BN_APPLY_FUSION_3X3=1 act2b)" "$(b RN_TUNE=19=2 band2b)" \
 "$(b RN_X=0 d4)" "$(b RN_TUNE=19=1 band1b)" "$(b RN_TUNE=10=0 nopersistb)" "$(b RN_STEM_CHUNKS=1 chunks1)"
for f in d1 mc64 act2 band2 d2 band1 recomp nopersist d3 mc64b act2b band2b d4 band1b nopersistb chunks1; do echo -n "$f "; tail -n1 gpurun_out/r04l_$f.log | grep -o '"ms_per_step": [0-9.]*'; done
