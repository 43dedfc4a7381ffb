# main-stream priority x split 45/50 (C2 pairs), then C4/C5 priority pairs
b() { echo "200 env $1 python bench.py $3 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04n_$2.log 2>&1"; }
tools/gpu_steps.sh \
 "$(b RN_X=0 d1)" "$(b RN_MAIN_PRIORITY=0 np1)" "$(b 'RN_MAIN_PRIORITY=0 RN_TUNE=21=45' np45a)" "$(b RN_TUNE=21=45 s45)" \
 "$(b RN_X=0 d2)" "$(b RN_MAIN_PRIORITY=0 np2)" "$(b 'RN_MAIN_PRIORITY=0 RN_TUNE=21=45' np45b)" "$(b 'RN_MAIN_PRIORITY=0 RN_TUNE=21=40' np40)" \
 "$(b RN_X=0 c4d '--model resnext50')" "$(b RN_MAIN_PRIORITY=0 c4np '--model resnext50')" \
 "$(b RN_X=0 c5d '--model resnet50_int8')" "$(b RN_MAIN_PRIORITY=0 c5np '--model resnet50_int8')"
for f in d1 np1 np45a s45 d2 np2 np45b np40 c4d c4np c5d c5np; do echo -n "$f "; tail -n1 gpurun_out/r04n_$f.log | grep -o '"ms_per_step": [0-9.]*'; done
