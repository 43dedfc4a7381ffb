# new defaults (split 45 %, equal stream priorities) vs the previous ones (RN_MAIN_PRIORITY=1 RN_TUNE=21=50): C2 pairs, C4, C5; then the GPU suite
b() { echo "200 env $1 python bench.py $3 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04o_$2.log 2>&1"; }
O='RN_MAIN_PRIORITY=1 RN_TUNE=21=50'
tools/gpu_steps.sh \
 "$(b RN_X=0 n1)" "$(b "$O" o1)" "$(b RN_X=0 n2)" "$(b "$O" o2)" \
 "$(b RN_X=0 c4n '--model resnext50')" "$(b "$O" c4o '--model resnext50')" \
 "$(b RN_X=0 c5n '--model resnet50_int8')" "$(b "$O" c5o '--model resnet50_int8')" \
 "900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04o_gputest.log 2>&1"
for f in n1 o1 n2 o2 c4n c4o c5n c5o; do echo -n "$f "; tail -n1 gpurun_out/r04o_$f.log | grep -o '"ms_per_step": [0-9.]*'; done
tail -n2 gpurun_out/r04o_gputest.log
