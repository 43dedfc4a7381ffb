# quantizer threshold state folded into the max kernel's last block: int8 tests, C5 layerwise, A/B pairs vs rn_set_tuning 22 = 4
b() { echo "200 env $1 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04ac_$2.log 2>&1"; }
tools/gpu_steps.sh \
 "300 python -u -m pytest tests/test_int8_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ac_kt.log 2>&1" \
 "600 python -u -m pytest tests/test_step_bf16_gpu.py -x -q -k 'int8' --timeout 500 --timeout-method thread > gpurun_out/r04ac_lw.log 2>&1" \
 "300 python -u -m pytest tests/test_step_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04ac_st.log 2>&1" \
 "$(b RN_X=0 n1)" "$(b RN_TUNE=22=4 o1)" "$(b RN_X=0 n2)" "$(b RN_TUNE=22=4 o2)"
tail -n2 gpurun_out/r04ac_kt.log; tail -n2 gpurun_out/r04ac_lw.log; tail -n2 gpurun_out/r04ac_st.log
for f in n1 o1 n2 o2; do echo -n "$f "; tail -n1 gpurun_out/r04ac_$f.log | grep -o '"ms_per_step": [0-9.]*'; done
