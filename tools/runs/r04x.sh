# int8 quantizer pass with two rows' loads per iteration: its kernel tests, C5 layerwise small, A/B vs rn_set_tuning 22 = 2
b() { echo "200 env $1 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04x_$2.log 2>&1"; }
tools/gpu_steps.sh \
 "300 python -u -m pytest tests/test_int8_gpu.py -x -q -k 'codes_bn' --timeout 120 --timeout-method thread > gpurun_out/r04x_kt.log 2>&1" \
 "300 python -u -m pytest tests/test_step_bf16_gpu.py -x -q -k 'int8_layerwise_small' --timeout 300 --timeout-method thread > gpurun_out/r04x_lw.log 2>&1" \
 "$(b RN_X=0 n1)" "$(b RN_TUNE=22=2 o1)" "$(b RN_X=0 n2)" "$(b RN_TUNE=22=2 o2)" \
 "300 bash tools/prof_bench.sh r04x --model resnet50_int8 --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0"
tail -n2 gpurun_out/r04x_kt.log; tail -n2 gpurun_out/r04x_lw.log
for f in n1 o1 n2 o2; do echo -n "$f "; tail -n1 gpurun_out/r04x_$f.log | grep -o '"ms_per_step": [0-9.]*'; done
python tools/step_breakdown.py gpurun_out/prof_r04x/run_kernel_trace.csv | grep bnq
