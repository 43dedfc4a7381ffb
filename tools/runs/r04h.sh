# unit-tail backward in the next unit's conv1 data gradient (rn_conv_bwd_data_relu_bnred): tests, C4 layerwise, C4 A/B
tools/gpu_steps.sh \
 "400 python -u -m pytest tests/test_kernels_gpu.py -k 'relu_bnred or maxpool or dgrad_bn_backward or bnstats or big_tiles or bnrelu_on_load' -x -q --timeout 300 --timeout-method thread > gpurun_out/r04h_tests.log 2>&1" \
 "600 python -u -m pytest tests/test_step_bf16_gpu.py -k 'resnext50 or cifar' -x -v -s --timeout 500 --timeout-method thread > gpurun_out/r04h_layerwise.log 2>&1" \
 "200 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04h_c4_a.log 2>&1" \
 "200 env RN_RELU_BNRED_DGRAD=0 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04h_c4_b.log 2>&1" \
 "200 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04h_c4_a2.log 2>&1" \
 "200 env RN_RELU_BNRED_DGRAD=0 python bench.py --model resnext50 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04h_c4_b2.log 2>&1" \
 "300 bash tools/prof_bench.sh r04h_c4 --model resnext50 --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04h_prof_c4.log 2>&1"
tail -n2 gpurun_out/r04h_tests.log; grep -E "passed|failed|Error" gpurun_out/r04h_layerwise.log | tail -3
for f in c4_a c4_b c4_a2 c4_b2; do tail -n1 gpurun_out/r04h_$f.log | cut -c1-150; done
d=gpurun_out/prof_r04h_c4; python tools/step_breakdown.py $d/run_kernel_trace.csv > $d/step_breakdown.txt; python tools/stream_util.py $d/run_kernel_trace.csv > $d/stream_util.txt; head -25 $d/step_breakdown.txt
