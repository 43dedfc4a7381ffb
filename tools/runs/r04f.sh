# deferred fake-quant values (C5): int8 tests, C5 layerwise, int8 step parity, C5 A/B; C4 / C5 profiles
tools/gpu_steps.sh \
 "400 python -u -m pytest tests/test_int8_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04f_tests.log 2>&1" \
 "500 python -u -m pytest tests/test_step_bf16_gpu.py -k 'int8' -x -v -s --timeout 450 --timeout-method thread > gpurun_out/r04f_layerwise.log 2>&1" \
 "500 python -u -m pytest tests -m gpu -k 'int8 and not layerwise and not test_int8_gpu' -x -v --timeout 450 --timeout-method thread > gpurun_out/r04f_steps.log 2>&1" \
 "200 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04f_c5_a.log 2>&1" \
 "200 env RN_QUANT_DEFER=0 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04f_c5_b.log 2>&1" \
 "200 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04f_c5_a2.log 2>&1" \
 "200 env RN_QUANT_DEFER=0 python bench.py --model resnet50_int8 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04f_c5_b2.log 2>&1" \
 "300 bash tools/prof_bench.sh r04f_c5 --model resnet50_int8 --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04f_prof_c5.log 2>&1" \
 "300 bash tools/prof_bench.sh r04f_c4 --model resnext50 --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/r04f_prof_c4.log 2>&1"
tail -n2 gpurun_out/r04f_tests.log; grep -E "passed|failed|Error" gpurun_out/r04f_layerwise.log | tail -3
grep -E "passed|failed|Error" gpurun_out/r04f_steps.log | tail -3
for f in c5_a c5_b c5_a2 c5_b2; do tail -n1 gpurun_out/r04f_$f.log | cut -c1-150; done
for d in gpurun_out/prof_r04f_c5 gpurun_out/prof_r04f_c4; do python tools/step_breakdown.py $d/run_kernel_trace.csv > $d/step_breakdown.txt; python tools/stream_util.py $d/run_kernel_trace.csv > $d/stream_util.txt; head -25 $d/step_breakdown.txt; done
