# C5 profile with the int8-codes weight gradients + full-size C5 layerwise + int8 kernel tests
tools/gpu_steps.sh \
 "300 bash tools/prof_bench.sh c5cw --model resnet50_int8 --steps 5 --warmup 3 --no-cpu-baseline --pcie-steps 0" \
 "600 python -u -m pytest tests/test_step_bf16_gpu.py -x -q -k 'int8_full_size' --timeout 500 --timeout-method thread > gpurun_out/r04s_lw.log 2>&1" \
 "300 python -u -m pytest tests/test_int8_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04s_int8.log 2>&1"
tail -n2 gpurun_out/r04s_lw.log; tail -n2 gpurun_out/r04s_int8.log
